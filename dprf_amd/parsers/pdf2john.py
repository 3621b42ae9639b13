"""PDF verification-data extractor: Python-3 counterpart of /root/reference/src/pdf-impl/pdf2john.py
(PdfParser.parse :54-109, get_passwords_for_JtR :111-141, get_password_from_byte_string :238-277),
producing the stream the reference parser prints under PYTHON 2.

Output: ``<basename>:$pdf$*V*R*Length*P*meta*idlen*id*ulen*u*olen*o``.

The reference scrapes the file with regular expressions; the behaviours that decide the stream are kept:
  * trailer = the lines from the first one containing ``trailer`` up to the first containing ``>>``
    (joined without separators); without one, ``DecodeParms`` .. ``stream`` (cross-reference streams);
  * the ``/Encrypt N G R`` object is the text after ``\\rN G obj`` (or ``\\nN G obj``) up to ``endobj``;
  * V and R are the first ``/V d`` and ``/R d`` (one digit); Length is the largest ``/Length n``; P is the
    first ``/P -n``; meta is 0 only for ``/EncryptMetadata false``;
  * the ID is the first ``<hex>`` (else ``(word)``) in the trailer, lower-cased;
  * U and O: a literal ``(...)`` string is decoded byte by byte with ``\\`` escapes (``\\n \\r \\t \\b \\f
    \\( \\) \\\\`` and the map's oddities ``\\s \\e \\v \\a``), and it is extended past an escaped ``)``
    exactly where Python 2 compares the one-character string ``pas[-2]`` with a backslash -- Python 3
    compares an int there and truncates (the R2 test file's U comes out as 8 bytes);
    a hex ``<...>`` string is taken verbatim, lower-cased.
"""
import os
import re
import sys

# unescape map of the reference (:279-285): the entries Python 2 evaluates "\s", "\e", "\v", "\a" as
_UNESCAPE = {b"n": 0x0a, b"s": 0x5c, b"e": 0x5c, b"r": 0x0d, b"t": 0x09, b"v": 0x0b, b"f": 0x0c, b"b": 0x08,
             b"a": 0x07, b")": 0x29, b"(": 0x28, b"\\": 0x5c}


def _between(data, s1, s2):
    out = b""
    inside = False
    for line in re.split(b"\n|\r", data):
        inside = inside or line.find(s1) != -1
        if inside:
            out += line
            if line.find(s2) != -1:
                break
    return out


def _trailer(data):
    t = _between(data, b"trailer", b">>")
    if t == b"":
        t = _between(data, b"DecodeParms", b"stream")
        if t == b"":
            raise ValueError("Can't find trailer")
    if t.find(b"Encrypt") == -1:
        raise ValueError("File not encrypted")
    return t


def _object_id(name, trailer):
    m = re.findall(b"/" + name + rb"\s\d+\s\d\sR", trailer)[0]
    return re.findall(rb"\d+ \d", m)[0]


def _pdf_object(data, oid):
    out = oid + b" obj" + data.partition(b"\r" + oid + b" obj")[2]
    if out == oid + b" obj":
        out = oid + b" obj" + data.partition(b"\n" + oid + b" obj")[2]
    return out.partition(b"endobj")[0] + b"endobj"


def _encryption_dictionary(data, oid):
    d = _pdf_object(data, oid)
    for o in d.split(b"endobj"):
        if oid + b" obj" in o:
            d = o
    return d


def _literal(raw):
    """Bytes of a matched ``/U(...)`` or ``/U (...)`` literal, reference (:238-277) semantics: returns
    'count*hex' where count excludes the key, the parentheses and one byte per escape, and the hex drops
    the closing parenthesis."""
    excluded = {0, 1, 2}
    if raw[2] != 0x28:                 # "/U (" : skip the space too
        excluded.add(3)
    hexs = ""
    escape = False
    escapes = 0
    for i, b in enumerate(raw):
        if i in excluded:
            continue
        if escape:
            hexs += "%02x" % _UNESCAPE[bytes([b])]
            escape = False
        elif b == 0x5c:
            escape = True
            escapes += 1
        else:
            hexs += "%02x" % b
    count = len(raw) - (len(excluded) + 1) - escapes
    return "%d*%s" % (count, hexs[:-2])


def _passwords(encdict):
    out = ""
    for key in (b"U", b"O"):
        pat = b"/" + key + rb"\s*\([^)]+\)"
        found = re.findall(pat, encdict)
        if found:
            raw = found[0]
            while raw[-2:-1] == b"\\":     # Python 2: pas[-2] is a 1-character string (:125)
                pat += rb"[^)]+\)"
                raw = re.findall(pat, encdict)[0]
            out += _literal(raw) + "*"
        else:
            m = re.findall(key + rb"\s*<\w+>", encdict)[0]
            h = re.findall(rb"<\w+>", m)[0].replace(b"<", b"").replace(b">", b"")
            out += "%d*%s*" % (len(h) // 2, h.lower().decode("ascii"))
    return out[:-1]


def get_hash(filename):
    data = open(filename, "rb").read()
    if not re.findall(rb"PDF-\d\.\d", data):
        raise ValueError("%s is not a PDF file!" % filename)
    trailer = _trailer(data)
    encdict = _encryption_dictionary(data, _object_id(b"Encrypt", trailer))
    v = re.findall(rb"\d+", re.findall(rb"/V \d", encdict)[0])[0].decode()
    r = re.findall(rb"\d+", re.findall(rb"/R \d", encdict)[0])[0].decode()
    longest, length = 0, ""
    for le in re.findall(rb"/Length \d+", encdict):
        n = int(re.findall(rb"\d+", le)[0])
        if n > longest:
            longest, length = n, str(n)
    p = re.findall(rb"-\d+", re.findall(rb"/P -\d+", encdict)[0])[0].decode()
    em = re.findall(rb"/EncryptMetadata\s\w+", encdict)
    meta = "0" if em and re.findall(rb"\w+", em[0])[-1] == b"false" else "1"
    ids = re.findall(rb"<\w+>", trailer) or re.findall(rb"\(\w+\)", trailer)
    i_d = ids[0].replace(b"<", b"").replace(b">", b"").lower().decode("ascii")
    out = "$pdf$*%s*%s*%s*%s*%s*%d*%s*%s" % (v, r, length, p, meta, len(i_d) // 2, i_d, _passwords(encdict))
    return "%s:%s" % (os.path.basename(filename), out)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    for f in argv:
        sys.stdout.write(get_hash(f) + "\n")


if __name__ == "__main__":
    main()
