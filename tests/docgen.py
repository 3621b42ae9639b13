"""Self-generated encrypted test documents (TEST INFRASTRUCTURE: used by tests/golden/make_docs.py and the
tests, never by dprf_amd/).

The reference ships four documents (test/files) and no way to make more.  These writers produce real
files of the three formats, built from the published specifications, so that the parsers, the oracle, the
reference verifiers and the GPU engine can all be run on the same documents with known passwords:

* ``write_docx``  MS-CFB (OLE2, v3, 512-byte sectors) with the ``EncryptionInfo`` (MS-OFFCRYPTO 2.3.4.5,
  Standard Encryption, AES-128 + SHA-1, version 3.2) and ``EncryptedPackage`` streams (2.3.4.4); key
  derivation 2.3.4.7 (50,000 SHA-1 iterations), password verifier 2.3.4.8.  The stream the reference's
  office2john.py reads: ``process_new_office`` :1728-1821.
* ``write_odt``   ODF 1.2 package: zip with ``META-INF/manifest.xml`` (encryption-data: sha256-1k checksum,
  AES-256-CBC, SHA-256 start key, PBKDF2-HMAC-SHA1 1024 iterations, 32-byte key) and encrypted, deflated
  entries, including the empty ``Configurations2/accelerator/current.xml`` that odt2hashes -e picks.
* ``write_pdf``   a one-page PDF with a Standard security handler ``/Encrypt`` dictionary: revisions 2, 3,
  4 (ISO 32000-1 7.6.3.3-4, algorithms 2-5, RC4) and 5, 6 (ISO 32000-2 7.6.4.3.3-4, SHA-256 / the hardened
  hash); ``/O`` ``/U`` and ``/ID`` are hex strings.  R5/R6 documents carry ``/U`` and ``/O`` only (no
  ``/UE /OE /Perms``): they verify user passwords, they are not meant to be opened by a viewer.

Hashes come from hashlib; AES and RC4 from the oracle's C primitives (pinned by FIPS 197 / RFC 6229 KATs in
tests/test_oracle_kat.py); every generated document is then accepted only if the REFERENCE verifier
(oracle/_ref, compiled from /root/reference) returns 1 for its password (tests/golden/make_docs.py).
Random fields never start with a 0x00 byte (the reference's hex decoder drops leading zero bytes:
SURVEY.md Appendix B.1).
"""
import base64
import hashlib
import io
import os
import random
import struct
import sys
import zipfile
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import pyoracle as O  # noqa: E402

PDF_PAD = bytes.fromhex("28bf4e5e4e758a4164004e56fffa01082e2e00b6d0683e802f0ca9fe6453697a")


def _rand(rng, n):
    """n random bytes whose first byte is not 0x00."""
    b = bytes(rng.getrandbits(8) for _ in range(n))
    return bytes([b[0] or 1]) + b[1:]


def _aes_ecb(key, data):
    return b"".join(O.aes_encrypt_block(key, data[i:i + 16]) for i in range(0, len(data), 16))


def _aes_cbc(key, iv, data):
    out, prev = [], iv
    for i in range(0, len(data), 16):
        prev = O.aes_encrypt_block(key, bytes(a ^ b for a, b in zip(data[i:i + 16], prev)))
        out.append(prev)
    return b"".join(out)


# ============================================================================ MS Office 2007 (.docx)
def office_key(password, salt):
    """MS-OFFCRYPTO 2.3.4.7 for AES-128 / SHA-1: the 16-byte key (what msoffcrypto...c:91-153 derives)."""
    h = hashlib.sha1(salt + password.encode("utf-16-le")).digest()
    for i in range(50000):
        h = hashlib.sha1(struct.pack("<I", i) + h).digest()
    h = hashlib.sha1(h + struct.pack("<I", 0)).digest()
    buf = bytearray(b"\x36" * 64)
    for i in range(20):
        buf[i] ^= h[i]
    return hashlib.sha1(bytes(buf)).digest()[:16]


def _encryption_info(salt, ev, evh):
    csp = "Microsoft Enhanced RSA and AES Cryptographic Provider\0".encode("utf-16-le")
    header = struct.pack("<IIIIIIII", 0x24, 0, 0x660E, 0x8004, 128, 0x18, 0, 0) + csp
    verifier = struct.pack("<I", 16) + salt + ev + struct.pack("<I", 20) + evh
    return struct.pack("<HHII", 3, 2, 0x24, len(header)) + header + verifier


def _cfb(streams):
    """A version-3 compound file holding the given {name: bytes} streams under the root storage.
    Streams < 4096 bytes go into the mini stream (MS-CFB 2.6.3)."""
    SS, MSS, CUT = 512, 64, 4096
    ENDC, FREE, FATS, NOS = 0xFFFFFFFE, 0xFFFFFFFF, 0xFFFFFFFD, 0xFFFFFFFF
    names = sorted(streams, key=lambda n: (len(n), n.upper()))
    mini, mfat, starts = b"", [], {}
    for n in names:
        d = streams[n]
        if len(d) < CUT:
            k = max(1, -(-len(d) // MSS))
            first = len(mfat)
            mfat += [first + i + 1 for i in range(k - 1)] + [ENDC]
            starts[n] = first
            mini += d + b"\0" * (k * MSS - len(d))
    # sectors: 0 FAT, 1 directory, 2 MiniFAT, then the mini stream container, then the big streams
    fat = [FATS, ENDC, ENDC]
    sectors = []
    root_start = ENDC
    if mini:
        k = -(-len(mini) // SS)
        root_start = len(fat)
        fat += [root_start + i + 1 for i in range(k - 1)] + [ENDC]
        sectors.append(mini + b"\0" * (k * SS - len(mini)))
    for n in names:
        d = streams[n]
        if len(d) >= CUT:
            k = -(-len(d) // SS)
            starts[n] = len(fat)
            fat += [starts[n] + i + 1 for i in range(k - 1)] + [ENDC]
            sectors.append(d + b"\0" * (k * SS - len(d)))
    assert len(fat) <= SS // 4, "one FAT sector only"
    fat += [FREE] * (SS // 4 - len(fat))
    mfat += [FREE] * (SS // 4 - len(mfat))

    def dirent(name, typ, child, left, right, start, size, color=1):
        nb = (name + "\0").encode("utf-16-le") if name else b""
        return (nb + b"\0" * (64 - len(nb)) + struct.pack("<HBB", len(nb), typ, color) +
                struct.pack("<III", left, right, child) + b"\0" * 16 + struct.pack("<I", 0) + b"\0" * 16 +
                struct.pack("<IQ", start, size))

    # siblings in (length, upper-case) order (MS-CFB 2.6.4): a black node with one red right child
    assert len(names) <= 2
    ents = [dirent("Root Entry", 5, 1, NOS, NOS, root_start, len(mini))]
    for i, n in enumerate(names):
        right = i + 2 if i + 1 < len(names) else NOS
        ents.append(dirent(n, 2, NOS, NOS, right, starts[n], len(streams[n]), color=1 if i == 0 else 0))
    ents += [b"\0" * 64 + struct.pack("<HBB", 0, 0, 0) + struct.pack("<III", NOS, NOS, NOS) + b"\0" * 48] * (4 - len(ents))
    assert len(ents) == 4
    header = (bytes.fromhex("d0cf11e0a1b11ae1") + b"\0" * 16 + struct.pack("<HHHHH", 0x3E, 3, 0xFFFE, 9, 6) +
              b"\0" * 6 + struct.pack("<IIIIIIIIII", 0, 1, 1, 0, CUT, 2, 1, ENDC, 0, 0) +
              struct.pack("<108I", *([FREE] * 108)))
    assert len(header) == SS
    body = struct.pack("<128I", *fat) + b"".join(ents) + struct.pack("<128I", *mfat) + b"".join(sectors)
    return header + body


def write_docx(path, password, seed):
    """Office 2007 Standard Encryption document; returns the key (for tests)."""
    rng = random.Random(seed)
    salt = _rand(rng, 16)
    key = office_key(password, salt)
    while True:
        verifier = bytes(rng.getrandbits(8) for _ in range(16))
        ev = _aes_ecb(key, verifier)
        evh = _aes_ecb(key, hashlib.sha1(verifier).digest() + b"\0" * 12)
        if ev[0] and evh[0]:
            break
    buf = io.BytesIO()
    with zipfile.ZipFile(buf, "w", zipfile.ZIP_DEFLATED) as z:
        z.writestr(zipfile.ZipInfo("[Content_Types].xml"), '<?xml version="1.0"?><Types xmlns="http://schemas.'
                   'openxmlformats.org/package/2006/content-types"/>', zipfile.ZIP_DEFLATED)
        z.writestr(zipfile.ZipInfo("word/document.xml"), "<w:document>%s</w:document>" % (" ".join(
            "%08x" % rng.getrandbits(32) for _ in range(600))), zipfile.ZIP_DEFLATED)
    plain = buf.getvalue()
    package = struct.pack("<Q", len(plain)) + _aes_ecb(key, plain + b"\0" * (-len(plain) % 16))
    with open(path, "wb") as f:
        f.write(_cfb({"EncryptionInfo": _encryption_info(salt, ev, evh), "EncryptedPackage": package}))
    return key


# ============================================================================ ODF 1.2 (.odt)
MANIFEST_NS = "urn:oasis:names:tc:opendocument:xmlns:manifest:1.0"


def odt_key(password, salt):
    """SHA-256 start key, then PBKDF2-HMAC-SHA1(1024, 32 bytes) (odt_password_verifier.c:78-85)."""
    return hashlib.pbkdf2_hmac("sha1", hashlib.sha256(password.encode()).digest(), salt, 1024, 32)


def _odt_entry(rng, password, data):
    """(encrypted bytes, manifest encryption-data xml) for one package entry."""
    salt, iv = _rand(rng, 16), _rand(rng, 16)
    key = odt_key(password, salt)
    comp = zlib.compressobj(9, zlib.DEFLATED, -15)
    deflated = comp.compress(data) + comp.flush()
    checksum = hashlib.sha256(deflated[:1024]).digest()
    pad = 16 - len(deflated) % 16                      # W3C xmlenc padding: random bytes, then the count
    plain = deflated + bytes(rng.getrandbits(8) for _ in range(pad - 1)) + bytes([pad])
    enc = _aes_cbc(key, iv, plain)
    b64 = lambda b: base64.b64encode(b).decode()
    xml = ('<manifest:encryption-data manifest:checksum-type="urn:oasis:names:tc:opendocument:xmlns:manifest:1.0'
           '#sha256-1k" manifest:checksum="%s"><manifest:algorithm manifest:algorithm-name="http://www.w3.org/2001/'
           '04/xmlenc#aes256-cbc" manifest:initialisation-vector="%s"/><manifest:start-key-generation '
           'manifest:start-key-generation-name="http://www.w3.org/2000/09/xmldsig#sha256" manifest:key-size="32"/>'
           '<manifest:key-derivation manifest:key-derivation-name="PBKDF2" manifest:key-size="32" '
           'manifest:iteration-count="1024" manifest:salt="%s"/></manifest:encryption-data>' % (b64(checksum), b64(iv),
                                                                                                 b64(salt)))
    return enc, xml, key, salt, iv


def write_odt(path, password, seed):
    rng = random.Random(seed)
    words = ["%06x" % rng.getrandbits(24) for _ in range(900)]
    files = [
        ("content.xml", ('<?xml version="1.0" encoding="UTF-8"?><office:document-content><office:body><office:text>'
                         '<text:p>%s</text:p></office:text></office:body></office:document-content>'
                         % " ".join(words)).encode()),
        ("styles.xml", ('<?xml version="1.0" encoding="UTF-8"?><office:document-styles>%s</office:document-styles>'
                        % " ".join(words[:700])).encode()),
        ("Configurations2/accelerator/current.xml", b""),
    ]
    entries = []
    for name, data in files:
        while True:
            enc, xml, _, salt, iv = _odt_entry(rng, password, data)
            if enc[0]:
                break
        entries.append((name, data, enc, xml))
    manifest = ['<?xml version="1.0" encoding="UTF-8"?>',
                '<manifest:manifest xmlns:manifest="%s" manifest:version="1.2">' % MANIFEST_NS,
                ' <manifest:file-entry manifest:full-path="/" manifest:version="1.2" '
                'manifest:media-type="application/vnd.oasis.opendocument.text"/>']
    for name, data, enc, xml in entries:
        manifest.append(' <manifest:file-entry manifest:full-path="%s" manifest:media-type="text/xml" '
                        'manifest:size="%d">%s</manifest:file-entry>' % (name, len(data), xml))
    manifest.append('</manifest:manifest>')
    with zipfile.ZipFile(path, "w") as z:
        z.writestr(zipfile.ZipInfo("mimetype"), "application/vnd.oasis.opendocument.text", zipfile.ZIP_STORED)
        for name, data, enc, xml in entries:
            z.writestr(zipfile.ZipInfo(name), enc, zipfile.ZIP_STORED)   # already deflated, then encrypted
        z.writestr(zipfile.ZipInfo("META-INF/manifest.xml"), "\n".join(manifest), zipfile.ZIP_DEFLATED)


# ============================================================================ PDF (.pdf)
def _pdf_key(pw, O_, P, ID, R, n, meta):
    """Algorithm 2 (ISO 32000-1 7.6.3.3)."""
    h = hashlib.md5((pw.encode()[:32] + PDF_PAD)[:32] + O_ + struct.pack("<i", P) + ID +
                    (b"\xff\xff\xff\xff" if R >= 4 and not meta else b"")).digest()
    if R >= 3:
        for _ in range(50):
            h = hashlib.md5(h[:n]).digest()
    return h[:n]


def _pdf_owner(owner, user, R, n):
    """Algorithm 3: the /O value."""
    h = hashlib.md5((owner.encode()[:32] + PDF_PAD)[:32]).digest()
    if R >= 3:
        for _ in range(50):
            h = hashlib.md5(h).digest()
    key = h[:n]
    c = O.rc4(key, (user.encode()[:32] + PDF_PAD)[:32])
    if R >= 3:
        for i in range(1, 20):
            c = O.rc4(bytes(k ^ i for k in key), c)
    return c


def pdf_r6_hash(pw, salt, udata=b""):
    """ISO 32000-2 Algorithm 2.B (the hardened hash), as pdf_password_verifier.c:226-291 computes it."""
    k = hashlib.sha256(pw + salt + udata).digest()
    i = 0
    while True:
        k1 = (pw + k + udata) * 64
        e = _aes_cbc(k[:16], k[16:32], k1)
        m = sum(e[:16]) % 3
        k = (hashlib.sha256, hashlib.sha384, hashlib.sha512)[m](e).digest()
        i += 1
        if i >= 64 and e[-1] <= i - 32:
            return k[:32]


def write_pdf(path, password, seed, R=3, length=128, P=-1028, meta=True, owner="owner"):
    rng = random.Random(seed)
    V = {2: 1, 3: 2, 4: 4, 5: 5, 6: 5}[R]
    while True:
        ID = _rand(rng, 16)
        if R <= 4:
            n = 5 if R == 2 else length // 8
            O_ = _pdf_owner(owner, password, R, n)
            key = _pdf_key(password, O_, P, ID, R, n, meta)
            if R == 2:
                U = O.rc4(key, PDF_PAD)
            else:
                c = O.rc4(key, hashlib.md5(PDF_PAD + ID).digest())
                for i in range(1, 20):
                    c = O.rc4(bytes(k ^ i for k in key), c)
                U = c + _rand(rng, 16)
        else:
            vs, ks = _rand(rng, 8), _rand(rng, 8)
            pw = password.encode()
            h = hashlib.sha256(pw[:127] + vs).digest() if R == 5 else pdf_r6_hash(pw, vs)
            U = h + vs + ks
            ovs, oks = _rand(rng, 8), _rand(rng, 8)
            ow = owner.encode()
            oh = hashlib.sha256(ow[:127] + ovs + U).digest() if R == 5 else pdf_r6_hash(ow, ovs, U)
            O_ = oh + ovs + oks
            length = 256
        if U[0] and O_[0]:
            break
    objs = [
        b"<< /Type /Catalog /Pages 2 0 R >>",
        b"<< /Type /Pages /Kids [3 0 R] /Count 1 >>",
        b"<< /Type /Page /Parent 2 0 R /MediaBox [0 0 612 792] >>",
        (b"<< /Filter /Standard /V %d /R %d /Length %d /P %d /O <%s> /U <%s>%s >>"
         % (V, R, length, P, O_.hex().encode(), U.hex().encode(),
            b" /EncryptMetadata false" if not meta else b"")),
    ]
    out = io.BytesIO()
    out.write(b"%PDF-" + (b"1.7" if R <= 4 else b"2.0") + b"\n%\xe2\xe3\xcf\xd3\n")
    offs = []
    for i, o in enumerate(objs):
        offs.append(out.tell())
        out.write(b"%d 0 obj\n%s\nendobj\n" % (i + 1, o))
    xref = out.tell()
    out.write(b"xref\n0 %d\n0000000000 65535 f \n" % (len(objs) + 1))
    for o in offs:
        out.write(b"%010d 00000 n \n" % o)
    out.write(b"trailer\n<< /Size %d /Root 1 0 R /Encrypt 4 0 R /ID [<%s> <%s>] >>\nstartxref\n%d\n%%%%EOF\n"
              % (len(objs) + 1, ID.hex().encode(), ID.hex().encode(), xref))
    with open(path, "wb") as f:
        f.write(out.getvalue())
