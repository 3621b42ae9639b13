"""ODF 1.2 verification-data extractor: Python-3 counterpart of
/root/reference/src/odt-impl/odt2hashes.py (get_hashes :53-86, template :43).

Output: ``<basename>:$odt$*<version>*<checksum hex>*<iv hex>*<salt hex>*<encrypted hex>*<len>``.
The encryption data of the SMALLEST file-entry whose manifest size exceeds 1024 (or -1 with
``-e``/experimental) is used, ties resolved in manifest order (:66-72).
"""
import argparse
import base64
import os
import sys
import xml.etree.ElementTree as et
import zipfile

NS = "{urn:oasis:names:tc:opendocument:xmlns:manifest:1.0}"
TEMPLATE = "{0}:$odt$*{1}*{2}*{3}*{4}*{5}*{6}"


def get_hashes(filename, experimental=False):
    with zipfile.ZipFile(filename, "r") as z:
        root = et.fromstring(z.read("META-INF/manifest.xml"))
        version = root.get(NS + "version")
        size_limit = -1 if experimental else 1024
        best, best_size = None, None
        for fe in root.iter(NS + "file-entry"):
            size = fe.get(NS + "size")
            if size is not None and int(size) > size_limit and (best is None or int(size) < best_size):
                best, best_size = fe, int(size)
        if best is None:
            raise ValueError("%s: no encrypted file-entry above the size limit" % filename)
        enc = best.find(NS + "encryption-data")
        checksum = base64.b64decode(enc.get(NS + "checksum"))
        iv = base64.b64decode(enc.find(NS + "algorithm").get(NS + "initialisation-vector"))
        salt = base64.b64decode(enc.find(NS + "key-derivation").get(NS + "salt"))
        data = z.read(best.get(NS + "full-path"))
    return TEMPLATE.format(os.path.basename(filename), version, checksum.hex(), iv.hex(), salt.hex(),
                           data.hex(), len(data))


def main(argv=None):
    p = argparse.ArgumentParser(prog="odt2hashes")
    p.add_argument("-v", "--verbose", default=False, action="store_true")
    p.add_argument("-e", "--experimental", default=False, action="store_true")
    p.add_argument("filename")
    a = p.parse_args(argv)
    sys.stdout.write(get_hashes(a.filename, a.experimental) + "\n")


if __name__ == "__main__":
    main()
