"""MS Office (OOXML in an OLE container) verification-data extractor: Python-3 counterpart of the
encrypted-OOXML path of /root/reference/src/ms-offcrypto-impl/office2john.py (process_new_office
:1728-1821), which the reference engine calls for document type 1 (brute_force.py:236).

Output, Standard Encryption (Office 2007, the only form the reference verifier handles):
    ``<basename>:$office$*2007*<verifierHashSize>*<keySize>*<saltSize>*<salt>*<encVerifier>*<encVerifierHash[0:32]>``
Agile Encryption (Office 2010/2013) is printed in the reference's form too
    ``<basename>:$office$*<2010|2013>*<spinCount>*<keyBits>*<saltSize>*<salt>*<encHashInput>*<encHashValue[0:32]>``
but libdprf.so rejects it (DPRF_E_DOMAIN): the reference verifier would misread those fields.

The OLE compound file (MS-CFB) is read by a small reader of our own: header, DIFAT/FAT chains,
directory, mini stream.
"""
import base64
import os
import struct
import sys
import xml.etree.ElementTree as et

_SIG = bytes.fromhex("d0cf11e0a1b11ae1")
_END, _FREE = 0xFFFFFFFE, 0xFFFFFFFF


class CompoundFile:
    def __init__(self, data):
        if data[:8] != _SIG:
            raise ValueError("not an OLE compound file")
        self.d = data
        self.ss = 1 << struct.unpack_from("<H", data, 0x1E)[0]
        self.mss = 1 << struct.unpack_from("<H", data, 0x20)[0]
        nfat, self.dir_start = struct.unpack_from("<II", data, 0x2C)
        self.cutoff, mfat_start, nmfat, difat_start, ndifat = struct.unpack_from("<IIIII", data, 0x38)
        difat = list(struct.unpack_from("<109I", data, 0x4C))
        s = difat_start
        for _ in range(ndifat):
            if s in (_END, _FREE):
                break
            vals = struct.unpack_from("<%dI" % (self.ss // 4), self._sector(s))
            difat += vals[:-1]
            s = vals[-1]
        fat = []
        for sec in difat[:nfat]:
            fat += struct.unpack_from("<%dI" % (self.ss // 4), self._sector(sec))
        self.fat = fat
        self.entries = self._directory()
        root = self.entries[0]
        self.mini_stream = self._chain_bytes(root["start"], root["size"], self.fat, self._sector)
        mfat_bytes = self._chain_bytes(mfat_start, nmfat * self.ss, self.fat, self._sector) if nmfat else b""
        self.mfat = list(struct.unpack_from("<%dI" % (len(mfat_bytes) // 4), mfat_bytes))

    def _sector(self, n):
        off = (n + 1) * self.ss
        return self.d[off:off + self.ss]

    def _mini_sector(self, n):
        return self.mini_stream[n * self.mss:(n + 1) * self.mss]

    def _chain_bytes(self, start, size, table, reader):
        out, s, seen = [], start, set()
        while s not in (_END, _FREE) and s < len(table) and s not in seen and len(out) * 1 < 1 << 24:
            seen.add(s)
            out.append(reader(s))
            s = table[s]
        return b"".join(out)[:size]

    def _directory(self):
        raw = self._chain_bytes(self.dir_start, 1 << 30, self.fat, self._sector)
        ents = []
        for off in range(0, len(raw) - 127, 128):
            nlen = struct.unpack_from("<H", raw, off + 0x40)[0]
            name = raw[off:off + max(0, nlen - 2)].decode("utf-16-le", errors="replace")
            typ = raw[off + 0x42]
            start = struct.unpack_from("<I", raw, off + 0x74)[0]
            size = struct.unpack_from("<Q", raw, off + 0x78)[0]
            if self.ss == 512:
                size &= 0xFFFFFFFF
            ents.append({"name": name, "type": typ, "start": start, "size": size})
        return ents

    def open_stream(self, name):
        for e in self.entries[1:]:
            if e["type"] == 2 and e["name"].lower() == name.lower():
                if e["size"] < self.cutoff:
                    return self._chain_bytes(e["start"], e["size"], self.mfat, self._mini_sector)
                return self._chain_bytes(e["start"], e["size"], self.fat, self._sector)
        raise KeyError(name)


def get_hash(filename):
    cf = CompoundFile(open(filename, "rb").read())
    s = cf.open_stream("EncryptionInfo")
    major, minor, flags = struct.unpack_from("<HHI", s, 0)
    if flags == 16:
        raise ValueError("%s : An external cryptographic provider is not supported!" % filename)
    base = os.path.basename(filename)
    if major == 4 and minor == 4:                    # Agile (Office 2010/2013), XML descriptor
        if flags != 0x40:
            raise ValueError("%s : The encryption flags are not consistent with the encryption type" % filename)
        root = et.fromstring(s[8:])
        for node in root.iter("{http://schemas.microsoft.com/office/2006/keyEncryptor/password}encryptedKey"):
            a = node.attrib
            version = {"SHA1": 2010, "SHA512": 2013}.get(a.get("hashAlgorithm"))
            if version is None:
                raise ValueError("%s uses un-supported hashing algorithm %s" % (filename, a.get("hashAlgorithm")))
            hv = base64.b64decode(a["encryptedVerifierHashValue"]).hex()
            return "%s:$office$*%d*%d*%d*%d*%s*%s*%s" % (
                base, version, int(a["spinCount"]), int(a["keyBits"]), int(a["saltSize"]),
                base64.b64decode(a["saltValue"]).hex(), base64.b64decode(a["encryptedVerifierHashInput"]).hex(),
                hv[0:64])
        raise ValueError("%s : no password key encryptor" % filename)
    # Standard Encryption (Office 2007): EncryptionHeader then EncryptionVerifier (MS-OFFCRYPTO 2.3.4.5)
    header_len = struct.unpack_from("<I", s, 8)[0]
    key_size = struct.unpack_from("<I", s, 12 + 16)[0]        # flags, sizeExtra, algId, algHashId, keySize
    off = 12 + header_len
    salt_size = struct.unpack_from("<I", s, off)[0]
    if salt_size != 16:
        raise ValueError("%s : salt size %d (expected 16)" % (filename, salt_size))
    salt = s[off + 4:off + 20]
    ev = s[off + 20:off + 36]
    vh_size = struct.unpack_from("<I", s, off + 36)[0]
    evh = s[off + 40:off + 72]
    return "%s:$office$*%d*%d*%d*%d*%s*%s*%s" % (base, 2007, vh_size, key_size, salt_size, salt.hex(), ev.hex(),
                                                 evh.hex()[0:64])


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    for f in argv:
        sys.stdout.write(get_hash(f) + "\n")


if __name__ == "__main__":
    main()
