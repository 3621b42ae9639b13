"""ctypes binding of the CPU restatement (oracle/oracle.c).  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module; the product
package (dprf_amd/) never does.  See oracle/oracle.h for the reference lines each function restates.
"""
import ctypes
import os
import re
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

NCOUNT = 10
COUNT_NAMES = ["sha1c", "sha256c", "sha512c", "md5c", "aes128_enc_blocks", "aes256_dec_blocks",
               "rc4_ksa", "rc4_prga_bytes", "aes128_key_exp", "aes256_key_exp"]
FLAG_NEVER_MATCHES = 1
FLAG_REF_NONDETERMINISTIC = 2


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        for name, n in (("orc_sha1", 20), ("orc_sha256", 32), ("orc_sha384", 48), ("orc_sha512", 64),
                        ("orc_md5", 16)):
            f = getattr(L, name)
            f.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
            f.restype = None
        L.orc_aes_encrypt_block.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p]
        L.orc_aes_decrypt_block.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p]
        L.orc_rc4.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
        L.orc_pbkdf2_hmac_sha1.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                           ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t]
        L.orc_bn_hex_decode.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]
        L.orc_bn_hex_decode.restype = ctypes.c_int
        L.orc_ctx_create.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
        L.orc_ctx_create.restype = ctypes.c_int
        L.orc_ctx_destroy.argtypes = [ctypes.c_void_p]
        L.orc_ctx_flags.argtypes = [ctypes.c_void_p]
        L.orc_ctx_format.argtypes = [ctypes.c_void_p]
        L.orc_verify.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int]
        L.orc_verify.restype = ctypes.c_int
        L.orc_search_range.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_uint64), ctypes.c_int64]
        L.orc_search_range.restype = ctypes.c_int64
        L.orc_verify_list.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64),
                                      ctypes.c_int64, ctypes.c_int, ctypes.POINTER(ctypes.c_int8)]
        L.orc_intermediates.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        L.orc_work_counts.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]
        _ = u8p
        _lib = L
    return _lib


def _digest(name, n, data):
    out = ctypes.create_string_buffer(n)
    getattr(lib(), name)(bytes(data), len(data), out)
    return out.raw


def sha1(d): return _digest("orc_sha1", 20, d)
def sha256(d): return _digest("orc_sha256", 32, d)
def sha384(d): return _digest("orc_sha384", 48, d)
def sha512(d): return _digest("orc_sha512", 64, d)
def md5(d): return _digest("orc_md5", 16, d)


def aes_encrypt_block(key, block):
    out = ctypes.create_string_buffer(16)
    lib().orc_aes_encrypt_block(bytes(key), len(key) * 8, bytes(block), out)
    return out.raw


def aes_decrypt_block(key, block):
    out = ctypes.create_string_buffer(16)
    lib().orc_aes_decrypt_block(bytes(key), len(key) * 8, bytes(block), out)
    return out.raw


def rc4(key, data):
    out = ctypes.create_string_buffer(len(data))
    lib().orc_rc4(bytes(key), len(key), bytes(data), len(data), out)
    return out.raw


def pbkdf2_hmac_sha1(pw, salt, iters, n):
    out = ctypes.create_string_buffer(n)
    lib().orc_pbkdf2_hmac_sha1(bytes(pw), len(pw), bytes(salt), len(salt), iters, out, n)
    return out.raw


def bn_hex_decode(hexstr, cap=512):
    out = ctypes.create_string_buffer(cap)
    n = lib().orc_bn_hex_decode(hexstr.encode(), out, cap)
    return out.raw[:n]


def split_stream(stream):
    """parse_verification_data (brute_force.py:245-264) minus the print/exit."""
    fields = re.split(r"(?:\*)", stream)
    m = re.search(r".*:\$(\w+)\$", fields[0])
    if not m:
        raise ValueError("unsupported stream")
    fields[0] = m.groups()[0]
    return fields


class Ctx:
    def __init__(self, stream_or_fields):
        fields = split_stream(stream_or_fields) if isinstance(stream_or_fields, str) else list(stream_or_fields)
        arr = (ctypes.c_char_p * len(fields))(*[f.encode() for f in fields])
        h = ctypes.c_void_p()
        rc = lib().orc_ctx_create(arr, len(fields), ctypes.byref(h))
        if rc != 0:
            raise ValueError("oracle: stream outside the parity domain: %r" % (fields[:3],))
        self.h = h
        self.fields = fields

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_ctx_destroy(self.h)
            self.h = None

    @property
    def flags(self):
        return lib().orc_ctx_flags(self.h)

    def verify(self, pw):
        pw = pw.encode() if isinstance(pw, str) else bytes(pw)
        return lib().orc_verify(self.h, pw, len(pw))

    def intermediates(self, pw):
        pw = pw.encode() if isinstance(pw, str) else bytes(pw)
        out = ctypes.create_string_buffer(128)
        n = lib().orc_intermediates(self.h, pw, len(pw), out, 128)
        return out.raw[:n] if n > 0 else b""

    def work_counts(self, pw):
        pw = pw.encode() if isinstance(pw, str) else bytes(pw)
        arr = (ctypes.c_uint64 * NCOUNT)()
        lib().orc_work_counts(self.h, pw, len(pw), arr)
        return dict(zip(COUNT_NAMES, list(arr)))

    def search_range(self, charset, pwlen, start, count, nthreads=None, cap=1 << 16):
        cs = charset.encode() if isinstance(charset, str) else bytes(charset)
        nthreads = nthreads or min(8, os.cpu_count() or 1)
        hits = (ctypes.c_uint64 * cap)()
        n = lib().orc_search_range(self.h, cs, len(cs), pwlen, start, count, nthreads, hits, cap)
        if n < 0:
            raise ValueError("oracle search_range error %d" % n)
        return sorted(list(hits[:min(n, cap)])), n

    def verify_list(self, passwords, nthreads=None):
        bs = [p.encode() if isinstance(p, str) else bytes(p) for p in passwords]
        blob = b"".join(bs)
        offs = [0]
        for b in bs:
            offs.append(offs[-1] + len(b))
        o = (ctypes.c_uint64 * len(offs))(*offs)
        v = (ctypes.c_int8 * max(1, len(bs)))()
        lib().orc_verify_list(self.h, blob, o, len(bs), nthreads or min(8, os.cpu_count() or 1), v)
        return list(v[:len(bs)])


def index_to_password(idx, charset, pwlen):
    out = []
    for _ in range(pwlen):
        out.append(charset[idx % len(charset)])
        idx //= len(charset)
    return "".join(reversed(out))
