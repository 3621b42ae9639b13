"""ctypes binding of libdprf.so (include/dprf.h) -- the only way Python reaches the verification kernels.

There is no CPU fallback: if the library is missing, ``lib()`` raises; if no gfx950 device is visible,
context creation raises :class:`DprfError` (DPRF_E_NODEVICE).
"""
import ctypes
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DPRF_LIB") or os.path.join(HERE, "libdprf.so")   # DPRF_LIB: A/B builds only

ABI_VERSION = 7
ALL_DEVICES = -1
FMT_OFFICE, FMT_ODT, FMT_PDF = 1, 2, 3
E_INVALID, E_DOMAIN, E_HIP, E_NODEVICE, E_PWLEN, E_CHARSET = -1, -2, -3, -4, -5, -6
FLAG_NEVER_MATCHES, FLAG_REF_NONDETERMINISTIC = 1, 2
MAX_PW, MAX_PW_RANGE, MAX_PW_R6 = 131071, 32, 176

EXPORTS = ["dprf_abi_version", "dprf_last_error", "dprf_device_count", "dprf_device_list", "dprf_ctx_create",
           "dprf_ctx_create_devices", "dprf_ctx_destroy", "dprf_ctx_format", "dprf_ctx_flags", "dprf_ctx_kernel",
           "dprf_ctx_devices", "dprf_search_range", "dprf_verify_list", "dprf_list_status", "dprf_build_id",
           "dprf_plan_chunk", "dprf_ctx_last_call_devices", "dprf_search_symbols"]


class DprfError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("dprf error %d: %s" % (code, msg))
        self.code = code


class Stats(ctypes.Structure):
    _fields_ = [("candidates", ctypes.c_uint64), ("launches", ctypes.c_uint64), ("kernel_ms", ctypes.c_double),
                ("wall_ms", ctypes.c_double), ("stopped_early", ctypes.c_uint32), ("devices", ctypes.c_uint32),
                ("main_kernel_ms", ctypes.c_double), ("hit_ms", ctypes.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class DeviceStats(ctypes.Structure):
    """dprf_device_stats (ABI 4; `evaluated` ABI 6): one device's share of the last call on a context."""
    _fields_ = [("device", ctypes.c_int32), ("launches", ctypes.c_uint32), ("candidates", ctypes.c_uint64),
                ("kernel_ms", ctypes.c_double), ("first_ms", ctypes.c_double), ("finish_ms", ctypes.c_double),
                ("evaluated", ctypes.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_lib = None
_lock = threading.Lock()


def lib():
    """Load libdprf.so (in-tree).  Raises if it has not been built: never falls back to a CPU path."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError("libdprf.so not found at %s: build it with `python -c 'import __graft_entry__ as g; "
                                  "g.build()'` (make -C dprf_amd/csrc)" % LIB_PATH)
            L = ctypes.CDLL(LIB_PATH)
            L.dprf_abi_version.restype = ctypes.c_int
            L.dprf_last_error.restype = ctypes.c_char_p
            L.dprf_device_count.restype = ctypes.c_int
            L.dprf_ctx_create.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.c_int, ctypes.c_int,
                                          ctypes.POINTER(ctypes.c_void_p)]
            L.dprf_ctx_create.restype = ctypes.c_int
            L.dprf_ctx_create_devices.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.c_int,
                                                  ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                                  ctypes.POINTER(ctypes.c_void_p)]
            L.dprf_ctx_create_devices.restype = ctypes.c_int
            L.dprf_ctx_devices.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.c_int]
            L.dprf_device_list.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int]
            L.dprf_list_status.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64),
                                           ctypes.c_int64, ctypes.POINTER(ctypes.c_int8)]
            L.dprf_list_status.restype = ctypes.c_int
            L.dprf_ctx_destroy.argtypes = [ctypes.c_void_p]
            L.dprf_ctx_format.argtypes = [ctypes.c_void_p]
            L.dprf_ctx_flags.argtypes = [ctypes.c_void_p]
            L.dprf_ctx_kernel.argtypes = [ctypes.c_void_p]
            L.dprf_ctx_kernel.restype = ctypes.c_char_p
            L.dprf_search_range.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
                                            ctypes.POINTER(ctypes.c_uint64), ctypes.c_int64,
                                            ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(Stats)]
            L.dprf_search_range.restype = ctypes.c_int
            L.dprf_search_symbols.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint32),
                                              ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
                                              ctypes.POINTER(ctypes.c_uint64), ctypes.c_int64,
                                              ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(Stats)]
            L.dprf_search_symbols.restype = ctypes.c_int
            L.dprf_verify_list.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64),
                                           ctypes.c_int64, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64),
                                           ctypes.c_int64, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(Stats)]
            L.dprf_verify_list.restype = ctypes.c_int
            L.dprf_build_id.restype = ctypes.c_char_p
            L.dprf_plan_chunk.argtypes = [ctypes.c_char_p, ctypes.c_double, ctypes.c_uint64, ctypes.c_uint64,
                                          ctypes.c_int, ctypes.c_int]
            L.dprf_plan_chunk.restype = ctypes.c_uint64
            L.dprf_ctx_last_call_devices.argtypes = [ctypes.c_void_p, ctypes.POINTER(DeviceStats), ctypes.c_int]
            L.dprf_ctx_last_call_devices.restype = ctypes.c_int
            if L.dprf_abi_version() != ABI_VERSION:
                raise ImportError("libdprf.so ABI %d != %d" % (L.dprf_abi_version(), ABI_VERSION))
            _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        raise DprfError(rc, lib().dprf_last_error().decode(errors="replace"))


def device_count():
    return lib().dprf_device_count()


def build_id():
    """Fingerprint of the sources / flags / compiler libdprf.so was built from (dprf_build_id)."""
    return lib().dprf_build_id().decode()


def plan_chunk(kernel, rate_per_ms, remaining, total, ndev, inflight=0):
    """The library's multi-device chunk policy (dprf_plan_chunk): a pure function, no device work.  0 = take
    nothing now (scarce work and a launch still in flight), or an unknown kernel family."""
    return int(lib().dprf_plan_chunk(kernel.encode(), float(rate_per_ms), int(remaining), int(total), int(ndev),
                                     int(inflight)))


def device_list():
    """HIP ordinals of the visible gfx950 devices (not simply range(device_count()): a non-gfx950 device
    may sit at any ordinal)."""
    arr = (ctypes.c_int * 64)()
    n = lib().dprf_device_list(arr, 64)
    return list(arr[:min(n, 64)])


def _to_bytes(p):
    return p.encode("utf-8") if isinstance(p, str) else bytes(p)


class Context:
    """One document on one or more GPUs: the compiled form of the verifier argv brute_force.py builds per
    candidate (brute_force.py:163-197).  ``devices``: a list of HIP ordinals (the library runs one worker
    thread and one stream per entry and splits every call over them); ``device``: one ordinal, or
    ALL_DEVICES for every gfx950 device."""

    def __init__(self, fields, device=0, devices=None):
        fields = list(fields)
        arr = (ctypes.c_char_p * len(fields))(*[_to_bytes(f) for f in fields])
        h = ctypes.c_void_p()
        if devices is not None:
            devs = [int(d) for d in devices]
            darr = (ctypes.c_int * max(1, len(devs)))(*devs)
            _check(lib().dprf_ctx_create_devices(arr, len(fields), darr, len(devs), ctypes.byref(h)))
        else:
            _check(lib().dprf_ctx_create(arr, len(fields), int(device), ctypes.byref(h)))
        self._h = h
        self.fields = fields
        out = (ctypes.c_int * 64)()
        n = lib().dprf_ctx_devices(h, out, 64)
        self.devices = list(out[:min(n, 64)])
        self.device = self.devices[0]

    def close(self):
        if getattr(self, "_h", None):
            lib().dprf_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def format(self):
        return lib().dprf_ctx_format(self._h)

    @property
    def flags(self):
        return lib().dprf_ctx_flags(self._h)

    @property
    def kernel(self):
        return lib().dprf_ctx_kernel(self._h).decode()

    def last_call_devices(self):
        """Per-device records of the last search/verify call (list of dicts, one per device)."""
        arr = (DeviceStats * 64)()
        n = lib().dprf_ctx_last_call_devices(self._h, arr, 64)
        if n < 0:
            _check(n)
        return [arr[k].as_dict() for k in range(min(n, 64))]

    def search_range(self, charset, pwlen, start, count, stop_on_first=False, cap=1 << 16):
        """Verify keyspace indices [start, start+count) of charset^pwlen (itertools.product order).
        Returns (sorted hit indices (at most cap), total hits, stats dict).  The library's symbols are bytes: a str
        charset must be ASCII (a character of several UTF-8 bytes would enumerate as several symbols -- a different
        keyspace; brute_force.search_round spells such windows on the host instead), a bytes charset is taken as
        byte symbols (include/dprf.h dprf_search_range)."""
        if isinstance(charset, str) and any(ord(ch) >= 0x80 for ch in charset):
            raise DprfError(E_CHARSET, "search_range enumerates byte symbols: charset %r has multi-byte characters "
                                       "(search_symbols enumerates characters)" % charset)
        cs = _to_bytes(charset)
        hits = (ctypes.c_uint64 * max(1, cap))()
        nh = ctypes.c_int64()
        st = Stats()
        _check(lib().dprf_search_range(self._h, cs, len(cs), int(pwlen), int(start), int(count),
                                       1 if stop_on_first else 0, hits, cap, ctypes.byref(nh), ctypes.byref(st)))
        return list(hits[:min(nh.value, cap)]), nh.value, st.as_dict()

    def search_symbols(self, charset, pwlen, start, count, stop_on_first=False, cap=1 << 16):
        """Verify keyspace indices [start, start+count) of charset^pwlen over the CHARACTERS of a str charset (each
        symbol its UTF-8 bytes; for Office the library converts each to UTF-16LE), spelled on the device (ABI 7,
        include/dprf.h dprf_search_symbols).  Returns (sorted hit indices -- keyspace indices, like search_range's --,
        total hits, stats dict).  DprfError(E_PWLEN) when a candidate could exceed a 64-byte list slot."""
        syms = [ch.encode("utf-8") for ch in charset] if isinstance(charset, str) else [bytes([b]) for b in charset]
        offs = [0]
        for b in syms:
            offs.append(offs[-1] + len(b))
        so = (ctypes.c_uint32 * len(offs))(*offs)
        hits = (ctypes.c_uint64 * max(1, cap))()
        nh = ctypes.c_int64()
        st = Stats()
        _check(lib().dprf_search_symbols(self._h, b"".join(syms), so, len(syms), int(pwlen), int(start), int(count),
                                         1 if stop_on_first else 0, hits, cap, ctypes.byref(nh), ctypes.byref(st)))
        return [int(start) + h for h in hits[:min(nh.value, cap)]], nh.value, st.as_dict()

    def verify_blob(self, blob, offsets, stop_on_first=False, cap=1 << 16):
        """verify_list without per-candidate Python work: candidate k is blob[offsets[k]:offsets[k+1]]
        (offsets: n+1 ascending uint64, e.g. a numpy array).  Used by the GPU client for server payloads."""
        import numpy as np
        offs = np.ascontiguousarray(offsets, dtype=np.uint64)
        n = len(offs) - 1
        if n < 0:
            raise ValueError("offsets needs n+1 entries")
        hits = (ctypes.c_uint64 * max(1, cap))()
        nh = ctypes.c_int64()
        st = Stats()
        _check(lib().dprf_verify_list(self._h, bytes(blob), offs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                      n, 1 if stop_on_first else 0, hits, cap, ctypes.byref(nh), ctypes.byref(st)))
        return list(hits[:min(nh.value, cap)]), nh.value, st.as_dict()

    def list_status(self, blob, offsets):
        """Per-candidate validity for this format without device work: a numpy int8 array, 0 = valid,
        else the DPRF_E_* code verify_blob would fail the whole payload with."""
        import numpy as np
        offs = np.ascontiguousarray(offsets, dtype=np.uint64)
        n = len(offs) - 1
        st = np.zeros(max(1, n), dtype=np.int8)
        rc = lib().dprf_list_status(self._h, bytes(blob), offs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), n,
                                    st.ctypes.data_as(ctypes.POINTER(ctypes.c_int8)))
        if rc < 0:
            _check(rc)
        return st[:n]

    def verify_list(self, passwords, stop_on_first=False, cap=1 << 16):
        """Verify an explicit candidate list (a client payload).  Returns (sorted hit list indices,
        total hits, stats dict)."""
        bs = [_to_bytes(p) for p in passwords]
        offs = [0]
        for b in bs:
            offs.append(offs[-1] + len(b))
        blob = b"".join(bs)
        o = (ctypes.c_uint64 * len(offs))(*offs)
        hits = (ctypes.c_uint64 * max(1, cap))()
        nh = ctypes.c_int64()
        st = Stats()
        _check(lib().dprf_verify_list(self._h, blob, o, len(bs), 1 if stop_on_first else 0, hits, cap,
                                      ctypes.byref(nh), ctypes.byref(st)))
        return list(hits[:min(nh.value, cap)]), nh.value, st.as_dict()
