"""ctypes binding of libhipminer.so (include/hipminer.h).

The library is built in-tree by ``__graft_entry__.build()`` (or ``make -C
distributed_bitcoinminer_amd/csrc``).  There is no silent fallback: if the
library or a GPU is missing, the calls raise ``HipMinerError``; ``scan_cpu``
(hm_scan_cpu) is the host scan a caller may pick explicitly.
"""
from __future__ import annotations

import ctypes
import os
import re
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libhipminer.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "hipminer.h")

HM_OK = 0
HM_ERR_INVALID = -1
HM_ERR_NO_DEVICE = -2
HM_ERR_HIP = -3
HM_ERR_NOMEM = -4
HM_ERR_RCCL = -5
HM_ERR_INTERNAL = -6
HM_ERR_TIMEOUT = -7

HM_KIND_NONE, HM_KIND_GENERIC, HM_KIND_TILED, HM_KIND_CHAINED, HM_KIND_FUSED = 0, 1, 2, 3, 4
HM_OPT_FORCE_GENERIC, HM_OPT_MERGE_RCCL, HM_OPT_GRID_PER_CU, HM_OPT_STREAMS = 1, 2, 3, 4
HM_OPT_TABLE_DIGITS = 7
HM_OPT_TABLE_ROWS_CAP = 8
HM_OPT_TEST_MID_SYNC = 9
HM_OPT_FUSED = 10
HM_OPT_FUSED_FLAGS = 11
HM_OPT_FUSED_PARTS = 12
HM_OPT_DEADLINE_MS = 13
HM_OPT_FUSED_TAIL = 14
HM_OPT_TAIL_FUSED = 15
HM_OPT_HOST_RESULT = 16
HM_OPT_QUEUE_BATCH = 17
HM_OPT_FUSED_TRACE = 18
HM_MERGE_NONE, HM_MERGE_HOST, HM_MERGE_RCCL = 0, 1, 2


class HipMinerError(RuntimeError):
    def __init__(self, rc: int, what: str = ""):
        self.rc = rc
        msg = strerror(rc) if _lib_or_none() else f"rc={rc}"
        super().__init__(f"{what}: {msg} (rc={rc})" if what else f"{msg} (rc={rc})")


class hm_result(ctypes.Structure):
    _fields_ = [("hash", ctypes.c_uint64), ("nonce", ctypes.c_uint64)]


class hm_request(ctypes.Structure):
    _fields_ = [("msg", ctypes.c_char_p), ("len", ctypes.c_size_t),
                ("lo", ctypes.c_uint64), ("hi", ctypes.c_uint64)]


class hm_stats(ctypes.Structure):
    _fields_ = [("wall_ms", ctypes.c_double), ("kernel_ms", ctypes.c_double),
                ("dom_kernel_ms", ctypes.c_double), ("nonces", ctypes.c_uint64),
                ("dom_nonces", ctypes.c_uint64), ("dom_compressions", ctypes.c_uint64),
                ("launches", ctypes.c_int32), ("dom_kind", ctypes.c_int32),
                ("ndev", ctypes.c_int32), ("dom_grid", ctypes.c_int32),
                ("dom_launches", ctypes.c_int32), ("merge", ctypes.c_int32),
                ("dom_kernel", ctypes.c_char * 64), ("dom_compressions_eff", ctypes.c_double),
                ("enqueue_ms", ctypes.c_double), ("mid_call_syncs", ctypes.c_int32),
                ("table_grows", ctypes.c_int32), ("deadline_ms", ctypes.c_double)]

    def as_dict(self) -> dict:
        d = {k: getattr(self, k) for k, _ in self._fields_}
        d["dom_kernel"] = self.dom_kernel.decode()
        return d


_lib = None
_lock = threading.Lock()


def _lib_or_none():
    return _lib


def load() -> ctypes.CDLL:
    """Load the in-tree libhipminer.so; raise if it has not been built."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise HipMinerError(HM_ERR_NO_DEVICE,
                                f"{LIB_PATH} missing: run __graft_entry__.build()")
        lib = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.c_char_p
        lib.hm_hash.restype = ctypes.c_uint64
        lib.hm_hash.argtypes = [u8p, ctypes.c_size_t, ctypes.c_uint64]
        lib.hm_open.restype = ctypes.c_int
        lib.hm_open.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                ctypes.POINTER(ctypes.c_void_p)]
        lib.hm_scan.restype = ctypes.c_int
        lib.hm_scan.argtypes = [ctypes.c_void_p, u8p, ctypes.c_size_t, ctypes.c_uint64,
                                ctypes.c_uint64, ctypes.POINTER(hm_result)]
        lib.hm_scan_many.restype = ctypes.c_int
        lib.hm_scan_many.argtypes = [ctypes.c_void_p, ctypes.POINTER(hm_request), ctypes.c_int,
                                     ctypes.POINTER(hm_result)]
        lib.hm_scan_checked.restype = ctypes.c_int
        lib.hm_scan_checked.argtypes = [ctypes.c_void_p, u8p, ctypes.c_size_t, ctypes.c_uint64,
                                        ctypes.c_uint64, ctypes.POINTER(hm_result),
                                        ctypes.POINTER(ctypes.c_uint64),
                                        ctypes.POINTER(ctypes.c_uint64)]
        lib.hm_scan_stats.restype = ctypes.c_int
        lib.hm_scan_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(hm_stats)]
        lib.hm_scan_stats_sized.restype = ctypes.c_int
        lib.hm_scan_stats_sized.argtypes = [ctypes.c_void_p, ctypes.POINTER(hm_stats),
                                            ctypes.c_size_t]
        lib.hm_debug_code_object.restype = ctypes.c_size_t
        lib.hm_debug_code_object.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
        lib.hm_set_option.restype = ctypes.c_int
        lib.hm_set_option.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64]
        lib.hm_strerror.restype = ctypes.c_char_p
        lib.hm_strerror.argtypes = [ctypes.c_int]
        lib.hm_close.restype = None
        lib.hm_close.argtypes = [ctypes.c_void_p]
        lib.hm_version.restype = ctypes.c_int
        lib.hm_version.argtypes = []
        lib.hm_build_id.restype = ctypes.c_char_p
        lib.hm_build_id.argtypes = []
        lib.hm_partition.restype = ctypes.c_int
        lib.hm_partition.argtypes = [u8p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint64,
                                     ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]
        lib.hm_scan_cpu.restype = ctypes.c_int
        lib.hm_scan_cpu.argtypes = [u8p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint64,
                                    ctypes.c_int, ctypes.POINTER(hm_result)]
        lib.hm_debug_auto_deadline_ms.restype = ctypes.c_double
        lib.hm_debug_auto_deadline_ms.argtypes = [u8p, ctypes.c_size_t, ctypes.c_uint64,
                                                  ctypes.c_uint64, ctypes.c_int]
        lib.hm_debug_fused_trace.restype = ctypes.c_int
        lib.hm_debug_fused_trace.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64),
                                             ctypes.c_int]
        lib.hm_debug_streams_made.restype = ctypes.c_int
        lib.hm_debug_streams_made.argtypes = [ctypes.c_void_p, ctypes.c_int]
        lib.hm_debug_plan.restype = ctypes.c_int
        lib.hm_debug_plan.argtypes = [u8p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint64,
                                      ctypes.c_int, ctypes.POINTER(ctypes.c_int64), ctypes.c_int]
        _lib = lib
        return lib


def strerror(rc: int) -> str:
    return load().hm_strerror(rc).decode()


def header_symbols() -> list[str]:
    """Function names declared in include/hipminer.h."""
    with open(HEADER_PATH) as f:
        text = f.read()
    return sorted(set(re.findall(r"\b(hm_[a-z_]+)\s*\(", text)))


def as_bytes(msg) -> bytes:
    """Go strings are byte strings; str is encoded as UTF-8 (Go source literals)."""
    return msg.encode("utf-8") if isinstance(msg, str) else bytes(msg)


class Context:
    """One hipminer context (hm_open .. hm_close) on a set of HIP devices."""

    def __init__(self, devices=None):
        lib = load()
        handle = ctypes.c_void_p()
        if devices:
            arr = (ctypes.c_int * len(devices))(*devices)
            rc = lib.hm_open(arr, len(devices), ctypes.byref(handle))
        else:
            rc = lib.hm_open(None, 0, ctypes.byref(handle))
        if rc != HM_OK:
            raise HipMinerError(rc, "hm_open")
        self._h = handle
        self._lib = lib

    def scan(self, msg, lo: int, hi: int) -> tuple[int, int]:
        m = as_bytes(msg)
        out = hm_result()
        rc = self._lib.hm_scan(self._h, m, len(m), lo, hi, ctypes.byref(out))
        if rc != HM_OK:
            raise HipMinerError(rc, "hm_scan")
        return int(out.hash), int(out.nonce)

    def scan_checked(self, msg, lo: int, hi: int) -> tuple[tuple[int, int], int, int]:
        """hm_scan_checked: ((hash, nonce), sum of all keys mod 2^64, nonces hashed)."""
        m = as_bytes(msg)
        out = hm_result()
        s, c = ctypes.c_uint64(), ctypes.c_uint64()
        rc = self._lib.hm_scan_checked(self._h, m, len(m), lo, hi, ctypes.byref(out),
                                       ctypes.byref(s), ctypes.byref(c))
        if rc != HM_OK:
            raise HipMinerError(rc, "hm_scan_checked")
        return (int(out.hash), int(out.nonce)), int(s.value), int(c.value)

    def scan_many(self, requests) -> list[tuple[int, int]]:
        """hm_scan_many over [(msg, lo, hi), ...]."""
        reqs = list(requests)
        n = len(reqs)
        keep = [as_bytes(m) for m, _, _ in reqs]
        arr = (hm_request * max(1, n))()
        for i, ((_, lo, hi), m) in enumerate(zip(reqs, keep)):
            arr[i] = hm_request(m, len(m), lo, hi)
        outs = (hm_result * max(1, n))()
        rc = self._lib.hm_scan_many(self._h, arr, n, outs)
        if rc != HM_OK:
            raise HipMinerError(rc, "hm_scan_many")
        return [(int(outs[i].hash), int(outs[i].nonce)) for i in range(n)]

    def stats(self) -> dict:
        st = hm_stats()
        rc = self._lib.hm_scan_stats_sized(self._h, ctypes.byref(st), ctypes.sizeof(st))
        if rc != HM_OK:
            raise HipMinerError(rc, "hm_scan_stats")
        return st.as_dict()

    def streams_made(self, device_index: int = 0) -> int:
        """HIP streams (hardware queues) the context has made on its
        device_index-th device (debug export; ABI 1.8 makes them on first use)."""
        return int(self._lib.hm_debug_streams_made(self._h, device_index))

    def fused_trace(self) -> list:
        """The last traced fused launch's timeline (HM_OPT_FUSED_TRACE):
        per wave slot (start, last task start, end, tasks), wall-clock ticks."""
        buf = (ctypes.c_uint64 * (4 * 32768))()
        n = self._lib.hm_debug_fused_trace(self._h, buf, 32768)
        if n < 0:
            raise HipMinerError(n, "hm_debug_fused_trace")
        return [tuple(int(x) for x in buf[4 * i: 4 * i + 4]) for i in range(n)]

    def set_option(self, opt: int, value: int) -> None:
        rc = self._lib.hm_set_option(self._h, opt, value)
        if rc != HM_OK:
            raise HipMinerError(rc, "hm_set_option")

    def close(self) -> None:
        if self._h:
            self._lib.hm_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def host_hash(msg, nonce: int) -> int:
    """hm_hash: bitcoin.Hash on the host (hash.go:13-17)."""
    m = as_bytes(msg)
    return int(load().hm_hash(m, len(m), nonce))


def scan_cpu(msg, lo: int, hi: int, threads: int = 0) -> tuple[int, int]:
    """hm_scan_cpu (ABI 1.7): the same scan as Context.scan on the host's
    cores, for callers whose GPU is missing or failed; never
    used by Context."""
    m = as_bytes(msg)
    out = hm_result()
    rc = load().hm_scan_cpu(m, len(m), lo, hi, threads, ctypes.byref(out))
    if rc != HM_OK:
        raise HipMinerError(rc, "hm_scan_cpu")
    return int(out.hash), int(out.nonce)


def partition(msg, lo: int, hi: int, n: int) -> list:
    """hm_partition: n contiguous shards of [lo, hi] with near-equal modelled
    GPU cost for msg; each entry is (lo_i, hi_i) or None when empty.  Host-only."""
    m = as_bytes(msg)
    buf = (ctypes.c_uint64 * (2 * max(1, n)))()
    rc = load().hm_partition(m, len(m), lo, hi, n, buf)
    if rc != HM_OK:
        raise HipMinerError(rc, "hm_partition")
    out = []
    for i in range(n):
        a, b = int(buf[2 * i]), int(buf[2 * i + 1])
        out.append((a, b) if a <= b else None)
    return out


def build_id() -> str:
    """hm_build_id: digest of the sources the loaded library was built from."""
    return load().hm_build_id().decode()


def build_matches_tree() -> bool:
    """True when the loaded libhipminer.so was built from this tree's sources
    (build_id.tree_digest over csrc/ and include/hipminer.h)."""
    from distributed_bitcoinminer_amd import build_id as bid
    return build_id() == bid.tree_digest()


def code_object_sha16() -> str:
    """sha256 (16 hex digits) of the scan kernels' code object embedded in the
    loaded libhipminer.so (the bytes hipModuleLoadData gets)."""
    import hashlib
    p = ctypes.c_void_p()
    n = load().hm_debug_code_object(ctypes.byref(p))
    return hashlib.sha256(ctypes.string_at(p.value, n)).hexdigest()[:16]


def debug_plan(msg, lo: int, hi: int, force_generic: bool = False) -> list[dict]:
    m = as_bytes(msg)
    cap = 32
    keys = ("d", "lo", "hi", "kind", "W1", "V", "trailer", "straddle", "cost", "lane3",
            "f", "tch", "fe")
    k = len(keys)
    buf = (ctypes.c_int64 * (k * cap))()
    n = load().hm_debug_plan(m, len(m), lo, hi, int(force_generic), buf, cap)
    out = []
    for i in range(min(n, cap)):
        row = dict(zip(keys, buf[k * i: k * i + k]))
        row["lo"] &= (1 << 64) - 1
        row["hi"] &= (1 << 64) - 1
        out.append(row)
    return out
