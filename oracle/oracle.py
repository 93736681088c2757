"""CPU oracle for the reference's min-hash scan -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module, and only as the checker or the timed CPU baseline.  The product
path never routes through it.

Two independent restatements of the reference hot path live here
(paths relative to /root/reference, cmu440/ = p1/src/github.com/cmu440/):

* ``py_hash`` / ``py_scan``: pure Python over ``hashlib`` (OpenSSL's SHA-256),
  restating ``cmu440/bitcoin/hash.go:13-17`` and ``miner/miner.go:46-59``.
  Slow (~1 MH/s); used for golden fixtures and small cases.
* ``c_hash`` / ``c_scan`` / ``c_miner_eval``: ctypes over ``oracle/build/
  liboracle.so`` (``oracle/hm_oracle.c``: its own FIPS 180-4 SHA-256 and the
  Sprintf formatting), multi-threaded; used for larger parity ranges and as
  the CPU baseline in bench.py.
* ``fast_scan_sum``: ctypes over ``oracle/build/liboracle_fast.so``
  (``oracle/hm_oracle_fast.c``): the same scan with a per-segment midstate,
  in-place ASCII digit increments and the x86 SHA extensions.  Used only in
  the build container to generate the full-size fixtures (2^40 nonces of
  config 4, config 5's 20-digit ranges); checked against ``c_scan_sum`` by
  ``tests/test_oracle_fast.py``.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import subprocess

MAXU64 = (1 << 64) - 1
_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_FAST_PATH = os.path.join(_HERE, "build", "liboracle_fast.so")
_lib = None
_fast = None


def build() -> str:
    """Compile the C oracle in-tree (gcc; seconds)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        lib = ctypes.CDLL(_LIB_PATH)
        lib.oracle_hash.restype = ctypes.c_uint64
        lib.oracle_hash.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint64]
        for fn in (lib.oracle_scan, lib.oracle_miner_eval):
            fn.restype = None
            fn.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint64,
                           ctypes.c_int, ctypes.POINTER(ctypes.c_uint64),
                           ctypes.POINTER(ctypes.c_uint64)]
        lib.oracle_scan_sum.restype = None
        lib.oracle_scan_sum.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint64,
                                        ctypes.c_uint64, ctypes.c_int] + \
            [ctypes.POINTER(ctypes.c_uint64)] * 4
        lib.oracle_sha256.restype = None
        lib.oracle_sha256.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
        _lib = lib
    return _lib


def _b(msg) -> bytes:
    return msg.encode("utf-8") if isinstance(msg, str) else bytes(msg)


# ---- pure-Python restatement (hashlib) -------------------------------------

def py_hash(msg, nonce: int) -> int:
    """hash.go:13-17: SHA256(Sprintf("%s %d", msg, nonce)), first 8 bytes BE."""
    data = _b(msg) + b" " + str(int(nonce)).encode("ascii")
    return int.from_bytes(hashlib.sha256(data).digest()[:8], "big")


def py_scan(msg, lo: int, hi: int):
    """miner.go:48-59 over inclusive [lo, hi]: strict <, ascending, init (MAX, 0)."""
    result, index = MAXU64, 0
    m = _b(msg)
    for i in range(lo, hi + 1):
        h = int.from_bytes(hashlib.sha256(m + b" " + str(i).encode()).digest()[:8], "big")
        if h < result:
            result, index = h, i
    return result, index


def py_miner_eval(msg, lower: int, upper: int):
    """miner.go:50-59 with the `upper := Upper+1` uint64 wrap (:52)."""
    up = (upper + 1) & MAXU64
    if not lower < up:
        return MAXU64, 0
    return py_scan(msg, lower, up - 1)


# ---- C restatement (ctypes) --------------------------------------------------

def c_sha256(data: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    _load().oracle_sha256(data, len(data), out)
    return out.raw


def c_hash(msg, nonce: int) -> int:
    m = _b(msg)
    return int(_load().oracle_hash(m, len(m), nonce))


def c_scan(msg, lo: int, hi: int, threads: int = 0):
    m = _b(msg)
    if threads <= 0:
        threads = min(16, os.cpu_count() or 1)
    h, n = ctypes.c_uint64(), ctypes.c_uint64()
    _load().oracle_scan(m, len(m), lo, hi, threads, ctypes.byref(h), ctypes.byref(n))
    return int(h.value), int(n.value)


def c_scan_sum(msg, lo: int, hi: int, threads: int = 0):
    """c_scan plus the coverage checksum of hm_scan_checked:
    ((hash, nonce), sum of every key mod 2^64, nonces hashed)."""
    m = _b(msg)
    if threads <= 0:
        threads = min(16, os.cpu_count() or 1)
    h, n, s, c = (ctypes.c_uint64() for _ in range(4))
    _load().oracle_scan_sum(m, len(m), lo, hi, threads, ctypes.byref(h), ctypes.byref(n),
                            ctypes.byref(s), ctypes.byref(c))
    return (int(h.value), int(n.value)), int(s.value), int(c.value)


def py_scan_sum(msg, lo: int, hi: int):
    """py_scan plus the coverage checksum (independent hashlib restatement)."""
    m = _b(msg)
    result, index, total = MAXU64, 0, 0
    for i in range(lo, hi + 1):
        h = int.from_bytes(hashlib.sha256(m + b" " + str(i).encode()).digest()[:8], "big")
        total += h
        if h < result:
            result, index = h, i
    return (result, index), total & MAXU64, max(0, hi - lo + 1)


def c_miner_eval(msg, lower: int, upper: int, threads: int = 0):
    m = _b(msg)
    if threads <= 0:
        threads = min(16, os.cpu_count() or 1)
    h, n = ctypes.c_uint64(), ctypes.c_uint64()
    _load().oracle_miner_eval(m, len(m), lower, upper, threads, ctypes.byref(h), ctypes.byref(n))
    return int(h.value), int(n.value)


# ---- fast C restatement (SHA extensions; fixture generation) ----------------

def _load_fast():
    global _fast
    if _fast is None:
        if not os.path.exists(_FAST_PATH):
            build()
        lib = ctypes.CDLL(_FAST_PATH)
        lib.oracle_fast_available.restype = ctypes.c_int
        lib.oracle_fast_available.argtypes = []
        lib.oracle_fast_scan_sum.restype = None
        lib.oracle_fast_scan_sum.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint64,
                                             ctypes.c_uint64, ctypes.c_int] + \
            [ctypes.POINTER(ctypes.c_uint64)] * 4
        _fast = lib
    return _fast


def fast_available() -> bool:
    """True when this CPU has the SHA extensions hm_oracle_fast.c needs."""
    return bool(_load_fast().oracle_fast_available())


def fast_scan_sum(msg, lo: int, hi: int, threads: int = 0):
    """c_scan_sum's contract, computed by oracle/hm_oracle_fast.c."""
    if not fast_available():
        raise RuntimeError("CPU lacks the SHA extensions (hm_oracle_fast.c)")
    m = _b(msg)
    if threads <= 0:
        threads = min(16, os.cpu_count() or 1)  # the GPU box's per-GPU CPU share
    h, n, s, c = (ctypes.c_uint64() for _ in range(4))
    _load_fast().oracle_fast_scan_sum(m, len(m), lo, hi, threads, ctypes.byref(h), ctypes.byref(n),
                                      ctypes.byref(s), ctypes.byref(c))
    return (int(h.value), int(n.value)), int(s.value), int(c.value)
