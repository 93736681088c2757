"""Interleaved A/B of libhipminer builds in ONE process (dev tool).
usage: python tools/ab_libs.py rounds lib1.so lib2.so[:K] ... [--no-check] [-- msg lo hi]
lib.so:K sets option 5 = K: the guided-self-scheduling build of the dequeue
experiment (profiles/r01/session2/gss/); plain paths set nothing."""
import ctypes, sys, time, json
sys.path.insert(0, '.')
from distributed_bitcoinminer_amd._lib import hm_result, hm_stats
args = sys.argv[1:]
check = "--no-check" not in args  # timing-only variants may give other answers
args = [a for a in args if a != "--no-check"]
msg, lo, hi = b"bradfitz", 0, 2**32 - 1
if "--" in args:
    i = args.index("--"); msg, lo, hi = args[i+1].encode(), int(args[i+2]), int(args[i+3]); args = args[:i]
    if msg == b"long120":  # BASELINE configs[2]'s message (random.Random(440))
        import random
        _r = random.Random(440)
        msg = bytes(_r.choice(range(0x21, 0x7F)) for _ in range(120))
rounds, libs = int(args[0]), args[1:]
ctxs = []
for p in libs:
    path, _, k = p.partition(":")
    L = ctypes.CDLL(path)
    L.hm_open.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    L.hm_scan.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(hm_result)]
    L.hm_scan_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(hm_stats)]
    h = ctypes.c_void_p(); dev = (ctypes.c_int * 1)(0)
    assert L.hm_open(dev, 1, ctypes.byref(h)) == 0
    if k:
        L.hm_set_option.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64]
        assert L.hm_set_option(h, 5, int(k)) == 0
    ctxs.append((p, L, h))
res = {p: [] for p in libs}
ref = None
for r in range(rounds):
    for p, L, h in ctxs:
        out = hm_result(); st = hm_stats()
        t = time.perf_counter(); rc = L.hm_scan(h, msg, len(msg), lo, hi, ctypes.byref(out)); dt = time.perf_counter() - t
        assert rc == 0
        L.hm_scan_stats(h, ctypes.byref(st))
        if ref is None: ref = (out.hash, out.nonce)
        assert not check or (out.hash, out.nonce) == ref, (p, out.hash, out.nonce, ref)
        res[p].append((dt, st.dom_nonces / st.dom_kernel_ms / 1e6))
for p in libs:
    v = sorted(x[1] for x in res[p][1:]); w = sorted(x[0] for x in res[p][1:])
    print(json.dumps({"lib": p, "median_dom_GHs": v[len(v)//2], "max_dom_GHs": v[-1], "median_wall_GHs": (hi-lo+1)/w[len(w)//2]/1e9}))
