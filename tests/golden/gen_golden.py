#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ (run in the build container).

The reference (Go; cmu440/bitcoin/hash.go:13-17 + miner/miner.go:46-59) cannot
run here -- no Go toolchain -- and its own tests hold no vectors for the hash
or the scan.  These fixtures therefore come from this
self-contained restatement over Python's ``hashlib`` (OpenSSL SHA-256, an
implementation independent of both oracle/hm_oracle.c and the HIP kernels):

  Hash(msg, n)  = BigEndian.Uint64(SHA256(msg ‖ " " ‖ decimal(n))[:8])
  scan(lo, hi)  = ascending strict-< min over inclusive [lo, hi], init (MAX, 0)
  miner_eval    = scan with miner.go:52's `upper := Upper+1` uint64 wrap

The FIPS 180-4 / NIST known answers in fips_kats are published constants and
pin the SHA-256 underneath.

Usage: python tests/golden/gen_golden.py   (≈1 min on 8 cores)
"""
from __future__ import annotations

import hashlib
import json
import os
import random
from multiprocessing import Pool

MAX = (1 << 64) - 1
HERE = os.path.dirname(os.path.abspath(__file__))


def H(msg: bytes, n: int) -> int:
    return int.from_bytes(hashlib.sha256(msg + b" " + str(n).encode()).digest()[:8], "big")


def scan(args):
    return scan_sum(args)[0]


def scan_sum(args):
    """(best, idx) plus the coverage checksum of hm_scan_checked:
    the sum of every key mod 2^64 and the count of nonces."""
    msg, lo, hi = args
    best, idx, total = MAX, 0, 0
    for i in range(lo, hi + 1):
        h = H(msg, i)
        total += h
        if h < best:
            best, idx = h, i
    return (best, idx), total & MAX, max(0, hi - lo + 1)


def miner_eval(msg, lower, upper):
    up = (upper + 1) & MAX
    if not lower < up:
        return MAX, 0
    return scan((msg, lower, up - 1))


def msg_of_len(L: int) -> bytes:
    """Deterministic message of L bytes over all byte values (NUL, '%', 0xFF ...)."""
    rng = random.Random(1000 + L)
    return bytes(rng.randrange(256) for _ in range(L))


def long120() -> bytes:
    rng = random.Random(440)
    return bytes(rng.choice(range(0x21, 0x7F)) for _ in range(120))


FIPS = [
    ("", "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"),
    ("abc", "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"),
    ("abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq",
     "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"),
    ("abcdefghbcdefghicdefghijdefghijkefghijklfghijklmghijklmnhijklmnoijklmnopjklmnopq"
     "klmnopqrlmnopqrsmnopqrstnopqrstu",
     "cf5b16a778af8380036ce59e7b0492370b249b11e8f07a51afac45037afee9d1"),
    ("a" * 1000000, "cdc76e5c9914fb9281a1c7e284d73e67f1809a48a497200e046d39ccc7112cd0"),
]

KAT_NONCES = sorted(set(
    [0, 1, 9, 10, 99, 100, 19970521, 2**32 - 1, 2**32, 2**63, MAX - 1, MAX]
    + [10**k - 1 for k in range(1, 20)] + [10**k for k in range(1, 20)]))
KAT_LENS = [0, 1, 2, 3, 7, 8, 9, 30, 35, 36, 41, 44, 45, 46, 50, 53, 54, 55, 56, 57, 60,
            62, 63, 64, 65, 100, 110, 118, 119, 120, 121, 126, 127, 128, 129, 150, 200]


def main():
    out = {}
    # 1. FIPS KATs (published), checked against hashlib here.
    fips = []
    for text, hexd in FIPS:
        assert hashlib.sha256(text.encode()).hexdigest() == hexd, text[:10]
        fips.append({"text": text if len(text) < 1000 else None,
                     "repeat_a": len(text) if len(text) >= 1000 else None, "sha256": hexd})
    out["fips_kats"] = fips

    # 2. single-hash KATs: every padding boundary x every digit-count change.
    named = {"bradfitz": b"bradfitz", "thom yorke": b"thom yorke",
             "jonny greenwood": b"jonny greenwood", "long120": long120()}
    hk = []
    for name, m in named.items():
        for n in KAT_NONCES:
            hk.append({"msg_hex": m.hex(), "name": name, "nonce": str(n), "hash": str(H(m, n))})
    for L in KAT_LENS:
        m = msg_of_len(L)
        for n in KAT_NONCES:
            hk.append({"msg_hex": m.hex(), "name": f"len{L}", "nonce": str(n), "hash": str(H(m, n))})
    out["hash_kats"] = hk

    # 3. range scans (inclusive [lo, hi]) and miner_eval (miner.go wrap quirk).
    b = b"bradfitz"
    cases = [
        ("bradfitz", b, 0, 9999),
        ("jonny greenwood", b"jonny greenwood", 200, 71010),
        ("bradfitz", b, 0, 10**7),                      # config 1 answer
        ("bradfitz", b, 99990, 100009),                 # 5 -> 6 digits
        ("bradfitz", b, MAX - 10**5, MAX - 1),          # 20-digit nonces
        ("bradfitz", b, MAX - 5, MAX),                  # inclusive to 2^64-1
        ("bradfitz", b, 0, 0),
        ("bradfitz", b, MAX, MAX),
        ("long120", long120(), 0, 10**5),
        ("long120", long120(), 10**9 - 2000, 10**9 + 2000),
        ("thom yorke", b"thom yorke", 19970000, 19971000),
        ("empty", b"", 0, 20000),
    ]
    rng = random.Random(12345)
    for L in KAT_LENS:
        m = msg_of_len(L)
        for k in (1, 2, 3, 5, 9, 10, 13, 19):
            c = 10**k
            cases.append((f"len{L}", m, max(0, c - 150), c + 150))
        lo = rng.randrange(10**19, MAX - 3000)
        cases.append((f"len{L}", m, lo, lo + 1500))
        lo = rng.randrange(0, 2**40)
        cases.append((f"len{L}", m, lo, lo + 1500))
    for L in (0, 8, 44, 45, 55, 56, 63, 64, 119, 120):
        cases.append((f"len{L}", msg_of_len(L), 0, 300000))
    with Pool(min(8, os.cpu_count() or 1)) as pool:
        res = pool.map(scan_sum, [(m, lo, hi) for _, m, lo, hi in cases], chunksize=1)
    sk = []
    for (name, m, lo, hi), ((h, n), sm, cnt) in zip(cases, res):
        sk.append({"name": name, "msg_hex": m.hex(), "lo": str(lo), "hi": str(hi),
                   "hash": str(h), "nonce": str(n), "sum": str(sm), "count": str(cnt)})
    sk.append({"name": "empty-range", "msg_hex": b.hex(), "lo": "5", "hi": "4",
               "hash": str(MAX), "nonce": "0", "sum": "0", "count": "0"})
    out["scan_kats"] = sk

    me = []
    for lower, upper in [(0, 9999), (MAX - 5, MAX), (5, 4), (MAX - 10, MAX - 1), (MAX, MAX)]:
        h, n = miner_eval(b, lower, upper)
        me.append({"msg_hex": b.hex(), "lower": str(lower), "upper": str(upper),
                   "hash": str(h), "nonce": str(n)})
    out["miner_eval_kats"] = me

    path = os.path.join(HERE, "golden.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print(f"wrote {path}: {len(hk)} hash KATs, {len(sk)} scans, {len(me)} miner_eval")


if __name__ == "__main__":
    main()
