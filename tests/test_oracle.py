"""The CPU oracle pinned against published SHA-256 KATs and the golden fixtures
(tests/golden/gen_golden.py, an independent hashlib restatement)."""
import hashlib

import pytest

MAX = (1 << 64) - 1


def test_fips_kats(oracle_mod, golden):
    for k in golden["fips_kats"]:
        data = k["text"].encode() if k["text"] is not None else b"a" * k["repeat_a"]
        assert oracle_mod.c_sha256(data).hex() == k["sha256"]
        assert hashlib.sha256(data).hexdigest() == k["sha256"]


def test_sha256_all_padding_lengths(oracle_mod):
    for n in range(0, 260):
        data = bytes((i * 131 + n) & 0xFF for i in range(n))
        assert oracle_mod.c_sha256(data) == hashlib.sha256(data).digest(), n


def test_hash_kats(oracle_mod, golden):
    for k in golden["hash_kats"]:
        m, n, h = bytes.fromhex(k["msg_hex"]), int(k["nonce"]), int(k["hash"])
        assert oracle_mod.c_hash(m, n) == h, (k["name"], n)
    for k in golden["hash_kats"][::17]:
        m, n, h = bytes.fromhex(k["msg_hex"]), int(k["nonce"]), int(k["hash"])
        assert oracle_mod.py_hash(m, n) == h


def test_scan_kats(oracle_mod, golden):
    for k in golden["scan_kats"]:
        m, lo, hi = bytes.fromhex(k["msg_hex"]), int(k["lo"]), int(k["hi"])
        if hi >= lo and hi - lo > 400_000:
            continue  # the 10^7 case is covered on the GPU and by test_config1_oracle
        exp = (int(k["hash"]), int(k["nonce"]))
        assert oracle_mod.c_scan(m, lo, hi, threads=4) == exp, (k["name"], lo, hi)
        assert oracle_mod.c_scan(m, lo, hi, threads=1) == exp
        if "sum" in k:  # coverage checksum of hm_scan_checked
            assert oracle_mod.c_scan_sum(m, lo, hi, threads=3) == \
                (exp, int(k["sum"]), int(k["count"])), (k["name"], lo, hi)


def test_scan_sum_thread_invariance_and_python(oracle_mod):
    for m, lo, hi in [(b"bradfitz", 0, 2000), (b"q" * 56, 99_000, 101_000), (b"", MAX - 40, MAX),
                      (b"x", 5, 4)]:
        exp = oracle_mod.py_scan_sum(m, lo, hi)
        for t in (1, 2, 7):
            assert oracle_mod.c_scan_sum(m, lo, hi, threads=t) == exp, (m, lo, hi, t)


def test_config1_oracle(oracle_mod):
    # reference client: `client host:port bradfitz 10000000` -> Result 356393768206 7645578
    assert oracle_mod.c_scan(b"bradfitz", 0, 10**7, threads=8) == (356393768206, 7645578)


def test_miner_eval_kats(oracle_mod, golden):
    for k in golden["miner_eval_kats"]:
        m = bytes.fromhex(k["msg_hex"])
        lo, up = int(k["lower"]), int(k["upper"])
        exp = (int(k["hash"]), int(k["nonce"]))
        assert oracle_mod.c_miner_eval(m, lo, up) == exp
        assert oracle_mod.py_miner_eval(m, lo, up) == exp


@pytest.mark.parametrize("threads", [1, 2, 3, 7, 16])
def test_thread_split_invariance(oracle_mod, threads):
    for lo, hi in [(0, 0), (0, 1), (5, 9), (99_990, 100_009), (MAX - 20, MAX), (MAX, MAX)]:
        assert oracle_mod.c_scan(b"x", lo, hi, threads) == oracle_mod.py_scan(b"x", lo, hi)
