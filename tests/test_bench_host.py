"""Host-side pieces of bench.py (no GPU): the oracle-fixture comparison of the
whole-job answer, the PMC summary gate on the code object, and the roofline
arithmetic of the JSON line."""
import json
import os

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_fixture_check_2p32_configs():
    got = bench.fixture_check(b"bradfitz", 0, 2**32 - 1, (5256245051, 1626825724))
    assert got["match"] and got["fixture"] == "tests/golden/large.json"
    got = bench.fixture_check(b"bradfitz", 0, 2**32 - 1, (5256245051, 1626825725))
    assert got["match"] is False
    with open(os.path.join(ROOT, "tests", "golden", "large.json")) as f:
        c3 = next(c for c in json.load(f) if c["name"] == "cfg3_long120")
    assert bench.fixture_check(bench.long120(), 0, 2**32 - 1,
                               (int(c3["hash"]), int(c3["nonce"])))["match"]
    assert bench.fixture_check(b"other", 0, 2**32 - 1, (1, 2)) is None


def test_fixture_check_weak_and_cfg4():
    with open(os.path.join(ROOT, "tests", "golden", "full_size.json")) as f:
        full = json.load(f)
    for w in full.get("weak", []):
        m = bytes.fromhex(w["msg_hex"])
        for n in (1, 2, 4, 8):
            best = min((int(p["hash"]), int(p["nonce"])) for p in w["pieces"][:n])
            assert bench.fixture_check(m, 0, (n << 32) - 1, best)["match"]
    if "cfg4" in full:
        wh = full["cfg4"]["whole"]
        assert bench.fixture_check(b"bradfitz", 0, (1 << 40) - 1,
                                   (int(wh["hash"]), int(wh["nonce"])))["match"]


def test_profiled_requires_this_code_object(tmp_path, monkeypatch):
    """A PMC summary measured on another build of the scan kernels is not used."""
    sha = bench.code_object_sha16()
    prof = tmp_path / "profiles" / "r99"
    prof.mkdir(parents=True)
    entry = {"hbm_bytes_per_launch": 4.0, "launches": 2, "nonces": 8,
             "f_eff_ghz_largest_dispatch": 2.3, "valu_insts_per_wave_iteration_64_nonces": 1200.0}
    (prof / "pmc_summary.json").write_text(json.dumps({"k": dict(entry, code_object_sha16="0" * 16)}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "code_object_sha16", lambda: sha or "f" * 16)
    assert bench.profiled("k") == (None, None, None, None)
    (prof / "pmc_summary.json").write_text(json.dumps({"k": dict(entry, code_object_sha16=sha or "f" * 16)}))
    assert bench.profiled("k")[:3] == (1.0, 2.3, 1200.0)


def test_roofline_prices_executed_compressions(monkeypatch):
    """frac uses C_eff (compressions the kernel executes per nonce), the
    algorithmic 1552*C is reported beside it."""
    from distributed_bitcoinminer_amd import _lib
    monkeypatch.setattr(bench, "profiled", lambda k: (None, None, None, None))
    st = {"dom_compressions": 2, "dom_compressions_eff": 1.001, "dom_launches": 3,
          "dom_kernel_ms": 90.0, "dom_nonces": 4_284_967_296, "dom_grid": 1792,
          "dom_kernel": "hm_chained_kernel"}
    rl = bench.roofline(st, bench.long120(), 0, 2**32 - 1)
    ghs = 4_284_967_296 / 0.09
    assert abs(rl["frac"] - ghs * 1552 * 1.001 / 78.6432e12) < 1e-3
    assert abs(rl["frac_algorithmic_C"] - ghs * 1552 * 2 / 78.6432e12) < 1e-3
    assert rl["compressions_per_nonce"] == 1.001 and rl["compressions_per_nonce_algorithmic"] == 2
    assert _lib.debug_plan(bench.long120(), 0, 2**32 - 1)  # the plan the line reads
    # frac_rounds: 64 table-driven rounds + the per-lane block 0 + the K+W
    # tables (10^f rows of 48 schedule words and 64 K adds per segment)
    segs = [s for s in _lib.debug_plan(bench.long120(), 0, 2**32 - 1) if s["kind"] == 3]
    n = sum(s["hi"] - s["lo"] + 1 for s in segs)
    ops = 1024 + 1552 * 0.001 + sum(10 ** s["f"] * (48 * 11 + 64) for s in segs) / n
    assert abs(rl["ops_per_nonce_rounds"] - ops) < 0.01
    assert abs(rl["frac_rounds"] - ghs * ops / 78.6432e12) < 1e-3


def test_rounds_ops_of_the_tiled_kernel():
    """cfg2's hm_tiled_kernel<4, false, false>: rounds 0..4 once per tens digit,
    round 4 then 2 adds per nonce, rounds 5..63 per nonce; the 45 schedule
    words W19..W63 depend on the loop word W4, W16..W18 once per task."""
    seg = {"kind": 2, "W1": 4, "straddle": 0, "trailer": 0}
    ops, table = bench.rounds_ops_per_nonce(seg, 1.0)
    assert table == 0
    assert abs(ops - (59 * 16 + 2 + 5 * 16 / 10 + 45 * 11 + 3 * 11 / 100)) < 1e-9
    assert bench._sched_deps({4}) == set(range(19, 64))
    # a constant trailer block adds 64 table-driven rounds per nonce
    ops_t, _ = bench.rounds_ops_per_nonce(dict(seg, W1=14, trailer=1), 2.0)
    ops_n, _ = bench.rounds_ops_per_nonce(dict(seg, W1=14), 1.0)
    assert abs(ops_t - ops_n - 64 * 16) < 1e-9
