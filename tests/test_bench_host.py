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


def test_roofline_prices_the_chained_kernel_by_rounds(monkeypatch):
    """the chained kernel's frac prices the rounds and schedule
    words it executes (frac == frac_rounds), not 1552 x C_eff; SURVEY's
    1552*C figure stays as frac_algorithmic_C (> 1 by the hoist)."""
    from distributed_bitcoinminer_amd import _lib
    monkeypatch.setattr(bench, "profiled", lambda k: (None, None, None, None))
    st = {"dom_compressions": 2, "dom_compressions_eff": 1.001, "dom_launches": 3,
          "dom_kernel_ms": 90.0, "dom_nonces": 4_284_967_296, "dom_grid": 1792,
          "dom_kernel": "hm_chained_kernel"}
    rl = bench.roofline(st, bench.long120(), 0, 2**32 - 1)
    ghs = 4_284_967_296 / 0.09
    assert rl["pricing"] == "rounds" and rl["frac"] == rl["frac_rounds"]
    assert abs(rl["ops_per_nonce"] - rl["ops_per_nonce_rounds"]) < 0.01
    assert "hoisted" in rl["pricing_note"]
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


def test_roofline_prices_the_tiled_kernel_at_1552_per_compression(monkeypatch):
    """cfg2's tiled kernel: frac = 1552 x C_eff (= C = 1) lane-ops per nonce,
    equal to frac_algorithmic_C; frac_rounds beside it."""
    monkeypatch.setattr(bench, "profiled", lambda k: (None, None, None, None))
    st = {"dom_compressions": 1, "dom_compressions_eff": 1.0, "dom_launches": 2,
          "dom_kernel_ms": 113.8, "dom_nonces": 4_194_967_296, "dom_grid": 1792,
          "dom_kernel": "hm_tiled_kernel<4, false, false>"}
    rl = bench.roofline(st, b"bradfitz", 0, 2**32 - 1)
    ghs = 4_194_967_296 / 0.1138
    assert rl["pricing"] == "1552 x C" and rl["ops_per_nonce"] == 1552
    assert abs(rl["frac"] - ghs * 1552 / 78.6432e12) < 1e-3
    assert rl["frac"] == rl["frac_algorithmic_C"]
    assert rl["frac_rounds"] < rl["frac"]
    assert rl["queue_units_per_launch"] == 4_194_967_296 // 2 // 6400
    assert rl["queue_tasks_per_atomic"] == 4
    # a launch of >= 10^11 nonces (cfg4's d = 12) fetches 16 tasks per atomic
    st4 = dict(st, dom_launches=1, dom_kernel_ms=23900.0, dom_nonces=900_000_000_000,
               dom_kernel="hm_tiled_kernel<5, true, false>")
    rl4 = bench.roofline(st4, b"bradfitz", 0, 2**40 - 1)
    assert rl4["queue_tasks_per_atomic"] == 16
    assert rl4["queue_atomics_per_launch"] == -(-(900_000_000_000 // 6400) // 16)


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


def _full():
    with open(os.path.join(ROOT, "tests", "golden", "full_size.json")) as f:
        return json.load(f)


def test_shard_check_weak_pieces_per_rank():
    """Each weak-scaling rank r's own answer is checked against the fixture
    piece [r*2^32, (r+1)*2^32) of its message (configs[1] and [2], r < 8)."""
    for w in _full()["weak"]:
        m = bytes.fromhex(w["msg_hex"])
        for r, p in enumerate(w["pieces"]):
            exp = (int(p["hash"]), int(p["nonce"]))
            got = bench.shard_check(m, r << 32, ((r + 1) << 32) - 1, exp)
            assert got["match"] is True and got["expected"]["nonce"] == exp[1], (w["name"], r)
            bad = bench.shard_check(m, r << 32, ((r + 1) << 32) - 1, (exp[0], exp[1] + 1))
            assert bad["match"] is False
    # no fixture: a shard the pieces do not tile exactly, or another message
    assert bench.shard_check(b"bradfitz", 5, (1 << 32) - 1, (1, 2)) is None
    assert bench.shard_check(b"other", 0, (1 << 32) - 1, (1, 2)) is None
    # an empty shard must answer the scan's seed
    assert bench.shard_check(b"bradfitz", None, None, (bench.MAXU64, 0))["match"] is True
    assert bench.shard_check(b"bradfitz", None, None, (5, 0))["match"] is False


def test_shard_check_cfg4_partition_shards():
    """configs[3]'s hm_partition shards for 1, 2, 4 and 8 ranks are unions of
    the fixture's pieces, so every rank of the driver's strong-scaling run is
    checked; their per-rank answers merge to the whole-range answer."""
    from distributed_bitcoinminer_amd.parallel import shard_range
    c4 = _full()["cfg4"]
    whole = (int(c4["whole"]["hash"]), int(c4["whole"]["nonce"]))
    for n in (1, 2, 4, 8):
        exps = []
        for r in range(n):
            lo, hi = shard_range(0, (1 << 40) - 1, n, r, msg=b"bradfitz")
            inside = [p for p in c4["pieces"] if int(p["lo"]) >= lo and int(p["hi"]) <= hi]
            exp = min((int(p["hash"]), int(p["nonce"])) for p in inside)
            got = bench.shard_check(b"bradfitz", lo, hi, exp)
            assert got is not None and got["match"] is True, (n, r)
            exps.append(exp)
        assert min(exps) == whole


def test_all_match():
    assert bench.all_match({"match": [True, True]}) is True
    assert bench.all_match({"match": [True, False, None]}) is False
    assert bench.all_match({"match": [True, None]}) is None


def test_single_process_failure_is_reported_not_raised():
    """bench.single_process_cfg4 runs (in a child) after every timed region of
    a multi-GPU line; a failure there (here: no GPU, hm_open fails) must land
    in the line, never abort the run that prints it."""
    import torch
    if torch.cuda.is_available():
        import pytest
        pytest.skip("GPU present")
    out = bench.single_process_cfg4([0, 1], rccl=True)
    assert out["devices"] == [0, 1] and "HipMinerError" in out["error"]
    assert out["merge_requested"] == "rccl"


def test_single_process_children_report_failures():
    """rank 0 runs the single-process workload as two fresh child processes
    (host merge, RCCL merge over the distinct ordinals): here, without a GPU,
    the real children start, fail in hm_open and report it as their entry;
    the per-GPU process count covers every rank's process plus the child."""
    import torch
    if torch.cuda.is_available():
        import pytest
        pytest.skip("GPU present")
    out = bench.run_single_process([0, 0], [0, 0, 0], timeout=120)
    assert out["host"]["devices"] == [0, 0] and out["rccl"]["devices"] == [0]
    for m in ("host", "rccl"):
        assert "HipMinerError" in out[m]["error"], out[m]
        assert out[m]["merge_requested"] == m and out[m]["child_s"] > 0
    assert out["processes_per_gpu"] == {"0": 4}
    out = bench.run_single_process([0, 1, 2, 3], [0, 1, 2, 3], timeout=120,
                                   child_cmd=lambda m, d: ["true"])
    assert out["processes_per_gpu"] == {str(g): 2 for g in range(4)}


def test_single_process_child_timeout_and_crash_become_entries():
    """A child that hangs is killed at its timeout, one that dies is an error
    entry with its exit status: run_single_process returns either way."""
    import sys
    import time
    t = time.perf_counter()
    out = bench.run_single_process(
        [0, 1], [0, 1], timeout=2,
        child_cmd=lambda m, d: [sys.executable, "-c", "import time; time.sleep(60)"] if m == "rccl"
        else [sys.executable, "-c", "import sys; sys.exit(3)"])
    assert time.perf_counter() - t < 40
    assert out["rccl"]["timeout"] == 2 and "killed" in out["rccl"]["error"]
    assert "exit status 3" in out["host"]["error"]
    ok = {"devices": [0, 1], "merge": "host", "result_vs_oracle": {"match": True}}
    out = bench.run_single_process(
        [0, 1], [0, 1], timeout=30,
        child_cmd=lambda m, d: [sys.executable, "-c",
                                "import json; print('banner'); print(json.dumps(%r))" % ok])
    assert out["host"]["result_vs_oracle"]["match"] is True and out["host"]["child_s"] > 0


def test_wrong_answers_ignores_child_errors():
    """The line's exit status: a child's error or timeout is reported, not a
    wrong answer; a child whose answer differs from the fixture is."""
    line = {"result_vs_oracle": {"match": True}, "ranks": {"match": [True]},
            "workloads": {"cfg4": {"result_vs_oracle": {"match": True}, "ranks": {"match": [True]}}},
            "single_process": {"host": {"error": "x"}, "rccl": {"timeout": 5, "error": "y"}}}
    assert bench.wrong_answers(line) == []
    line["single_process"]["rccl"] = {"result_vs_oracle": {"match": False}}
    assert len(bench.wrong_answers(line)) == 1
    line["ranks"]["match"] = [True, False]
    assert "primary" in bench.wrong_answers(line)


def test_kfd_queue_sampler_reads_sysfs(tmp_path, monkeypatch):
    """single_process.<merge>.queues_per_gpu: the queues (and processes) KFD
    lists per GPU while a child runs, keyed by the GPU's PCI address from
    KFD's topology; a host without KFD gives an error entry, not a failure."""
    proc, topo = tmp_path / "proc", tmp_path / "nodes"
    for pid, qs in {"101": ["1111", "1111", "2222"], "202": ["1111"], "303": []}.items():
        for i, g in enumerate(qs):
            d = proc / pid / "queues" / str(i)
            d.mkdir(parents=True)
            (d / "gpuid").write_text(g + "\n")
        (proc / pid).mkdir(parents=True, exist_ok=True)
    for n, (gid, loc) in enumerate([("0", None), ("1111", (0x75 << 8) | (0 << 3)),
                                    ("2222", (0xf5 << 8) | (0 << 3))]):
        d = topo / str(n)
        d.mkdir(parents=True)
        (d / "gpu_id").write_text(gid + "\n")
        (d / "properties").write_text(("location_id %d\ndomain 0\n" % loc) if loc else "cpu 1\n")
    monkeypatch.setattr(bench, "KFD_PROC", str(proc))
    monkeypatch.setattr(bench, "KFD_TOPOLOGY", str(topo))
    assert bench.kfd_queues() == {"1111": {"queues": 3, "processes": 2},
                                  "2222": {"queues": 1, "processes": 1}}
    assert bench.kfd_gpu_pci() == {"1111": "0000:75:00.0", "2222": "0000:f5:00.0"}
    with bench.QueueSampler(period_s=0.01) as qs:
        import time
        time.sleep(0.05)
    r = qs.result()
    assert r["samples"] >= 1 and r["max_queues_any_gpu"] == 3
    assert r["max"]["0000:75:00.0"] == {"queues": 3, "processes": 2}
    with bench.QueueSampler(period_s=0.01, pcis={"0000:f5:00.0"}) as qs:
        time.sleep(0.05)
    r = qs.result()
    assert r["max"] == {"0000:f5:00.0": {"queues": 1, "processes": 1}} and r["other_gpus"] == 1
    assert r["max_queues_any_gpu"] == 1
    monkeypatch.setattr(bench, "KFD_PROC", str(tmp_path / "none"))
    with bench.QueueSampler(period_s=0.01) as qs:
        pass
    assert "error" in qs.result()
    out = bench.run_single_process([0, 1], [0, 1], timeout=30, child_cmd=lambda m, d: ["true"])
    assert "queues_per_gpu" in out["host"] and "queues_per_gpu" in out["rccl"]
