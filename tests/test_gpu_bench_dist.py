"""bench.py's torch.distributed path with the HIP scan underneath, launched the
way the driver launches it (python -m torch.distributed.run ... bench.py
--gpus N), on the GPU box:

* 2 ranks with the gloo backend sharing GPU 0 (RCCL refuses two ranks on one
  device): cfg2 weak scaling ([0, 2 * 2^32)) and the cfg4 secondary (strong
  scaling: [0, 2^40) as 2 hm_partition shards), each whole-job answer equal to
  its oracle fixture (tests/golden/full_size.json);
* 1 rank with the nccl backend (RCCL) and HM_BENCH_FORCE_DIST=1, so the
  RCCL all-gather of the 16-B candidates runs end to end: cfg2 and the cfg3
  secondary against tests/golden/large.json.

The reference's split and merge: cmu440/bitcoin/server/server.go:165-205 and
:273-276.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _torchrun(nproc, args, env_extra, timeout):
    # generous limits: on a fresh box these children may be the first to
    # import torch (1-2 minutes while the image pages in)
    env = dict(os.environ, **env_extra)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1",
           "--nproc-per-node", str(nproc), "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), "bench.py", "--gpus", str(nproc)] + args
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 prints exactly one JSON line
    return json.loads(lines[0])


def _per_rank(ranks, n, ordinals=None):
    """Every rank reports its own answer, device and kernel rate, and its
    answer equals the fixture piece(s) of its own shard."""
    assert ranks["match"] == [True] * n, ranks
    assert len(ranks["answer"]) == n and len(ranks["device"]) == n
    assert all(g > 0 for g in ranks["kernel_GHs"]), ranks["kernel_GHs"]
    if ordinals is not None:
        assert [d["ordinal"] for d in ranks["device"]] == ordinals
    assert all(len(d["pci_bus_id"]) == 12 for d in ranks["device"]), ranks["device"]


def test_bench_torchrun_gloo_two_ranks_cfg2_and_cfg4():
    """Also the multi-rank single-process pass: rank 1 parks in the host-side
    wait group while rank 0 runs both children (HM_BENCH_SP_DEVICES=0: one
    context on GPU 0, host merge and a 1-rank RCCL merge)."""
    line = _torchrun(2, ["--steps", "1", "--warmup", "0", "--secondary", "cfg4",
                         "--no-cpu-baseline"],
                     {"HM_BENCH_BACKEND": "gloo", "HM_BENCH_SP_DEVICES": "0"}, timeout=600)
    assert line["n_gpus"] == 2 and line["config"]["merge"] == "gloo"
    assert line["result_vs_oracle"]["match"] is True, line["result_vs_oracle"]
    assert len(line["ranks"]["local_ms"]) == 2
    assert line["build_matches_tree"] is True, line["build_id"]
    assert line["all_ranks_match"] is True
    _per_rank(line["ranks"], 2, [0, 0])  # gloo rehearsal: both ranks on GPU 0
    # the merged answer is the minimum of the ranks' own answers
    best = min((a["hash"], a["nonce"]) for a in line["ranks"]["answer"])
    assert best == (line["result"]["hash"], line["result"]["nonce"])
    c4 = line["workloads"]["cfg4"]
    assert c4["all_ranks_match"] is True
    _per_rank(c4["ranks"], 2, [0, 0])
    assert c4["scaling"] == "strong"
    assert c4["result_vs_oracle"]["fixture"] == "tests/golden/full_size.json"
    assert c4["result_vs_oracle"]["match"] is True, c4["result_vs_oracle"]
    assert len(c4["ranks"]["local_ms"]) == 2 and c4["ranks"]["spread_pct"] >= 0
    # rank 0's shard is the first hm_partition shard of [0, 2^40)
    from distributed_bitcoinminer_amd import _lib
    lo, hi = _lib.partition(b"bradfitz", 0, (1 << 40) - 1, 2)[0]
    assert c4["nonces_rank0"] == hi - lo + 1
    sp = line["single_process"]
    assert sp["processes_per_gpu"] == {"0": 3}, sp  # both ranks and the child
    # the queues the job's GPU carried, measured (KFD sysfs): after the timed
    # regions, and while each child ran
    pci = line["ranks"]["device"][0]["pci_bus_id"]
    assert line["config"]["hip_streams_per_gpu"] == 2
    q = line["queues_per_gpu"]
    assert "error" in q or set(q["max"]) <= {pci}, q
    for m, merge in (("host", "none"), ("rccl", "RCCL all-gather")):
        e = sp[m]
        assert "error" not in e, e
        assert e["devices"] == [0] and e["merge"] == merge, e
        assert e["result_vs_oracle"]["match"] is True and e["mid_call_syncs"] == 0, e
        assert e["streams_per_gpu"] == 2, e
        qs = e["queues_per_gpu"]
        assert "error" in qs or (qs["samples"] >= 1 and set(qs["max"]) <= {pci}), qs


def test_bench_torchrun_rccl_world1_cfg2_and_cfg3():
    line = _torchrun(1, ["--steps", "2", "--warmup", "1", "--secondary", "cfg3",
                         "--no-cpu-baseline"], {"HM_BENCH_FORCE_DIST": "1"}, timeout=300)
    assert line["config"]["merge"] == "RCCL all-gather"
    assert line["result_vs_oracle"]["match"] is True, line["result_vs_oracle"]
    assert line["all_ranks_match"] is True and line["build_matches_tree"] is True
    _per_rank(line["ranks"], 1, [0])
    c3 = line["workloads"]["cfg3"]
    assert c3["all_ranks_match"] is True
    assert c3["result_vs_oracle"]["match"] is True, c3["result_vs_oracle"]
    rl = c3["roofline"]
    assert rl["kernel"] == "hm_chained_kernel"
    # the chained kernel is priced by the rounds it executes
    assert rl["pricing"] == "rounds" and 0 < rl["frac"] == rl["frac_rounds"] <= 1.0
    assert rl["frac_algorithmic_C"] > 1.0  # SURVEY's 1552 x C: block 0 hoisted


def test_bench_torchrun_rccl_all_visible_gpus():
    """With >= 2 visible GPUs (a multi-GPU test box), the driver's launch line
    itself: one RCCL rank per GPU over xGMI, cfg2 weak ([0, N*2^32)) and the
    cfg4 strong split of [0, 2^40), both against their oracle fixtures, and
    every rank reporting its own timing.  Skipped on a 1-GPU box."""
    import torch
    n = min(torch.cuda.device_count(), 8)
    if n < 2:
        pytest.skip(f"{n} visible GPU(s): the RCCL launch line needs >= 2")
    line = _torchrun(n, ["--steps", "2", "--warmup", "1", "--secondary", "cfg4",
                         "--no-cpu-baseline"], {}, timeout=600)
    assert line["n_gpus"] == n and line["config"]["merge"] == "RCCL all-gather"
    assert line["result_vs_oracle"]["match"] is True, line["result_vs_oracle"]
    c4 = line["workloads"]["cfg4"]
    assert c4["result_vs_oracle"]["match"] is True, c4["result_vs_oracle"]
    assert len(line["ranks"]["local_ms"]) == n and len(c4["ranks"]["local_ms"]) == n
    # one rank per GPU: distinct ordinals and PCI addresses, each rank's own
    # shard equal to its fixture piece (n <= 8: every rank has one)
    _per_rank(line["ranks"], n, list(range(n)))
    _per_rank(c4["ranks"], n, list(range(n)))
    assert len({d["pci_bus_id"] for d in line["ranks"]["device"]}) == n
    assert line["all_ranks_match"] is True and c4["all_ranks_match"] is True
    # configs[3] again through one process driving all n GPUs: two children,
    # host merge and the in-library RCCL all-gather over distinct ordinals
    sp = line["single_process"]
    assert sp["processes_per_gpu"] == {str(g): 2 for g in range(n)}, sp
    for m, merge in (("host", "host"), ("rccl", "RCCL all-gather")):
        e = sp[m]
        assert e["devices"] == list(range(n)) and e["merge"] == merge, e
        assert e["result_vs_oracle"]["match"] is True and e["mid_call_syncs"] == 0, e


def test_bench_single_process_workload_on_one_gpu():
    """bench.py's single-process configs[3] measurement (the line's
    `single_process`, taken on multi-GPU runs) exercised on a 1-GPU box:
    HM_BENCH_SP_DEVICES=0,0 opens GPU 0 twice in the host-merge child, so the
    hm_partition shards, the per-device enqueue and the host merge of a
    2-device context run on [0, 2^40); the RCCL child gets the distinct
    ordinal 0 (a 1-rank communicator, ncclCommInitAll + ncclAllGather +
    device fold).  Both answers equal full_size.json's.  Launched as the
    driver launches bench.py (torch.distributed.run, RCCL process group at
    world size 1 via HM_BENCH_FORCE_DIST), so the host-side (gloo) wait group
    the other ranks park on is created and used too."""
    line = _torchrun(1, ["--steps", "1", "--warmup", "0", "--secondary", "cfg4",
                         "--no-cpu-baseline"],
                     {"HM_BENCH_FORCE_DIST": "1", "HM_BENCH_SP_DEVICES": "0,0"}, timeout=500)
    assert line["config"]["merge"] == "RCCL all-gather"
    sp = line["single_process"]
    assert "skipped" not in sp, sp
    # GPU 0 holds the rank's own process and the child
    assert sp["processes_per_gpu"] == {"0": 2}, sp
    for m, devs, merge in (("host", [0, 0], "host"), ("rccl", [0], "RCCL all-gather")):
        e = sp[m]  # each measured in a fresh child process
        assert "error" not in e, e
        assert e["devices"] == devs and e["merge"] == merge, e
        assert e["result_vs_oracle"]["match"] is True, e
        assert e["result"] == line["workloads"]["cfg4"]["result"]
        assert e["mid_call_syncs"] == 0 and e["value"] > 0 and e["child_s"] > 0
