"""Scan rate against the number of idle processes holding GPU queues on the
same GPU (dev tool, GPU box; DESIGN §6 "Processes and hardware queues per
GPU").  The round-4 rehearsal put 8 bench ranks on ONE GPU and saw the
single-process scan drop from 37.6 to 26.2 GH/s; this pins the mechanism.

For P in the sweep, P idle child processes each initialise torch on GPU 0
and run one kernel on `--streams` torch streams (so each holds that many
user-mode queues, counted from KFD's sysfs), then wait.  Meanwhile this
process (no torch) runs hm_scan of bradfitz [0, 2^32) 3 times and reports
the median wall and kernel GH/s, and the queue counts of itself and of the
idle processes.  At most 1 + max(P) processes touch the GPU (keep <= 15).
usage: python tools/coresident.py [--sweep 0,1,3,5,7,11] [--streams 1]"""
import argparse
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

IDLE = r"""
import os, sys, torch
n = int(sys.argv[1])
torch.zeros(1, device="cuda:0")
ss = [torch.cuda.Stream() for _ in range(n - 1)]
for s in ss:
    with torch.cuda.stream(s):
        torch.ones(1, device="cuda:0").add_(1)
torch.cuda.synchronize()
q = f"/sys/class/kfd/kfd/proc/{os.getpid()}/queues"
try:
    nq = len(os.listdir(q))
except OSError:
    nq = -1
print(nq, flush=True)
sys.stdin.read()
"""


def kfd_queues(pid):
    try:
        return len(os.listdir(f"/sys/class/kfd/kfd/proc/{pid}/queues"))
    except OSError:
        return -1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sweep", default="0,1,3,5,7,11")
    ap.add_argument("--streams", type=int, default=1)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    sweep = [int(x) for x in a.sweep.split(",")]
    assert max(sweep) <= 14, "at most 15 processes on the GPU"
    from distributed_bitcoinminer_amd import _lib
    c = _lib.Context([0])
    m, hi = b"bradfitz", (1 << 32) - 1
    c.scan(m, 0, 10**8)
    for p in sweep:
        kids = []
        try:
            for _ in range(p):
                kids.append(subprocess.Popen([sys.executable, "-c", IDLE, str(a.streams)],
                                             stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                             text=True))
            idle_q = [int(k.stdout.readline().strip() or -1) for k in kids]
            walls, kern = [], []
            for _ in range(a.reps):
                t = time.perf_counter()
                res = c.scan(m, 0, hi)
                walls.append(time.perf_counter() - t)
                kern.append(c.stats()["kernel_ms"])
                assert res == (5256245051, 1626825724), res
            w, k = statistics.median(walls), statistics.median(kern)
            print(json.dumps({"idle_processes": p, "streams_per_idle": a.streams,
                              "idle_queues": idle_q, "scanner_queues": kfd_queues(os.getpid()),
                              "processes_on_gpu": p + 1,
                              "wall_GHs": round((hi + 1) / w / 1e9, 3),
                              "kernel_GHs": round((hi + 1) / k / 1e6, 3)}), flush=True)
        finally:
            for k in kids:
                try:
                    k.stdin.close()
                except OSError:
                    pass
            for k in kids:
                try:
                    k.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    k.kill()
                    k.wait()
    c.close()


if __name__ == "__main__":
    main()
