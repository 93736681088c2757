"""Count this process's GPU user-mode queues (dev tool, GPU box) at each stage
of what one rank of the N-GPU bench line does on its GPU, from KFD's
per-process sysfs (/sys/class/kfd/kfd/proc/<pid>/queues/<qid>/{gpuid,type}):
torch's CUDA context, a torch stream, an RCCL (world-1) all-gather, a hipminer
context (streams made on first use since ABI 1.8; HM_QC_STREAMS = its
HM_OPT_STREAMS, default 2 as in bench.py), a fused and a multi-segment scan,
and after hm_close.  DESIGN §6 uses the
counts to price the processes and hardware queues per GPU of the N = 8 line.
One JSON line per stage."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

KFD = "/sys/class/kfd/kfd/proc"
# KFD names its per-process directories by HOST pid, which a container's pid
# is not: this process's directory is the one that appears when it first
# opens the GPU (the box runs nothing else of ours meanwhile)
BEFORE = set()
MINE = []


def _listing():
    try:
        return set(os.listdir(KFD))
    except OSError:
        return None


def queues():
    if not MINE:
        now = _listing()
        if now is None:
            return {"error": f"{KFD} not readable"}
        new = sorted(now - BEFORE)
        if len(new) != 1:
            return {"error": f"{len(new)} new KFD process directories", "new": new[:8]}
        MINE.append(new[0])
    d = os.path.join(KFD, MINE[0], "queues")
    try:
        qs = sorted(os.listdir(d), key=lambda s: int(s) if s.isdigit() else 0)
    except OSError as e:
        return {"error": f"{type(e).__name__}: {e}"}
    out = []
    for q in qs:
        rec = {"qid": q}
        for f in ("gpuid", "type", "size"):
            try:
                with open(os.path.join(d, q, f)) as fh:
                    rec[f] = fh.read().strip()
            except OSError:
                pass
        out.append(rec)
    return {"kfd_pid": MINE[0], "count": len(out), "queues": out}


def stage(name):
    print(json.dumps({"stage": name, **queues()}), flush=True)


def main():
    BEFORE.update(_listing() or ())
    print(json.dumps({"stage": "start", "kfd_processes": len(BEFORE)}), flush=True)
    import torch
    torch.zeros(1, device="cuda:0")
    torch.cuda.synchronize()
    stage("torch context (null stream, one kernel)")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        torch.ones(1, device="cuda:0").add_(1)
    torch.cuda.synchronize()
    stage("torch side stream")
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29517")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    out = [torch.zeros(2, dtype=torch.int64, device="cuda:0")]
    dist.all_gather(out, torch.ones(2, dtype=torch.int64, device="cuda:0"))
    torch.cuda.synchronize()
    stage("RCCL world-1 all-gather")
    from distributed_bitcoinminer_amd import _lib
    streams = int(os.environ.get("HM_QC_STREAMS", "2"))
    c = _lib.Context([0])
    c.set_option(_lib.HM_OPT_STREAMS, streams)
    stage("hm_open (ABI 1.8: stream 0 only)")
    c.scan(b"bradfitz", 0, 10**7)
    stage("hm_scan [0, 10^7] (fused launch, stream 0)")
    c.scan(b"bradfitz", 0, 2**32 - 1)
    stage(f"hm_scan [0, 2^32) with HM_OPT_STREAMS={streams}")
    c.close()
    stage("hm_close")
    dist.destroy_process_group()
    stage("destroy_process_group")


if __name__ == "__main__":
    main()
