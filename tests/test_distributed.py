"""N>1 path on CPU: world_size-2, 3 and 8 gloo ranks shard the range and all-gather the
16-byte candidates; the merged answer equals the single-range scan.  The GPU
scan is replaced by the CPU oracle here (test double)."""
import os
import socket

import pytest
import torch.multiprocessing as mp

from distributed_bitcoinminer_amd import parallel

MAX = (1 << 64) - 1
CASES = [(b"bradfitz", 0, 9999), (b"jonny greenwood", 200, 71010), (b"x", 5, 4),
         (b"bradfitz", MAX - 3000, MAX), (b"q", 7, 7), (b"q", 7, 8)]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from oracle import oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = []
    for msg, lo, hi in CASES:
        out.append(parallel.distributed_scan(
            msg, lo, hi, lambda m, a, b: oracle.c_scan(m, a, b, threads=1)))
    dist.destroy_process_group()
    q.put((rank, out))


@pytest.mark.parametrize("world", [2, 3, 8])
def test_gloo_distributed_scan(oracle_mod, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = [oracle_mod.c_scan(m, lo, hi, threads=2) for m, lo, hi in CASES]
    for r in range(world):
        assert results[r] == expect


def test_shard_range_partitions():
    for lo, hi in [(0, 0), (0, 9), (3, 100), (0, MAX), (MAX - 2, MAX), (10, 12)]:
        for world in (1, 2, 3, 8):
            shards = [parallel.shard_range(lo, hi, world, r) for r in range(world)]
            got = [s for s in shards if s is not None]
            assert got[0][0] == lo and got[-1][1] == hi
            for a, b in zip(got, got[1:]):
                assert b[0] == a[1] + 1
            sizes = [b - a + 1 for a, b in got]
            assert max(sizes) - min(sizes) <= 1
    assert parallel.shard_range(5, 4, 2, 0) is None


def test_merge_lexicographic():
    assert parallel.merge([]) == (MAX, 0)
    assert parallel.merge([(3, 9), (3, 2), (4, 0)]) == (3, 2)
    assert parallel.merge([(MAX, 5)]) == (MAX, 0)
