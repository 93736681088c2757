#!/bin/bash
# GPU-box rehearsals of the multi-rank bench path (the driver runs N=2..8 on
# an 8-GPU node): 2 gloo ranks sharing GPU 0, and RCCL at world size 1.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/dist; mkdir -p $O
HM_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 > $O/gloo2.json 2> $O/gloo2.err &&
HM_BENCH_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline > $O/rccl1.json 2> $O/rccl1.err
rc=$?; cat $O/gloo2.json $O/rccl1.json; tail -3 $O/gloo2.err $O/rccl1.err; exit $rc
