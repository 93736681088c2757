#!/bin/bash
# Round 6 rehearsal of the driver's N = 8 launch line on one GPU (8 gloo ranks
# sharing GPU 0; HM_BENCH_SP_DEVICES=0 so rank 0 also runs the two
# single-process children while ranks 1..7 park in the host-side wait
# group): the line's per-rank checks, queue records and children on the
# round-6 tree (2 streams per context, tail segments fused).
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r06g}
mkdir -p $O
HM_BENCH_BACKEND=gloo HM_BENCH_SP_DEVICES=0 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --steps 3 --warmup 1 \
  > $O/bench_gloo8_sp.json 2> $O/bench_gloo8_sp.err
rc=$?
cut -c1-600 $O/bench_gloo8_sp.json
echo "rc=$rc"
exit $rc
