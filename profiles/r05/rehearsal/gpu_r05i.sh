#!/bin/bash
# Round 5 rehearsal of the driver's N = 8 launch line on one GPU (8 gloo ranks
# sharing GPU 0; HM_BENCH_SP_DEVICES=0 so rank 0 also runs the two
# single-process children while ranks 1..7 park in the host-side wait group),
# then a longer randomised soak of the final build.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r05i}
mkdir -p $O
HM_BENCH_BACKEND=gloo HM_BENCH_SP_DEVICES=0 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --steps 3 --warmup 1 \
  > $O/bench_gloo8_sp.json 2> $O/bench_gloo8_sp.err &&
HM_SOAK_SECONDS=${SOAK:-400} HM_SOAK_SEED=5050 timeout -k 10 900 python -u -m pytest tests/test_gpu_soak.py -m gpu -x -v -s \
  --timeout 800 --timeout-method thread > $O/soak_${SOAK:-400}s_seed5050.log 2>&1
rc=$?
cut -c1-400 $O/bench_gloo8_sp.json; tail -3 $O/soak_*.log
echo "rc=$rc"
exit $rc
