#!/bin/bash
# Round-4 evidence (GPU box): the 8-rank gloo rehearsal of the driver's N=8
# bench line on GPU 0 (every rank's own answer against its fixture piece:
# ranks.match / all_ranks_match), then rocprofv3 --stats of the default cfg2
# bench with serial launches (HM_BENCH_STREAMS=1) for the kernel-time record,
# then a 240-s soak (sequential checked scans + fresh-context batches).
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r04b}
mkdir -p $O
HM_BENCH_BACKEND=gloo timeout -k 10 420 python -m torch.distributed.run --nnodes 1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 8 --steps 2 --warmup 1 --no-cpu-baseline \
  > $O/bench_gloo8.json 2> $O/bench_gloo8.err &&
HM_BENCH_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/serial -o run --output-format csv \
  -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-secondary > $O/bench_serial.json 2> $O/serial.log &&
HM_SOAK_SECONDS=240 HM_SOAK_SEED=404 timeout -k 10 500 python -u -m pytest tests/test_gpu_soak.py -x -v -s \
  --timeout 450 --timeout-method thread > $O/soak_240s_seed404.log 2>&1
rc=$?
tail -4 $O/soak_240s_seed404.log
python -c "
import json; l=json.load(open('$O/bench_gloo8.json'))
print('gloo8', l['value'], l['all_ranks_match'], l['ranks']['match'], {k: (w['all_ranks_match'], w['ranks']['match']) for k, w in l.get('workloads', {}).items()})" 2>&1
head -3 $O/serial/run_kernel_stats.csv 2>/dev/null
echo "final rc=$rc"
exit $rc
