#!/bin/bash
# GPU-box recipe (round 2, final validation): GPU suite, smoke, bench (cfg2 +
# secondary cfg3, cpu baseline), cfg4 on one GPU, the rocprofv3 kernel trace
# of the bench summarised per stream, multi-rank rehearsals, per-rank shard
# timings (predicted 1/2/4/8-GPU values) and config 1 end to end.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r02f}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python bench.py --workload cfg4 --steps 1 --warmup 0 --no-cpu-baseline > $O/bench_cfg4.json 2> $O/bench_cfg4.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-secondary > $O/trace.log 2>&1 &&
python tools/kernel_stats_by_stream.py $O/trace/run_kernel_trace.csv $O/kernel_stats_by_stream.csv &&
HM_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 > $O/gloo2.json 2> $O/gloo2.err &&
HM_BENCH_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline > $O/rccl1.json 2> $O/rccl1.err &&
timeout -k 10 300 python -u tools/rank_sweep.py --workload cfg2 --reps 3 > $O/ranks_cfg2.jsonl 2>&1 &&
timeout -k 10 300 python -u tools/rank_sweep.py --workload cfg3 --reps 3 > $O/ranks_cfg3.jsonl 2>&1 &&
timeout -k 10 400 python -u tools/rank_sweep.py --workload cfg4 --reps 1 > $O/ranks_cfg4.jsonl 2>&1 &&
timeout -k 10 300 python -u tools/e2e_cfg1.py > $O/e2e_cfg1.json 2> $O/e2e_cfg1.err
rc=$?
tail -n 3 $O/pytest_gpu.log; cat $O/smoke.log $O/bench.json $O/bench_cfg4.json
grep -h predicted $O/ranks_*.jsonl
echo "r02 final rc=$rc"
exit $rc
