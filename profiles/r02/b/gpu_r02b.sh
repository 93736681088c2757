set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02b; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "medium or stats or rccl" > $O/pytest_gpu.log 2>&1 &&
HM_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 > $O/gloo2.json 2> $O/gloo2.err &&
HM_BENCH_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline > $O/rccl1.json 2> $O/rccl1.err &&
timeout -k 10 300 python -u tools/rank_sweep.py --workload cfg2 --reps 3 > $O/ranks_cfg2.jsonl 2>&1 &&
timeout -k 10 300 python -u tools/rank_sweep.py --workload cfg3 --reps 3 > $O/ranks_cfg3.jsonl 2>&1
rc=$?
tail -n 3 $O/pytest_gpu.log; grep -h predicted $O/ranks_*.jsonl; echo rc=$rc; exit $rc
