#!/bin/bash
# Round-6 final validation, part 2 (GPU box, same tree as part 1): request
# sizes, config 1 end to end through LSP, the torchrun world-1 RCCL bench
# line with its queue record, the fused-tail A/B on the small sizes, and a
# 180-s randomised soak through hm_scan_checked / hm_scan_many.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r06final2}
mkdir -p $O
timeout -k 10 200 python -u tools/request_sizes.py > $O/request_sizes.jsonl 2> $O/request_sizes.err &&
timeout -k 10 120 python -u tools/e2e_cfg1.py > $O/e2e_cfg1.json 2> $O/e2e_cfg1.err &&
HM_BENCH_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline \
  --no-secondary > $O/bench_rccl_world1.json 2> $O/bench_rccl_world1.err &&
timeout -k 10 240 python -u tools/ab_opts.py 300 t2:FUSED_TAIL=2 t1:FUSED_TAIL=1 t10:FUSED_TAIL=10 -- bradfitz 0 10000001 > $O/ab_tail_cfg1.jsonl 2> $O/ab.err &&
timeout -k 10 240 python -u tools/ab_opts.py 300 t2:FUSED_TAIL=2 t1:FUSED_TAIL=1 t10:FUSED_TAIL=10 -- long120 0 10000000 > $O/ab_tail_long120_1e7.jsonl 2>> $O/ab.err &&
timeout -k 10 240 python -u tools/ab_opts.py 300 t2:FUSED_TAIL=2 t1:FUSED_TAIL=1 t10:FUSED_TAIL=10 -- bradfitz 0 1000000 > $O/ab_tail_1e6.jsonl 2>> $O/ab.err &&
HM_SOAK_SECONDS=180 HM_SOAK_SEED=606 timeout -k 10 360 python -u -m pytest tests/test_gpu_soak.py -m gpu -x -v -s --timeout 340 --timeout-method thread > $O/soak_180s_seed606.log 2>&1
rc=$?
cat $O/request_sizes.jsonl | cut -c1-150; cat $O/ab_*.jsonl | cut -c1-180; tail -3 $O/soak_180s_seed606.log
echo "final rc=$rc"
exit $rc
