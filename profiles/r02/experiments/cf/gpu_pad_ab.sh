#!/bin/bash
# GPU-box recipe: the GPU suite on the current build, then an interleaved
# one-process A/B of library variants (tools/build_pad_variants.sh) on cfg2,
# cfg4's d = 12 segment and cfg3, both orders, then the 8-rank gloo
# rehearsal of bench.py on one GPU.
# usage: tools/gpu_pad_ab.sh <outdir> <lib.so>...
set -o pipefail
export TMPDIR=/tmp
O=$1; shift; mkdir -p $O
L="$*"; R=""
for l in "$@"; do R="$l $R"; done
M3=$(python -c "import random;r=random.Random(440);print(''.join(chr(r.choice(range(0x21,0x7f))) for _ in range(120)))")
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py 7 $L > $O/ab_cfg2_fwd.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py 7 $R > $O/ab_cfg2_rev.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py 5 $L -- bradfitz 100000000000 104999999999 > $O/ab_d12_fwd.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py 5 $R -- bradfitz 100000000000 104999999999 > $O/ab_d12_rev.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py 5 $L -- "$M3" 0 4294967295 > $O/ab_cfg3_fwd.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py 5 $R -- "$M3" 0 4294967295 > $O/ab_cfg3_rev.txt 2>&1 &&
HM_BENCH_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 8 --steps 2 --warmup 1 > $O/gloo8.json 2> $O/gloo8.err &&
HM_BENCH_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29522 bench.py --gpus 8 --workload cfg4 --steps 1 --warmup 0 > $O/gloo8_cfg4.json 2> $O/gloo8_cfg4.err
rc=$?; tail -n 2 $O/pytest_gpu.log; for f in $O/ab_*.txt; do echo $f; cat $f; done; cat $O/gloo8.json $O/gloo8_cfg4.json; exit $rc
