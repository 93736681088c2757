#!/bin/bash
# GPU-box recipe: per-rank shard times of the weak-scaling bench (8 ranks)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ranks; mkdir -p $O
timeout -k 10 300 python -u tools/rank_sweep.py --workload cfg2 --partition > $O/cfg2.jsonl 2>&1 &&
timeout -k 10 300 python -u tools/rank_sweep.py --workload cfg3 --partition > $O/cfg3.jsonl 2>&1
rc=$?
grep worst $O/*.jsonl
exit $rc
