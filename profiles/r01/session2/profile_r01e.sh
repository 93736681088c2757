#!/bin/bash
# GPU-box recipe (round 1, session 2, after guided tasks): smoke, bench and
# kernel trace of cfg2; per-dispatch trace kept for the tail analysis.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r01e
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1
rc=$?
cat $O/smoke.log $O/bench.json
echo "profile rc=$rc"
exit $rc
