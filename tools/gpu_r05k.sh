#!/bin/bash
# Round 5, last check of the final tree (host-side changes only after
# gpu_r05_final.sh: hm_miner's test hook, hm_scan_cpu's default threads; the
# scan code object is unchanged): the GPU suite as the driver runs it,
# smoke(), and the default bench line.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r05k}
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?
tail -2 $O/pytest_gpu.log; cut -c1-300 $O/bench.json
echo "rc=$rc"
exit $rc
