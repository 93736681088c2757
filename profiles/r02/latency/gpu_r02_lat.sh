#!/bin/bash
# GPU-box recipe: small-request latency (config 1's miner Request through
# hm_scan, and end to end through hm_miner + LSP), its kernel trace, the
# cfg2 bench line, and the GPU suite.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/lat2}; mkdir -p $O
timeout -k 10 120 python tools/quick_scan.py bradfitz 0 10000001 20 > $O/q.txt 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python tools/quick_scan.py bradfitz 0 10000001 5 > $O/t.txt 2>&1 &&
timeout -k 10 300 python -u tools/e2e_cfg1.py > $O/e2e_cfg1.json 2> $O/e2e_cfg1.err &&
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -n 1 $O/pytest_gpu.log; cat $O/e2e_cfg1.json; echo "lat rc=$rc"; exit $rc
