set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/lat4; mkdir -p $O
timeout -k 10 120 python tools/quick_scan.py bradfitz 0 10000001 20 > $O/q.txt 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python tools/quick_scan.py bradfitz 0 10000001 5 > $O/t.txt 2>&1 &&
timeout -k 10 300 python -u tools/e2e_cfg1.py > $O/e2e_cfg1.json 2> $O/e2e_cfg1.err &&
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "scan_many or golden or random or layout_sweep_segment or miner" > $O/pytest_gpu.log 2>&1
rc=$?; tail -n 1 $O/pytest_gpu.log; cat $O/e2e_cfg1.json; exit $rc
