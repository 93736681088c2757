set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r01d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python tools/wall_sweep.py > $O/wall_sweep.txt 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?
tail -3 $O/pytest_gpu.log; cat $O/wall_sweep.txt $O/bench.json; exit $rc
