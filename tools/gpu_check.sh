set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/s2/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/s2/bench.json 2> gpurun_out/s2/bench.err
rc=$?
tail -5 gpurun_out/s2/pytest_gpu.log; cat gpurun_out/s2/bench.json; exit $rc
