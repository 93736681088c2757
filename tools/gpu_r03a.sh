set -o pipefail
mkdir -p gpurun_out/r03a
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_dist.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r03a/pytest.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r03a/bench.json 2> gpurun_out/r03a/bench.err
rc=$?; tail -5 gpurun_out/r03a/pytest.log; cat gpurun_out/r03a/bench.json | head -c 3000; exit $rc
