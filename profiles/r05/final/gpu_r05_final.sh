#!/bin/bash
# Round-5 final validation (GPU box), after the last kernel change: the GPU
# suite as the driver runs it, smoke(), the PMC passes of the cfg2 / cfg3 /
# d = 12 dominant kernels summarised for the loaded code object (copied to
# profiles/r05/pmc_summary.json on the box so the bench line's `traffic`
# uses it), the default bench line, rocprofv3 --stats of the bench with
# serial launches, the request-size sweep, config 1 end to end, and a 180-s
# randomised soak through hm_scan_checked / hm_scan_many.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r05final}
mkdir -p $O/cfg3 $O/cfg4
M=$(python -c "import random;r=random.Random(440);print(''.join(chr(r.choice(range(0x21,0x7f))) for _ in range(120)))")
P="timeout -s KILL 90 rocprofv3 --kernel-trace"
V="--pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
$P $V -d $O/pmc_valu -o run --output-format csv -- python tools/quick_scan.py bradfitz 0 4294967295 1 > $O/pmc_valu.log 2>&1 &&
$P --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python tools/quick_scan.py bradfitz 0 4294967295 1 > $O/pmc_fetch.log 2>&1 &&
$P --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python tools/quick_scan.py bradfitz 0 4294967295 1 > $O/pmc_write.log 2>&1 &&
$P $V -d $O/cfg3/pmc_valu -o run --output-format csv -- python tools/quick_scan.py "$M" 0 4294967295 1 > $O/cfg3/pmc_valu.log 2>&1 &&
$P --pmc FETCH_SIZE -d $O/cfg3/pmc_fetch -o run --output-format csv -- python tools/quick_scan.py "$M" 0 4294967295 1 > $O/cfg3/pmc_fetch.log 2>&1 &&
$P --pmc WRITE_SIZE -d $O/cfg3/pmc_write -o run --output-format csv -- python tools/quick_scan.py "$M" 0 4294967295 1 > $O/cfg3/pmc_write.log 2>&1 &&
$P $V -d $O/cfg4/pmc_valu -o run --output-format csv -- python tools/quick_scan.py bradfitz 100000000000 119999999999 1 > $O/cfg4/pmc_valu.log 2>&1 &&
$P --pmc FETCH_SIZE -d $O/cfg4/pmc_fetch -o run --output-format csv -- python tools/quick_scan.py bradfitz 100000000000 119999999999 1 > $O/cfg4/pmc_fetch.log 2>&1 &&
$P --pmc WRITE_SIZE -d $O/cfg4/pmc_write -o run --output-format csv -- python tools/quick_scan.py bradfitz 100000000000 119999999999 1 > $O/cfg4/pmc_write.log 2>&1 &&
python tools/summarize_profile.py $O $O/summary > /dev/null &&
python tools/summarize_profile.py $O/cfg3 $O/summary > /dev/null &&
python tools/summarize_profile.py $O/cfg4 $O/summary > /dev/null &&
mkdir -p profiles/r05 && cp $O/summary/pmc_summary.json profiles/r05/pmc_summary.json &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
HM_BENCH_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/serial -o run --output-format csv \
  -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-secondary > $O/bench_serial.json 2> $O/serial.log &&
timeout -k 10 200 python -u tools/request_sizes.py > $O/request_sizes.jsonl 2> $O/request_sizes.err &&
timeout -k 10 120 python -u tools/e2e_cfg1.py > $O/e2e_cfg1.json 2> $O/e2e_cfg1.err &&
HM_SOAK_SECONDS=180 HM_SOAK_SEED=505 timeout -k 10 360 python -u -m pytest tests/test_gpu_soak.py -m gpu -x -v -s --timeout 340 --timeout-method thread > $O/soak_180s_seed505.log 2>&1
rc=$?
tail -2 $O/pytest_gpu.log; head -2 $O/serial/run_kernel_stats.csv 2>/dev/null; tail -3 $O/soak_180s_seed505.log
echo "final rc=$rc"
exit $rc
