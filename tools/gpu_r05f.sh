#!/bin/bash
# Round 5, validation of the round-5 tree (fused small-request launch, LDS
# task dispenser, hm_scan_cpu, single-process children): the GPU suite as the
# driver runs it, smoke(), the default bench line, rocprofv3 --stats of the
# bench with serial launches, the request-size sweep, and the PMC passes (one
# counter group per rocprofv3 run) of the cfg2 / cfg3 / d = 12 dominant
# kernels, summarised per kernel for the loaded code object (the round-5
# kernels are a new code object, so bench.py needs a new summary).
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r05f}
mkdir -p $O/cfg3 $O/cfg4
M=$(python -c "import random;r=random.Random(440);print(''.join(chr(r.choice(range(0x21,0x7f))) for _ in range(120)))")
P="timeout -s KILL 90 rocprofv3 --kernel-trace"
V="--pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
# SUITE="tests/test_gpu_smoke.py ..." runs a subset instead of the whole GPU suite
timeout -k 10 700 python -u -m pytest ${SUITE:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 120 python -u tools/queue_count.py > $O/queue_count.jsonl 2> $O/queue_count.err &&
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
timeout -k 10 300 python -u tools/fused_ab.py 15 ${FUSED_FLAGS:-1} ${FUSED_PER_CU:-3,4,6} ${FUSED_PARTS:-1,2,5} > $O/fused_parts_ab.jsonl 2> $O/fused_parts_ab.err &&
timeout -k 10 240 python -u tools/coresident.py --sweep 0,1,3,5,7,11 --streams 1 > $O/coresident_s1.jsonl 2> $O/coresident_s1.err &&
timeout -k 10 240 python -u tools/coresident.py --sweep 0,3,5,7,11 --streams 4 > $O/coresident_s4.jsonl 2> $O/coresident_s4.err
rc=$?
tail -2 $O/pytest_gpu.log; head -2 $O/serial/run_kernel_stats.csv 2>/dev/null
echo "final rc=$rc"
exit $rc
