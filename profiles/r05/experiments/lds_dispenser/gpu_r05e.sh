#!/bin/bash
# Round 5: (1) fused-launch task dispensing A/B (static first task,
# prefetch, grid per CU) on small requests, after the fused GPU tests;
# (2) the workgroup-level LDS task dispenser (build/ab_var/lds, -DHM_LDS_DISPENSER)
# against the same build without it (build/ab_var/base): interleaved A/B on
# cfg2, cfg3 and d = 12, and FETCH_SIZE / WRITE_SIZE passes on cfg2 and d = 12.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r05e}
mkdir -p $O
B=build/ab_var/base/libhipminer.so; L=build/ab_var/lds/libhipminer.so
P="timeout -s KILL 90 rocprofv3 --kernel-trace"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_fused.py > $O/pytest.log 2>&1 &&
timeout -k 10 600 python -u tools/fused_ab.py 25 0,1,2,3 2,3,4 > $O/fused_ab.jsonl 2> $O/fused_ab.err &&
timeout -k 10 120 python -u tools/ab_libs.py 9 $B $L -- bradfitz 0 4294967295 > $O/lds_cfg2.txt 2>&1 &&
timeout -k 10 120 python -u tools/ab_libs.py 9 $B $L -- long120 0 4294967295 > $O/lds_cfg3.txt 2>&1 &&
timeout -k 10 200 python -u tools/ab_libs.py 7 $B $L -- bradfitz 100000000000 119999999999 > $O/lds_d12.txt 2>&1 &&
$P --pmc FETCH_SIZE -d $O/pmc/base_fetch -o run --output-format csv -- python tools/quick_scan.py --lib $B bradfitz 0 4294967295 1 > $O/pmc_bf.log 2>&1 &&
$P --pmc WRITE_SIZE -d $O/pmc/base_write -o run --output-format csv -- python tools/quick_scan.py --lib $B bradfitz 0 4294967295 1 > $O/pmc_bw.log 2>&1 &&
$P --pmc FETCH_SIZE -d $O/pmc/lds_fetch -o run --output-format csv -- python tools/quick_scan.py --lib $L bradfitz 0 4294967295 1 > $O/pmc_lf.log 2>&1 &&
$P --pmc WRITE_SIZE -d $O/pmc/lds_write -o run --output-format csv -- python tools/quick_scan.py --lib $L bradfitz 0 4294967295 1 > $O/pmc_lw.log 2>&1 &&
$P --pmc FETCH_SIZE -d $O/pmc/base_fetch_d12 -o run --output-format csv -- python tools/quick_scan.py --lib $B bradfitz 100000000000 119999999999 1 > $O/pmc_bf12.log 2>&1 &&
$P --pmc WRITE_SIZE -d $O/pmc/base_write_d12 -o run --output-format csv -- python tools/quick_scan.py --lib $B bradfitz 100000000000 119999999999 1 > $O/pmc_bw12.log 2>&1 &&
$P --pmc FETCH_SIZE -d $O/pmc/lds_fetch_d12 -o run --output-format csv -- python tools/quick_scan.py --lib $L bradfitz 100000000000 119999999999 1 > $O/pmc_lf12.log 2>&1 &&
$P --pmc WRITE_SIZE -d $O/pmc/lds_write_d12 -o run --output-format csv -- python tools/quick_scan.py --lib $L bradfitz 100000000000 119999999999 1 > $O/pmc_lw12.log 2>&1
rc=$?
tail -3 $O/pytest.log; cat $O/fused_ab.jsonl $O/lds_cfg2.txt $O/lds_cfg3.txt $O/lds_d12.txt
echo "rc=$rc"
exit $rc
