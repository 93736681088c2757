#!/bin/bash
# PMC passes for the chained kernel on the cfg3 message (run under gpurun).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r01_cfg3pmc
mkdir -p $O
M=$(python -c "import random;r=random.Random(440);print(''.join(chr(r.choice(range(0x21,0x7f))) for _ in range(120)))")
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/pmc_valu -o run --output-format csv -- python tools/quick_scan.py "$M" 0 4294967295 1 > $O/pmc_valu.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python tools/quick_scan.py "$M" 0 4294967295 1 > $O/pmc_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python tools/quick_scan.py "$M" 0 4294967295 1 > $O/pmc_write.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
