#!/bin/bash
# Round-6 run b: the fused-launch changes (guided tail of the last partial
# wave-round, a large request's tail segments as one fused launch, results
# stored to pinned host memory, queue batch 16 for >= 10^11-nonce launches)
# -- their GPU tests first, then interleaved A/Bs of each option on configs
# [0]'s request, 10^6 / 10^8 nonces, the 120-B message at 10^7, cfg2 and a
# d = 12 piece of cfg4, and WRITE_SIZE of that piece with either queue batch.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r06b}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_enqueue.py tests/test_gpu_deadline.py tests/test_gpu_parity.py tests/test_gpu_checked.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_fused.log 2>&1
prc=$?
tail -3 $O/pytest_fused.log
if [ $prc -gt 1 ]; then echo "pytest rc=$prc: stopping"; exit $prc; fi
A="timeout -k 10 240 python -u tools/ab_opts.py"
$A 300 t10:FUSED_TAIL=10 t1:FUSED_TAIL=1 t2:FUSED_TAIL=2 t5:FUSED_TAIL=5 lds:FUSED_FLAGS=9 lds1:FUSED_FLAGS=9,FUSED_TAIL=1 -- bradfitz 0 10000001 > $O/ab_tail_cfg1.jsonl 2> $O/ab.err &&
$A 300 h1:HOST_RESULT=1 h0:HOST_RESULT=0 poll:DEADLINE_MS=60000 -- bradfitz 0 10000001 > $O/ab_host_cfg1.jsonl 2>> $O/ab.err &&
$A 300 t10:FUSED_TAIL=10 t1:FUSED_TAIL=1 -- long120 0 10000000 > $O/ab_tail_long120_1e7.jsonl 2>> $O/ab.err &&
$A 300 t10:FUSED_TAIL=10 t1:FUSED_TAIL=1 -- bradfitz 0 1000000 > $O/ab_tail_1e6.jsonl 2>> $O/ab.err &&
$A 60 t10:FUSED_TAIL=10 t1:FUSED_TAIL=1 -- bradfitz 0 99999999 > $O/ab_tail_1e8.jsonl 2>> $O/ab.err &&
$A 4 qa:QUEUE_BATCH=0 q4:QUEUE_BATCH=4 -- bradfitz 100000000000 299999999999 > $O/ab_queue_d12.jsonl 2>> $O/ab.err &&
$A 15 qa:QUEUE_BATCH=0 h0:HOST_RESULT=0 > $O/ab_cfg2.jsonl 2>> $O/ab.err &&
P="timeout -s KILL 90 rocprofv3 --kernel-trace" &&
$P --pmc WRITE_SIZE -d $O/pmc_write_d12_auto -o run --output-format csv -- python tools/quick_scan.py bradfitz 100000000000 299999999999 1 > $O/pmc_write_d12_auto.log 2>&1 &&
$P --pmc WRITE_SIZE -d $O/pmc_write_d12_q4 -o run --output-format csv -- python tools/quick_scan.py bradfitz 100000000000 299999999999 1 --opt QUEUE_BATCH=4 > $O/pmc_write_d12_q4.log 2>&1
rc=$?
cat $O/ab_*.jsonl | cut -c1-200
echo "final rc=$rc"
exit $rc
