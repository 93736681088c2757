#!/bin/bash
# Round-6 first GPU run: the whole GPU suite on the ABI-1.8 tree (deadline /
# HM_ERR_TIMEOUT, streams made on first use, retired tables kept to hm_close),
# smoke(), the per-process queue count with HM_OPT_STREAMS = 2, the
# interleaved A/B of 2 vs 4 streams (cfg2, cfg3, a d = 12 piece of cfg4) and
# the default bench line.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r06a}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
prc=$?
tail -3 $O/pytest_gpu.log
# test failures (rc 1) still let the measurements run; a time limit, abort
# or crash ends the call here
if [ $prc -gt 1 ]; then echo "pytest rc=$prc: stopping"; exit $prc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 120 python -u tools/queue_count.py > $O/queue_count.jsonl 2> $O/queue_count.err &&
timeout -k 10 200 python -u tools/ab_opts.py 15 s4:STREAMS=4 s2:STREAMS=2 > $O/ab_streams_cfg2.jsonl 2> $O/ab.err &&
timeout -k 10 200 python -u tools/ab_opts.py 15 s4:STREAMS=4 s2:STREAMS=2 -- long120 0 4294967295 > $O/ab_streams_cfg3.jsonl 2>> $O/ab.err &&
timeout -k 10 200 python -u tools/ab_opts.py 6 s4:STREAMS=4 s2:STREAMS=2 -- bradfitz 0 137438953471 > $O/ab_streams_cfg4_shard0of8.jsonl 2>> $O/ab.err &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?
tail -3 $O/pytest_gpu.log; tail -2 $O/smoke.log; cat $O/ab_streams_*.jsonl; head -c 600 $O/bench.json
echo "final rc=$rc"
exit $rc
