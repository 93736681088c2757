#!/bin/bash
# Round 5, first call: where configs[0]'s small request spends its time
# (tools/small_req_diag.py, a kernel trace of the request), the request-size
# curve of the round-4 build, and the KFD scheduler parameters that bound how
# many processes share a GPU's hardware queues.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r05a}
mkdir -p $O
for p in hws_max_conc_proc sched_policy mes; do
  printf '%s=' $p >> $O/kfd_params.txt
  cat /sys/module/amdgpu/parameters/$p >> $O/kfd_params.txt 2>/dev/null || echo '?' >> $O/kfd_params.txt
done
timeout -k 10 240 python -u tools/small_req_diag.py 15 > $O/diag.jsonl 2> $O/diag.err &&
timeout -k 10 240 python -u tools/request_sizes.py > $O/request_sizes.jsonl 2> $O/rs.err &&
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv \
  -- python tools/quick_scan.py bradfitz 0 10000001 8 > $O/trace.txt 2>&1
rc=$?
cat $O/kfd_params.txt; cat $O/diag.jsonl | cut -c1-200
echo "rc=$rc"
exit $rc
