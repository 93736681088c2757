#!/bin/bash
# GPU-box recipe (round 2, after a kernel change): PMC passes of the new
# build (tools/profile_r02.sh), summarised on the box into
# profiles/r02/pmc_summary.json (merged with the committed entries; copied
# back under $O/summ), then smoke, bench (cfg2 + secondary cfg3, cpu
# baseline), cfg4 on one GPU, the RCCL world-1 rehearsal and the per-rank
# shard timings.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r02pf}; mkdir -p $O/summ
cp profiles/r02/pmc_summary.json $O/summ/pmc_summary.json
bash tools/profile_r02.sh $O/prof > $O/profile.log 2>&1 &&
python tools/summarize_profile.py $O/prof $O/summ > /dev/null &&
python tools/summarize_profile.py $O/prof/cfg3 $O/summ > /dev/null &&
python tools/summarize_profile.py $O/prof/cfg4 $O/summ > /dev/null &&
cp $O/summ/pmc_summary.json profiles/r02/pmc_summary.json &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python bench.py --workload cfg4 --steps 1 --warmup 0 --no-cpu-baseline > $O/bench_cfg4.json 2> $O/bench_cfg4.err &&
HM_BENCH_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline > $O/rccl1.json 2> $O/rccl1.err &&
timeout -k 10 300 python -u tools/rank_sweep.py --workload cfg2 --reps 3 > $O/ranks_cfg2.jsonl 2>&1 &&
timeout -k 10 300 python -u tools/rank_sweep.py --workload cfg3 --reps 3 > $O/ranks_cfg3.jsonl 2>&1 &&
timeout -k 10 400 python -u tools/rank_sweep.py --workload cfg4 --reps 1 > $O/ranks_cfg4.jsonl 2>&1
rc=$?
tail -n 2 $O/profile.log; cat $O/smoke.log $O/bench.json $O/bench_cfg4.json
grep -h predicted $O/ranks_*.jsonl
echo "r02 pmc+final rc=$rc"
exit $rc
