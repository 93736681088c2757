set -o pipefail
mkdir -p gpurun_out/r04i
HM_BENCH_SP_DEVICES=0 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --secondary cfg4 --no-cpu-baseline > gpurun_out/r04i/plain_sp0.json 2> gpurun_out/r04i/plain_sp0.err &&
HM_BENCH_SP_DEVICES=0,0 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --secondary cfg4 --no-cpu-baseline > gpurun_out/r04i/plain_sp00.json 2> gpurun_out/r04i/plain_sp00.err
rc=$?
for f in gpurun_out/r04i/*.json; do python -c "
import json,sys; l=json.load(open('$f')); w=l['workloads']['cfg4']; s=l['single_process']; print('$f', 'cfg4', w['value'], 'sp', s.get('value'), s.get('wall_ms'), s.get('kernel_GHs_per_device'), s.get('merge'))"; done
exit $rc
