# round 4: the C5 detector's segment length (one scan wave per segment) on the exact path
set -o pipefail
mkdir -p gpurun_out
for sl in 8192 4096 2048 1024; do
MSD_BENCH_SEG_LEN=$sl timeout -k 10 250 python bench.py --workload c5 --c5-mode exact --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/c5l_$sl.json 2> gpurun_out/c5l_$sl.err &&
python3 -c "
import json; d=json.loads(open('gpurun_out/c5l_$sl.json').read().strip().splitlines()[-1]); print('seg', $sl, d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['certification']['certified'], d['state_rounds'], d['detections_per_step'])" || exit 1
done
