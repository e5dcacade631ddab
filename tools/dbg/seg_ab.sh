#!/bin/bash
# Debug (GPU box): C5 bench step time against the stream detector's scan segment length
# (MSD_BENCH_SEG_LEN; 8192 is the default and measured fastest in total step time).
set -e
for i in 1 2; do for sl in 8192 4096 2048 1024; do
MSD_BENCH_SEG_LEN=$sl timeout -k 10 200 python3 bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/seg_${sl}_$i.log 2>&1
python3 -c "
import json,sys; d=json.loads(open('gpurun_out/seg_${sl}_$i.log').read().strip().splitlines()[-1]); print($sl, d['ms_per_step'], d['kernel_ms_per_step'], d['state_rounds'], d['exact_threshold_frames'])"
done; done
