# round 4: the refine planner without N cosines per call -- C5 tests and two exact-mode benches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_iq.py tests/test_gpu_stream.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4r_gpu.log 2>&1 &&
tail -2 gpurun_out/r4r_gpu.log &&
for r in 1 2; do
timeout -k 10 250 python bench.py --workload c5 --c5-mode exact --steps 20 --warmup 10 --no-cpu-baseline > gpurun_out/r4r_c5_$r.json 2> gpurun_out/r4r_c5_$r.err &&
python3 -c "
import json; d=json.loads(open('gpurun_out/r4r_c5_$r.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernel_ms_per_step'], d['certification']['certified'])" || exit 1
done
