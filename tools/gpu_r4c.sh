set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_certify.py tests/test_gpu_stream.py -q --timeout 120 --timeout-method thread -k "int8 or float64_refinement or end_to_end or ordinary or csv or overlap" > gpurun_out/t_i8b.log 2>&1; tail -6 gpurun_out/t_i8b.log
for ov in 0 16 48; do
timeout -k 10 250 python bench.py --workload c5 --c5-mode exact --c5-overlap $ov --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/c5_ov$ov.json 2> gpurun_out/c5_ov$ov.err; python3 -c "
import json,sys; d=json.loads(open('gpurun_out/c5_ov$ov.json').read().strip().splitlines()[-1]); print('ov', $ov, d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['certification']['certified'], d.get('exact_delta'))"
done
