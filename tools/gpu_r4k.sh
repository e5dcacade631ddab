# round 4: int8 delta with interleaved tiles and plain loads -- int8 tests, delta timing, exact C5 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_certify.py tests/test_gpu_stream.py tests/test_iq.py -q -x --timeout 120 --timeout-method thread -k "int8 or end_to_end or csv or overlap or detrend or ordinary" > gpurun_out/t_k.log 2>&1; tail -2 gpurun_out/t_k.log
timeout -k 10 200 python3 tools/i8_time.py cur > gpurun_out/i8_time_k.txt 2>&1; grep delta64 gpurun_out/i8_time_k.txt
timeout -k 10 250 python bench.py --workload c5 --c5-mode exact --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/c5k.json 2> gpurun_out/c5k.err &&
python3 -c "
import json; d=json.loads(open('gpurun_out/c5k.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['roofline']['frac'], d['certification']['certified'])"
