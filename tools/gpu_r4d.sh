# round 4: the 4-block-tile int8 delta kernel -- int8 parity tests, then the exact C5 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_certify.py tests/test_gpu_stream.py -q --timeout 120 --timeout-method thread -k "int8 or float64_refinement or end_to_end or ordinary or csv or overlap" > gpurun_out/t_i8d.log 2>&1 && tail -4 gpurun_out/t_i8d.log &&
timeout -k 10 250 python bench.py --workload c5 --c5-mode exact --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/c5_d.json 2> gpurun_out/c5_d.err &&
python3 -c "
import json; d=json.loads(open('gpurun_out/c5_d.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['certification']['certified'], d['certification'].get('same_detections'), d.get('exact_delta'))"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5d -o c5d -- python3 bench.py --workload c5 --c5-mode exact --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/prof_c5d.log 2>&1 &&
python3 tools/trace_gaps.py gpurun_out/prof_c5d > gpurun_out/c5d_gaps.txt 2>&1; tail -25 gpurun_out/c5d_gaps.txt
