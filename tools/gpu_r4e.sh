# round 4: int8 delta with 64-B row loads + host interval fast path -- tests, exact C5 bench (overlap 0 / 16), trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_certify.py tests/test_gpu_stream.py -q --timeout 120 --timeout-method thread -k "int8 or float64_refinement or end_to_end or ordinary or csv or overlap" > gpurun_out/t_i8e.log 2>&1 && tail -3 gpurun_out/t_i8e.log &&
for ov in 0 16; do
timeout -k 10 250 python bench.py --workload c5 --c5-mode exact --c5-overlap $ov --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/c5e_ov$ov.json 2> gpurun_out/c5e_ov$ov.err &&
python3 -c "
import json; d=json.loads(open('gpurun_out/c5e_ov$ov.json').read().strip().splitlines()[-1]); print('ov', $ov, d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['certification']['certified'], d.get('exact_delta'))" || exit 1
done &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5e -o c5e -- python3 bench.py --workload c5 --c5-mode exact --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/prof_c5e.log 2>&1 &&
python3 tools/trace_gaps.py gpurun_out/prof_c5e > gpurun_out/c5e_gaps.txt 2>&1; head -8 gpurun_out/c5e_gaps.txt; tail -22 gpurun_out/c5e_gaps.txt
