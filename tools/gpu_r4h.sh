# round 4: C5 detrend from the exact delta's frame sums -- parity tests, exact C5 bench, trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_iq.py tests/test_gpu_certify.py tests/test_gpu_stream.py -q -x --timeout 120 --timeout-method thread > gpurun_out/t_fs.log 2>&1; tail -3 gpurun_out/t_fs.log
timeout -k 10 250 python bench.py --workload c5 --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/c5_fs.json 2> gpurun_out/c5_fs.err &&
python3 -c "
import json; d=json.loads(open('gpurun_out/c5_fs.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['roofline']['frac'], d['certification']['certified'], {m: (v['ms_per_step'], v.get('same_detections')) for m, v in d.get('modes', {}).items()})"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5f -o c5f -- python3 bench.py --workload c5 --c5-mode exact --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/prof_c5f.log 2>&1 &&
python3 tools/trace_gaps.py gpurun_out/prof_c5f > gpurun_out/c5f_gaps.txt 2>&1; head -12 gpurun_out/c5f_gaps.txt; tail -3 gpurun_out/c5f_gaps.txt
