set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_certify.py tests/test_gpu_stream.py -q --timeout 120 --timeout-method thread -k "int8 or float64_refinement or end_to_end or ordinary or csv" > gpurun_out/t_i8b.log 2>&1; tail -6 gpurun_out/t_i8b.log
timeout -k 10 250 python bench.py --workload c5 --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/c5b.json 2> gpurun_out/c5b.err; tail -c 2600 gpurun_out/c5b.json; tail -3 gpurun_out/c5b.err
