set -o pipefail
L=meteor-scatter_amd/meteorgpu
timeout -k 10 60 tools/ubench/mfma_i8 > gpurun_out/mfma_i8.txt 2>&1; cat gpurun_out/mfma_i8.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_certify.py -q --timeout 120 --timeout-method thread -k "int8 or float64_refinement" > gpurun_out/t_i8.log 2>&1; tail -25 gpurun_out/t_i8.log
timeout -k 10 250 tools/stft_ab 6 $L/libmsdsp.so $L/libmsdsp_tabg.so $L/libmsdsp_t16.so > gpurun_out/ab_c3_tabg.txt 2>&1; tail -6 gpurun_out/ab_c3_tabg.txt
STFT_AB_MODE=c5 timeout -k 10 200 tools/stft_ab 6 $L/libmsdsp.so $L/libmsdsp_tw2g.so > gpurun_out/ab_c5_tw2g.txt 2>&1; tail -6 gpurun_out/ab_c5_tw2g.txt
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1; tail -15 gpurun_out/gputest.log
timeout -k 10 250 python bench.py --workload c5 --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/c5.json 2> gpurun_out/c5.err; tail -c 3000 gpurun_out/c5.json; tail -5 gpurun_out/c5.err
