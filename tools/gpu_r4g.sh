# round 4: cstft post-FFT detrend (PD) -- parity tests, then the C5 kernel A/B against the round-start kernel
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_iq.py tests/test_gpu_certify.py tests/test_gpu_stream.py -q -x --timeout 120 --timeout-method thread > gpurun_out/t_pd.log 2>&1; tail -4 gpurun_out/t_pd.log
STFT_AB_MODE=c5 timeout -k 10 300 tools/stft_ab 8 meteor-scatter_amd/meteorgpu/libmsdsp_base.so meteor-scatter_amd/meteorgpu/libmsdsp.so > gpurun_out/ab_pd2.txt 2>&1; tail -6 gpurun_out/ab_pd2.txt
STFT_AB_MODE=c5 STFT_AB_ENERGY=1,1 timeout -k 10 300 tools/stft_ab 4 meteor-scatter_amd/meteorgpu/libmsdsp_base.so meteor-scatter_amd/meteorgpu/libmsdsp.so > gpurun_out/ab_pd2e.txt 2>&1; tail -3 gpurun_out/ab_pd2e.txt
