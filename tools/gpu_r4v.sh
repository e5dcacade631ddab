# round 4: frame_kernel occupancy (launch bounds 6 / 8 workgroups per CU) vs current, exact delta step
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 tools/i8_time.py cur fk6 fk8 cur fk6 fk8 > gpurun_out/r4v.txt 2>&1 && cat gpurun_out/r4v.txt
