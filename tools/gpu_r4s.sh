# round 4: block_delta2_kernel persistent grid 8 (current) / 16 / 32 / 1000 workgroups per CU, C3 A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 bash tools/ab_bench.sh 3 cur bd16 bd32 bd1000 > gpurun_out/r4s_ab.txt 2>&1 && cat gpurun_out/r4s_ab.txt
