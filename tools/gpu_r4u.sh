# round 4: dc_fix_kernel with non-temporal stores vs plain, C5 exact A/B
set -o pipefail
mkdir -p gpurun_out
WL=c5 timeout -k 10 900 bash tools/ab_bench.sh 3 cur dcnt > gpurun_out/r4u_ab.txt 2>&1 && cat gpurun_out/r4u_ab.txt
