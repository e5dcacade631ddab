# round 4: PMC passes over block_i8_kernel (exact C5 delta) -- where its time goes
set -o pipefail
mkdir -p gpurun_out
REGEX="block_i8|frame_kernel" bash tools/pmc_stft.sh r4_i8 --workload c5 --c5-mode exact --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_i8.log 2>&1; cat gpurun_out/pmc_i8.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_I8 --kernel-include-regex block_i8 -d gpurun_out/pmc/r4_i8/p5 -o pmc --output-format csv -- python3 bench.py --workload c5 --c5-mode exact --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc/r4_i8/p5.log 2>&1; echo "p5 rc=$?"
python3 tools/pmc_summary.py gpurun_out/pmc/r4_i8 > gpurun_out/pmc_i8_summary.txt 2>&1; cat gpurun_out/pmc_i8_summary.txt
WL=c5 timeout -k 10 400 bash tools/ab_bench.sh 2 cur nostore nodump
