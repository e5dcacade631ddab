# round 4: frame_kernel A/B (old runtime-R loop vs compile-time R with gathered tap loads)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 python3 tools/i8_time.py fkold cur fkold cur &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4p -o fk -- python3 tools/i8_time.py fkold cur > gpurun_out/r4p.log 2>&1 &&
find gpurun_out/r4p -name '*kernel_stats.csv' | head -1 | xargs grep -E 'frame_kernel|block_i8'
