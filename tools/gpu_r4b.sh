set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_exact -o run -- python3 bench.py --workload c5 --c5-mode exact --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/pe.json 2>gpurun_out/pe.err; tail -c 600 gpurun_out/pe.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_refine -o run -- python3 bench.py --workload c5 --c5-mode refine --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/pr.json 2>gpurun_out/pr.err; tail -c 600 gpurun_out/pr.json
find gpurun_out/prof_exact gpurun_out/prof_refine -name "*stats*" | head
