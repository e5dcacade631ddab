# round 4, final code: the full GPU suite and smoke on one box
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4m_gpu.log 2>&1 &&
tail -3 gpurun_out/r4m_gpu.log &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
