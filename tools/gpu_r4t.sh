# round 4, last code: the full GPU suite, smoke and the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4t_gpu.log 2>&1 &&
tail -2 gpurun_out/r4t_gpu.log &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" &&
timeout -k 10 400 python bench.py > gpurun_out/r4t_bench.json 2> gpurun_out/r4t_bench.err &&
python3 -c "
import json; b=json.loads(open('gpurun_out/r4t_bench.json').read().strip().splitlines()[-1]); c=b['c5']
print(b['value'], b['ms_per_step'], b['roofline']['frac'], b['kernel_ms_per_step'], c['value'], c['ms_per_step'], c['roofline']['frac'], c['certification']['certified'])"
