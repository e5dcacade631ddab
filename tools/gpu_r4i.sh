# round 4: the driver's round-end checks -- full GPU suite, smoke, default bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1; tail -3 gpurun_out/t_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1; tail -2 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench_r4i.json 2> gpurun_out/bench_r4i.err; python3 -c "
import json; d=json.loads(open('gpurun_out/bench_r4i.json').read().strip().splitlines()[-1]); c=d.get('c5',{}); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value']); print('c5', c.get('value'), c.get('ms_per_step'), c.get('roofline',{}).get('frac'), c.get('certification',{}).get('certified'))"
