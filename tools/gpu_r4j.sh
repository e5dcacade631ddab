# round 4: exact C5 with the detector beside the spectrogram (sibling context, reserved slots)
set -o pipefail
mkdir -p gpurun_out
for ov in 0 4 16 32; do
timeout -k 10 250 python bench.py --workload c5 --c5-mode exact --c5-overlap $ov --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/c5j_ov$ov.json 2> gpurun_out/c5j_ov$ov.err &&
python3 -c "
import json; d=json.loads(open('gpurun_out/c5j_ov$ov.json').read().strip().splitlines()[-1]); print('ov', $ov, d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['certification']['certified'])" || exit 1
done
