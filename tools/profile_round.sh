#!/bin/bash
# One round's measurements on the GPU box: the default bench line, rocprofv3 kernel-trace
# summaries of short runs of every workload, and the PMC passes over the headline STFT
# (tools/pmc_stft.sh).  Usage: tools/profile_round.sh TAG
set -u
TAG=${1:-r1}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/round_$TAG
# kernel-trace runs: timed steps after a warm-up long enough for the shader clock to settle
# (the first ~5 dispatches of a fresh process run while it ramps)
KS=${KT_STEPS:-10}; KW=${KT_WARMUP:-10}
mkdir -p "$OUT"
# STAGE=kt: the bench line and the kernel traces; STAGE=pmc: the PMC passes; default both (two calls
# fit gpurun's per-call limit better than one)
STAGE=${STAGE:-all}
if [ "$STAGE" != pmc ]; then
timeout -k 10 400 python3 "$ROOT/bench.py" > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- \
    python3 "$ROOT/bench.py" --steps $KS --warmup $KW --no-cpu-baseline --no-c5 --no-live > "$OUT/kt.log" 2>&1 || exit 1
for wl in live c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_$wl" -o kt -- \
      python3 "$ROOT/bench.py" --workload $wl --steps $KS --warmup $KW --no-cpu-baseline --c5-mode off > "$OUT/kt_$wl.log" 2>&1 || exit 1
done
# the certified C5 path (round 3): exact decisions, the float64 refinement kernels in the trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_c5x" -o kt -- \
    python3 "$ROOT/bench.py" --workload c5 --steps $KS --warmup $KW --no-cpu-baseline --c5-mode exact > "$OUT/kt_c5x.log" 2>&1 || exit 1
fi
[ "$STAGE" = kt ] && exit 0
cd /tmp && export TMPDIR=/tmp
bash "$ROOT/tools/pmc_stft.sh" "$TAG" || exit 1
REGEX=cstft bash "$ROOT/tools/pmc_stft.sh" "${TAG}_c5" --workload c5 --steps 2 --warmup 1 --no-cpu-baseline --c5-mode exact
REGEX="block_i8|frame_kernel" bash "$ROOT/tools/pmc_stft.sh" "${TAG}_c5i8" --workload c5 --steps 2 --warmup 1 --no-cpu-baseline --c5-mode exact
REGEX="fresh_list_kernel|scan_kernel|approx_kernel|iq_band_delta" bash "$ROOT/tools/pmc_stft.sh" "${TAG}_c5det" --workload c5 --steps 1 --warmup 0 --no-cpu-baseline --c5-mode off
