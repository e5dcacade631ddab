#!/bin/bash
# Alternate bench runs between in-tree library variants (GPU box).
# Usage: [WL=c3|live|c5] [AB_ARGS="more bench.py args"] tools/ab_bench.sh ROUNDS TAG...
# ("cur" = meteorgpu/libmsdsp.so, TAG = tools/ubench/bin/libmsdsp_TAG.so)
# Logs to gpurun_out/ab_<wl>_<tag>_<i>.log; prints ms/step, the roofline kernel's ms and the
# per-kernel ms of every run.
set -u
N=$1; shift
WL=${WL:-c3}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
for i in $(seq 1 "$N"); do
  for t in "$@"; do
    lib=$ROOT/tools/ubench/bin/libmsdsp_$t.so
    [ "$t" = cur ] && lib=$ROOT/meteor-scatter_amd/meteorgpu/libmsdsp.so
    extra=""; [ "$WL" = c3 ] && extra="--no-c5"
    MSD_LIB_PATH=$lib timeout -k 10 200 python3 "$ROOT/bench.py" --workload "$WL" --steps 10 --warmup 2 \
        --no-cpu-baseline $extra ${AB_ARGS:-} > "$ROOT/gpurun_out/ab_${WL}_${t}_$i.log" 2>&1 || exit 1
  done
done
for t in "$@"; do
  python3 - "$ROOT" "$WL" "$t" "$N" <<'PY'
import json, sys
root, wl, t, n = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
rows = []
for i in range(1, n + 1):
    d = json.loads(open(f"{root}/gpurun_out/ab_{wl}_{t}_{i}.log").read().strip().splitlines()[-1])
    ks = "/".join(f"{v:.3f}" for v in d.get("kernel_ms_per_step", {}).values())
    rows.append(f"{d['ms_per_step']:.3f}|{d['roofline']['kernel_ms']:.3f}|{ks}")
print(wl, t, " ".join(rows))
PY
done
