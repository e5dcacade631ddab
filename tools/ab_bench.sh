#!/bin/bash
# Alternate bench runs between in-tree library variants (GPU box).  Usage: tools/ab_bench.sh ROUNDS TAG... 
# "cur" = meteorgpu/libmsdsp.so.  Logs to gpurun_out/ab_<tag>_<i>.log
set -u
N=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
for i in $(seq 1 "$N"); do
  for t in "$@"; do
    lib=$ROOT/meteor-scatter_amd/meteorgpu/libmsdsp_$t.so
    [ "$t" = cur ] && lib=$ROOT/meteor-scatter_amd/meteorgpu/libmsdsp.so
    MSD_LIB_PATH=$lib timeout -k 10 200 python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline \
        > "$ROOT/gpurun_out/ab_${t}_$i.log" 2>&1 || exit 1
  done
done
for t in "$@"; do
  python3 - "$ROOT" "$t" "$N" <<'PY'
import json, sys
root, t, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
ks = []
for i in range(1, n + 1):
    d = json.loads(open(f"{root}/gpurun_out/ab_{t}_{i}.log").read().strip().splitlines()[-1])
    ks.append((d["ms_per_step"], d["kernel_ms_per_step"]["stft"], d["kernel_ms_per_step"]["block_delta"], d["kernel_ms_per_step"]["detect"]))
print(t, " ".join(f"{a:.3f}/{b:.3f}/{c:.3f}/{e:.3f}" for a, b, c, e in ks))
PY
done
