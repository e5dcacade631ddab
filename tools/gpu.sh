#!/bin/bash
# The GPU-box runner: one parametrised script for the measurement steps of every round (replaces the
# per-call scripts of rounds 1-4).  Every step runs under its own `timeout -k 10`, the steps of one
# call are chained so that the first failure ends the call, and outputs go under gpurun_out/.
#
#   tools/gpu.sh test   NAME [pytest args]      pytest -m gpu over the args (default: the whole suite)
#   tools/gpu.sh smoke                          __graft_entry__.smoke()
#   tools/gpu.sh bench  NAME [bench.py args]    one bench line → gpurun_out/NAME.json, summary printed
#   tools/gpu.sh c5     NAME REPS [bench args]  REPS exact-mode C5 benches (certified headline)
#   tools/gpu.sh trace  NAME [bench.py args]    rocprofv3 --kernel-trace --stats of a bench run +
#                                               tools/trace_gaps.py step timeline
#   tools/gpu.sh ab     WL ROUNDS TAG...        tools/ab_bench.sh (variants in tools/ubench/bin)
#   tools/gpu.sh stft_ab NAME MODE ROUNDS LIB... tools/stft_ab (MODE c3 | c5; STFT_AB_* env passed on)
#   tools/gpu.sh pmc    TAG REGEX [bench args]  tools/pmc_stft.sh's four PMC passes
#   tools/gpu.sh round  TAG                     tools/profile_round.sh (bench + traces + PMC)
#   tools/gpu.sh py     NAME SECONDS SCRIPT [args]  a python script under a time limit
#
# Several steps in one call: tools/gpu.sh multi 'test t1 tests/test_iq.py' 'c5 c5a 2' ...
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT" || exit 1
mkdir -p gpurun_out
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"

summary() {  # the last JSON line of a bench output, condensed
  python3 - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d.get("c5") or {}
cert = d.get("certification") or c.get("certification") or {}
print(json.dumps({k: d.get(k) for k in ("value", "ms_per_step", "kernel_ms_per_step")} |
                 {"frac": d.get("roofline", {}).get("frac"), "certified": cert.get("certified"),
                  "c5": c.get("value"), "c5_ms": c.get("ms_per_step"),
                  "c5_frac": c.get("roofline", {}).get("frac"), "ranks_seen": d.get("ranks_seen")}))
PY
}

step() {
  local cmd=$1; shift
  case "$cmd" in
    test)
      local name=$1; shift
      timeout -k 10 900 $PYT -m gpu "${@:-tests}" > "gpurun_out/$name.log" 2>&1; local rc=$?
      tail -3 "gpurun_out/$name.log"; return $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" ;;
    bench)
      local name=$1; shift
      timeout -k 10 600 python bench.py "$@" > "gpurun_out/$name.json" 2> "gpurun_out/$name.err" || { tail -5 "gpurun_out/$name.err"; return 1; }
      summary "gpurun_out/$name.json" ;;
    c5)
      local name=$1 reps=$2; shift 2
      for r in $(seq 1 "$reps"); do
        timeout -k 10 300 python bench.py --workload c5 --c5-mode exact --steps 20 --warmup 10 --no-cpu-baseline "$@" \
          > "gpurun_out/${name}_$r.json" 2> "gpurun_out/${name}_$r.err" || { tail -5 "gpurun_out/${name}_$r.err"; return 1; }
        summary "gpurun_out/${name}_$r.json" || return 1
      done ;;
    trace)
      local name=$1; shift
      (cd /tmp && export TMPDIR=/tmp && cd "$ROOT" &&
       timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/$name" -o "$name" -- \
         python3 bench.py "$@" > "gpurun_out/$name.log" 2>&1) || return 1
      python3 tools/trace_gaps.py "gpurun_out/$name" > "gpurun_out/${name}_gaps.txt" 2>&1
      head -14 "gpurun_out/${name}_gaps.txt" ;;
    ab)
      local wl=$1; shift
      WL=$wl timeout -k 10 1100 bash tools/ab_bench.sh "$@" ;;
    stft_ab)
      local name=$1 mode=$2 rounds=$3; shift 3
      STFT_AB_MODE=$mode timeout -k 10 400 tools/stft_ab "$rounds" "$@" > "gpurun_out/$name.txt" 2>&1; local rc=$?
      tail -8 "gpurun_out/$name.txt"; return $rc ;;
    pmc)
      local tag=$1 regex=$2; shift 2
      REGEX=$regex timeout -k 10 900 bash tools/pmc_stft.sh "$tag" "$@" || return 1
      python3 tools/pmc_summary.py "gpurun_out/pmc/$tag" > "gpurun_out/pmc_$tag.txt" 2>&1; cat "gpurun_out/pmc_$tag.txt" ;;
    round)
      timeout -k 10 1100 bash tools/profile_round.sh "$1" ;;
    py)
      local name=$1 secs=$2; shift 2
      timeout -k 10 "$secs" python3 -u "$@" > "gpurun_out/$name.txt" 2>&1; local rc=$?
      tail -40 "gpurun_out/$name.txt"; return $rc ;;
    *)
      echo "tools/gpu.sh: unknown step '$cmd'" >&2; return 2 ;;
  esac
}

if [ "$1" = multi ]; then
  shift
  for s in "$@"; do
    echo "== $s"
    # shellcheck disable=SC2086
    step $s || { echo "step failed: $s"; exit 1; }
  done
else
  step "$@"
fi
