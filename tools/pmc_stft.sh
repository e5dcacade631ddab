#!/bin/bash
# PMC passes (one counter group per run, --pmc never combined with tracing) over a
# short bench run; outputs under gpurun_out/pmc/<tag>/.  Usage: tools/pmc_stft.sh TAG [bench args]
set -u
TAG=${1:-r1}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/pmc/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS=${*:-"--files 1440 --steps 2 --warmup 1 --no-cpu-baseline --no-c5 --no-live"}
i=0
# PMC_GROUPS="grp1;grp2": other counter groups (one pass each)
IFS=';' read -r -a GROUPS_ <<< "${PMC_GROUPS:-}"
[ ${#GROUPS_[@]} -gt 0 ] || GROUPS_=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
  "FETCH_SIZE"
  "WRITE_SIZE")
for grp in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -s KILL ${PMC_TIMEOUT:-300} rocprofv3 --pmc $grp --kernel-include-regex "${REGEX:-stft|block_delta|block_band_i8|detect}" -d "$OUT/p$i" -o pmc \
      --output-format csv -- python3 "$ROOT/bench.py" $ARGS > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -gt 1 ]; then exit $rc; fi
done
