#!/bin/bash
# Build libmsdsp.so from a git revision into tools/ubench/bin/libmsdsp_<tag>.so (A/B timing runs:
# MSD_LIB_PATH=tools/ubench/bin/libmsdsp_<tag>.so python bench.py ...).
# Usage: tools/ab_build.sh REV TAG
set -euo pipefail
REV=$1; TAG=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d /tmp/ab_XXXX)
git -C "$ROOT" archive "$REV" meteor-scatter_amd/csrc include | tar -x -C "$W"
mkdir -p "$ROOT/tools/ubench/bin"
make -s -C "$W/meteor-scatter_amd/csrc" -j8 OUT="$ROOT/tools/ubench/bin/libmsdsp_$TAG.so" >/dev/null
rm -rf "$W"
echo "built tools/ubench/bin/libmsdsp_$TAG.so from $REV"
