#!/bin/bash
# Build the WORKING TREE's libmsdsp.so with extra compiler flags into
# tools/ubench/bin/libmsdsp_<tag>.so (experiment variants selected by -D macros; timing with
# tools/ab_bench.sh).  Usage: tools/variant_build.sh TAG "EXTRA FLAGS"
set -euo pipefail
TAG=$1; EXTRA=${2:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d /tmp/var_XXXX)
mkdir -p "$W/meteor-scatter_amd" && cp -r "$ROOT/meteor-scatter_amd/csrc" "$W/meteor-scatter_amd/" && cp -r "$ROOT/include" "$W/"
rm -rf "$W/meteor-scatter_amd/csrc/build"
mkdir -p "$ROOT/tools/ubench/bin"
make -s -C "$W/meteor-scatter_amd/csrc" -j8 EXTRA="$EXTRA" ${MKARGS:-} OUT="$ROOT/tools/ubench/bin/libmsdsp_$TAG.so" >/dev/null
rm -rf "$W"
echo "built tools/ubench/bin/libmsdsp_$TAG.so (EXTRA=$EXTRA)"
