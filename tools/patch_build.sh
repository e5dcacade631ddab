#!/bin/bash
# Build the working tree's libmsdsp.so with experiment patches applied to a temporary copy of
# csrc into tools/ubench/bin/libmsdsp_<tag>.so (A/B variants stay out of the product sources; time them
# with tools/stft_ab or tools/ab_bench.sh).  Usage: tools/patch_build.sh TAG [PATCH ...]
# (patches: unified diffs relative to meteor-scatter_amd/csrc, e.g. tools/experiments/*.patch)
set -euo pipefail
TAG=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d /tmp/pvar_XXXX)
mkdir -p "$W/meteor-scatter_amd" && cp -r "$ROOT/meteor-scatter_amd/csrc" "$W/meteor-scatter_amd/" && cp -r "$ROOT/include" "$W/"
rm -rf "$W/meteor-scatter_amd/csrc/build"
for p in "$@"; do
  patch -s -d "$W/meteor-scatter_amd/csrc" -p1 < "$ROOT/$p"
done
mkdir -p "$ROOT/tools/ubench/bin"
make -s -C "$W/meteor-scatter_amd/csrc" -j8 ${MKARGS:-} OUT="$ROOT/tools/ubench/bin/libmsdsp_$TAG.so" >/dev/null
rm -rf "$W"
echo "built tools/ubench/bin/libmsdsp_$TAG.so ($*)"
