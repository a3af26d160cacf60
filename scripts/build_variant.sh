#!/bin/bash
# Build an experiment variant of liblcfir.so without touching the product
# source: copy audio-fir-filter_amd/ and include/ to a scratch tree, apply a
# patch (git diff format, paths relative to the repo root), build there and
# put the library in abvar/NAME.so (git-ignored; gpurun ships it).  The
# product tree never carries experiment switches;
# scripts/gpu_run.sh's ab: and parity: steps time and check the variants.
# usage: bash scripts/build_variant.sh NAME [PATCH]    (no PATCH: the product as NAME)
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
NAME=${1:?name}; PATCH=${2:-}
W=$(mktemp -d /tmp/variant_XXXX)
trap 'rm -rf "$W"' EXIT
cp -r "$ROOT/audio-fir-filter_amd" "$ROOT/include" "$W/"
rm -f "$W/audio-fir-filter_amd/liblcfir.so"
if [ -n "$PATCH" ]; then (cd "$W" && patch -p1 --quiet < "$(realpath "$PATCH")"); fi
make -C "$W/audio-fir-filter_amd" liblcfir.so > "$W/build.log" 2>&1 || { tail -30 "$W/build.log"; exit 1; }
mkdir -p "$ROOT/abvar"
cp "$W/audio-fir-filter_amd/liblcfir.so" "$ROOT/abvar/$NAME.so"
cp "$W/audio-fir-filter_amd/liblcfir.remarks" "$ROOT/abvar/$NAME.remarks"
grep -A9 "fir_fft32r_kernelILi4ELb0" "$W/audio-fir-filter_amd/liblcfir.remarks" | grep -E "VGPRs|Spill|Scratch" | sed 's/.*remark: *//; s/ \[-Rpass.*//' | tr '\n' ' '
echo " -> abvar/$NAME.so"
