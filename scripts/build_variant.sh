#!/bin/bash
# Build an experiment variant of liblcfir.so without touching the product
# source: copy audio-fir-filter_amd/ and include/ to a scratch tree, apply a
# patch (git diff format, paths relative to the repo root), build there and
# put the library in abvar/NAME.so (git-ignored; gpurun ships it).  The
# product tree never carries experiment switches;
# scripts/gpu_run.sh's ab: and parity: steps time and check the variants.
# usage: bash scripts/build_variant.sh NAME [PATCH]    (no PATCH: the product as NAME;
# the patches measured so far are scripts/variants/*.patch, README there)
# Also builds tools/fft32r_trace from the patched source as abvar/NAME.trace.
# abvar/NAME.base stamps the base: the unpatched tree's build id
# (audio-fir-filter_amd/src_hash.sh) and commit; scripts/gpu_run.sh refuses a
# variant whose base id is not the id of the tree it runs in (a variant built
# on an older tree would otherwise time a different product).
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
NAME=${1:?name}; PATCH=${2:+$(realpath "$2")}
W=$(mktemp -d /tmp/variant_XXXX)
trap 'rm -rf "$W"' EXIT
cp -r "$ROOT/audio-fir-filter_amd" "$ROOT/include" "$W/"
rm -f "$W/audio-fir-filter_amd/liblcfir.so"
BASE_ID=$(bash "$W/audio-fir-filter_amd/src_hash.sh")
BASE_COMMIT=$(git -C "$ROOT" rev-parse --short HEAD 2>/dev/null || echo none)
git -C "$ROOT" diff --quiet HEAD -- audio-fir-filter_amd include 2>/dev/null || BASE_COMMIT="$BASE_COMMIT+dirty"
if [ -n "$PATCH" ]; then (cd "$W" && patch -p1 --quiet < "$PATCH"); fi
make -C "$W/audio-fir-filter_amd" liblcfir.so > "$W/build.log" 2>&1 || { tail -30 "$W/build.log"; exit 1; }
mkdir -p "$ROOT/abvar"
cp "$W/audio-fir-filter_amd/liblcfir.so" "$ROOT/abvar/$NAME.so"
cp "$W/audio-fir-filter_amd/liblcfir.remarks" "$ROOT/abvar/$NAME.remarks"
echo "base_build_id=$BASE_ID base_commit=$BASE_COMMIT patch=${2:-none} variant_build_id=$(bash "$W/audio-fir-filter_amd/src_hash.sh")" \
    > "$ROOT/abvar/$NAME.base"
# the phase-trace tool of the same source (abvar/NAME.trace: gpu_run.sh trace:ARGS takes TRACE=...)
/opt/rocm/bin/hipcc -O3 -std=c++2b --offload-arch=gfx950 -I"$W/audio-fir-filter_amd/csrc" \
    "$W/audio-fir-filter_amd/tools/fft32r_trace.hip" -o "$ROOT/abvar/$NAME.trace" > "$W/trace.log" 2>&1 \
    || { tail -20 "$W/trace.log"; exit 1; }
grep -A9 "fir_fft32r_kernelILi4ELb0" "$W/audio-fir-filter_amd/liblcfir.remarks" | grep -E "VGPRs|Spill|Scratch" | sed 's/.*remark: *//; s/ \[-Rpass.*//' | tr '\n' ' '
echo " -> abvar/$NAME.so"
