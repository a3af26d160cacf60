#!/bin/bash
# Device assembly of liblcfir (gfx950) into /tmp/isa/lcfir.s; with a kernel
# name pattern, also that kernel's body into /tmp/isa/k.s and a map of its
# barriers, branches and scratch (spill) accesses.
# usage: bash scripts/isa.sh [kernel-regex]
cd "$(dirname "$0")/../audio-fir-filter_amd" || exit 1
mkdir -p /tmp/isa
/opt/rocm/bin/hipcc -O3 -std=c++2b --offload-arch=gfx950 -I../include -Icsrc --cuda-device-only -S \
    -o /tmp/isa/lcfir.s csrc/lcfir.hip 2>/dev/null || exit 1
[ -z "${1:-}" ] && exit 0
awk -v pat="$1" '$0 ~ "^"pat".*:" && !f {f=1} f {print} f && /s_endpgm/ {exit}' /tmp/isa/lcfir.s > /tmp/isa/k.s
grep -n "s_barrier\|scratch_\|^\.LBB\|s_cbranch" /tmp/isa/k.s | sed 's/\s\+/ /g; s/;.*//' | cut -c1-60
