#!/bin/bash
# Kernel resource report (VGPRs, spills, occupancy) of liblcfir's device code,
# one line per kernel.  usage: bash scripts/spills.sh [extra hipcc flags...]
cd "$(dirname "$0")/../audio-fir-filter_amd" || exit 1
/opt/rocm/bin/hipcc -O3 -std=c++2b --offload-arch=gfx950 -I../include -Icsrc --cuda-device-only -c -o /dev/null \
    csrc/lcfir.hip -Rpass-analysis=kernel-resource-usage "$@" 2>&1 |
  awk '/Function Name:/ {n=$(NF-1)} /VGPRs:/ {v=$(NF-1)} /AGPRs:/ {a=$(NF-1)} /SGPRs Spill:/ {ss=$(NF-1)}
       /VGPRs Spill:/ {vs=$(NF-1)} /Occupancy/ {o=$(NF-1)}
       /LDS Size/ {printf "%-70s vgpr %s agpr %s vspill %s sspill %s occ %s\n", substr(n,1,70), v, a, vs, ss, o}'
