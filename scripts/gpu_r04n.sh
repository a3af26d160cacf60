#!/bin/bash
# Round 4: phase traces of the register kernel, where the final phase's time
# goes: product, no output stores, no next-unit DMA (both timing-only,
# wrong outputs), odd workgroups staggered by 2 / 4 x 8 128 cycles.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r04n; mkdir -p "$OUT"
T=audio-fir-filter_amd/tools/fft32r_trace
for r in 1 2; do
for v in "" _nost _nodma _stg2 _stg4; do
  timeout -k 10 60 $T$v 4001 32768 > "$OUT/trace${v:-_base}_$r.log" 2>&1 || { tail "$OUT/trace${v:-_base}_$r.log"; exit 1; }
  echo "${v:-_base} $r $(grep kernel "$OUT/trace${v:-_base}_$r.log")"
done
done
echo "== done"
