#!/bin/bash
# Round 4: the next unit's LDS-DMA issued in quarters between the final
# phase's VALU blocks (LCFIR_R32_DMASPLIT=4) and/or non-temporal
# (LCFIR_R32_DMA_AUX=2), against the product (ds0): parity subset on ds4,
# phase traces, alternating driver-shaped lines.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r04o; mkdir -p "$OUT"
cp audio-fir-filter_amd/liblcfir.so /tmp/prod.so
for v in ds4 lw; do
cp abvar/$v.so audio-fir-filter_amd/liblcfir.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_baseline_configs.py tests/test_gpu_parity.py > "$OUT/tests_$v.log" 2>&1; rc=$?
tail -1 "$OUT/tests_$v.log"
cp /tmp/prod.so audio-fir-filter_amd/liblcfir.so
[ $rc -ne 0 ] && { tail -40 "$OUT/tests_$v.log"; exit $rc; }
done
T=audio-fir-filter_amd/tools/fft32r_trace
for v in "" _ds4 _lw; do timeout -k 10 60 $T$v 4001 32768 > "$OUT/trace${v:-_base}.log" 2>&1 || exit 1; grep kernel "$OUT/trace${v:-_base}.log"; done
echo "== config 2"; bash scripts/gpu_ab_variants.sh "ds0 ds4 lw nt" 3 | tee "$OUT/ab_c2.txt" || exit 1
echo "== config 3"; bash scripts/gpu_ab_variants.sh "ds0 ds4 lw nt" 2 --config 3 | tee "$OUT/ab_c3.txt" || exit 1
echo "== done"
