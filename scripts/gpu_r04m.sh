#!/bin/bash
# Round 4: L2 prefetch of the next unit's samples at barrier 1 (LCFIR_R32_PF=1,
# abvar/pf1.so) against the product (pf0): parity subset on pf1, alternating
# driver-shaped lines (configs 2, 3, the config-5 per-rank step), phase traces.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r04m; mkdir -p "$OUT"
cp audio-fir-filter_amd/liblcfir.so /tmp/prod.so
cp abvar/pf1.so audio-fir-filter_amd/liblcfir.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_baseline_configs.py tests/test_gpu_parity.py > "$OUT/tests_pf1.log" 2>&1; rc=$?
tail -3 "$OUT/tests_pf1.log"
cp /tmp/prod.so audio-fir-filter_amd/liblcfir.so
[ $rc -ne 0 ] && { tail -40 "$OUT/tests_pf1.log"; exit $rc; }
T=audio-fir-filter_amd/tools
timeout -k 10 60 $T/fft32r_trace 4001 32768 > "$OUT/trace_pf0.log" 2>&1 || exit 1
timeout -k 10 60 $T/fft32r_trace_pf 4001 32768 > "$OUT/trace_pf1.log" 2>&1 || exit 1
grep kernel "$OUT"/trace_pf*.log
echo "== config 2"; bash scripts/gpu_ab_variants.sh "pf0 pf1" 3 | tee "$OUT/ab_c2.txt" || exit 1
echo "== config 3"; bash scripts/gpu_ab_variants.sh "pf0 pf1" 2 --config 3 | tee "$OUT/ab_c3.txt" || exit 1
echo "== config 5 per rank"; bash scripts/gpu_ab_variants.sh "pf0 pf1" 2 --config 5 --files 1 --force-exchange --steps 10 --warmup 3 | tee "$OUT/ab_c5f1x.txt" || exit 1
echo "== done"
