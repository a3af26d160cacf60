#!/bin/bash
# Round 4: pair stores through a per-unit buffer resource (LCFIR_R32_STORE=2,
# abvar/st2.so) against the quad-store product (st1): parity on st2 first
# (the whole GPU suite), then alternating
# driver-shaped lines, configs 2 and 3.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r04l; mkdir -p "$OUT"
cp audio-fir-filter_amd/liblcfir.so /tmp/prod.so
cp abvar/st2.so audio-fir-filter_amd/liblcfir.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ \
  > "$OUT/tests_st2.log" 2>&1; rc=$?
tail -3 "$OUT/tests_st2.log"
cp /tmp/prod.so audio-fir-filter_amd/liblcfir.so
[ $rc -ne 0 ] && { tail -40 "$OUT/tests_st2.log"; exit $rc; }
echo "== config 2"; bash scripts/gpu_ab_variants.sh "st1 st2" 3 | tee "$OUT/ab_c2.txt" || exit 1
echo "== config 3"; bash scripts/gpu_ab_variants.sh "st1 st2" 2 --config 3 | tee "$OUT/ab_c3.txt" || exit 1
echo "== done"
