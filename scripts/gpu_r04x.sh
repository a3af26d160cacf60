#!/bin/bash
# Round 4: the pair table's second half loaded entry by entry in the pair step
# (LCFIR_R32_PAIR2=1, abvar/p21.so) against the product (p20): parity
# subset on p21, alternating driver-shaped lines, configs 2 and 3.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r04x; mkdir -p "$OUT"
cp audio-fir-filter_amd/liblcfir.so /tmp/prod.so
cp abvar/p21.so audio-fir-filter_amd/liblcfir.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_baseline_configs.py tests/test_gpu_parity.py > "$OUT/tests_p21.log" 2>&1; rc=$?
tail -1 "$OUT/tests_p21.log"
cp /tmp/prod.so audio-fir-filter_amd/liblcfir.so
[ $rc -ne 0 ] && { tail -40 "$OUT/tests_p21.log"; exit $rc; }
echo "== config 2"; bash scripts/gpu_ab_variants.sh "p20 p21" 3 | tee "$OUT/ab_c2.txt" || exit 1
echo "== config 3"; bash scripts/gpu_ab_variants.sh "p20 p21" 2 --config 3 | tee "$OUT/ab_c3.txt" || exit 1
echo "== done"
