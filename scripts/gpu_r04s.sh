#!/bin/bash
# Round 4: output-store cache policy of the register kernel's pair stores
# (LCFIR_FFT32_STORE_AUX: 2 = nt, the product; 0 plain; 3 nt sc0; 18 nt sc1),
# alternating driver-shaped config-2 lines and the config-4 one-file step.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r04s; mkdir -p "$OUT"
cp audio-fir-filter_amd/liblcfir.so abvar/sa2.so
echo "== config 2"; bash scripts/gpu_ab_variants.sh "sa2 sa0 sa3 sa18" 2 | tee "$OUT/ab_c2.txt" || exit 1
echo "== config 4 one file"; bash scripts/gpu_ab_variants.sh "sa2 sa0 sa18" 1 --config 4 --files 1 --steps 10 --warmup 3 | tee "$OUT/ab_c4f1.txt" || exit 1
echo "== done"
