#!/bin/bash
# twiddle bases read ahead of the exchanges (LCFIR_FFT_TW_AHEAD) A/B: config 2, config 3, config 3 at L = 32768
set -u -o pipefail
cd "${GRAFT_REPO_ROOT}"
echo "== config 2"; bash scripts/gpu_ab_variants.sh "tw0 tw1" 4 || exit 1
echo "== config 3"; bash scripts/gpu_ab_variants.sh "tw0 tw1" 3 --config 3 || exit 1
echo "== config 3, L = 32768"; bash scripts/gpu_ab_variants.sh "tw0 tw1" 2 --config 3 --seg-len 32768 || exit 1
