#!/bin/bash
# store-skip A/B: config 2, config 3 (L = 16 384), config 3 at L = 32 768
set -u -o pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
echo "== config 2"; bash scripts/gpu_ab_variants.sh "skip0 skip1" 3 || exit 1
echo "== config 3"; bash scripts/gpu_ab_variants.sh "skip0 skip1" 3 --config 3 || exit 1
echo "== config 3, L = 32768"; bash scripts/gpu_ab_variants.sh "skip0 skip1" 2 --config 3 --seg-len 32768 || exit 1
echo "== 19201 taps (L = 32768)"; bash scripts/gpu_ab_variants.sh "skip0 skip1" 2 --ntaps 19201 || exit 1
