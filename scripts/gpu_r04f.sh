#!/bin/bash
# output-store cache policy A/B on config 2 and config 3 (aux 2 = nt, the product; 16 = sc1; 18 = nt sc1; 0 = plain),
# then the drop-in tool's pinned mode (buffers pinned on the loop thread only)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT}"
echo "== config 2"; bash scripts/gpu_ab_variants.sh "aux2 aux16 aux18 aux0" 3 || exit 1
echo "== config 3"; bash scripts/gpu_ab_variants.sh "aux2 aux16 aux18" 2 --config 3 || exit 1
mkdir -p gpurun_out/r04f
timeout -k 10 600 tests/cpp/dropin_bench --threads 1,16,ref --reps 3 --modes pageable,pinned > gpurun_out/r04f/dropin.log 2>&1 || { tail -5 gpurun_out/r04f/dropin.log; exit 1; }
cut -c1-330 gpurun_out/r04f/dropin.log
