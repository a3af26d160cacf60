#!/bin/bash
# Round 4: cache policy of the fused normalize slice's loads
# (LCFIR_NRM_LOAD_AUX: 2 = nt, the product; 0 plain; 18 nt sc1), the N = 8
# per-rank config-5 step, alternating.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r04v; mkdir -p "$OUT"
bash scripts/gpu_ab_variants.sh "na2 na0 na18" 3 --config 5 --files 1 --force-exchange --steps 10 --warmup 3 | tee "$OUT/ab_c5f1x.txt" || exit 1
echo "== done"
