#!/bin/bash
# Round 4, the late-wait register kernel as the product: smoke, the GPU suite,
# the config-2 line, rocprofv3 trace + PMC, then a seeded fuzz campaign.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT}"
bash scripts/gpu_check.sh r04p --steps 20 --warmup 5 || exit 1
FUZZ_TIMEOUT=300 bash scripts/gpu_fuzz.sh 30000 3000 800 r04p || exit 1
echo "== all done"
