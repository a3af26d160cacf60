#!/bin/bash
# Round 4, final product kernel: a wider seeded fuzz campaign (new seeds) and
# the config-3 / config-4 rocprofv3 kernel traces.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT}"
FUZZ_TIMEOUT=600 bash scripts/gpu_fuzz.sh 40000 12000 3000 r04t || exit 1
bash scripts/gpu_configs.sh r04t || exit 1
echo "== all done"
