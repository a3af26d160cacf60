#!/bin/bash
# LLVM scheduling-flag variants of liblcfir (same source), config 2
set -u -o pipefail
cd "${GRAFT_REPO_ROOT}"
bash scripts/gpu_ab_variants.sh "base bias0 postbu nohrp nocluster nopost" 3 || exit 1
