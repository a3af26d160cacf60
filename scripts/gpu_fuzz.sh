#!/bin/bash
# Extended seeded fuzz campaign on one GPU: tests/test_gpu_fuzz.py over a
# wider seed range than the round-end suite.  Usage (from the repo root):
#   scripts/gpu_fuzz.sh SEED0 CASES NORM_CASES [TAG]
# Writes gpurun_out/fuzz_<TAG>.log (pytest -v: one line per case).
set -o pipefail
seed0=${1:-120}; cases=${2:-600}; norm=${3:-300}; tag=${4:-campaign}
mkdir -p gpurun_out
LCFIR_FUZZ_SEED0=$seed0 LCFIR_FUZZ_CASES=$cases LCFIR_FUZZ_NORM_CASES=$norm \
    timeout -k 10 ${FUZZ_TIMEOUT:-700} python -u -m pytest tests/test_gpu_fuzz.py -m gpu -v -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/fuzz_$tag.log 2>&1
rc=$?
tail -n 3 gpurun_out/fuzz_$tag.log
exit $rc
