#!/bin/bash
# config-5 fused normalize with LDS-DMA'd slice blocks: parity subset on the
# DMA build, then A/B of 0 / 3 / 5 staged blocks on the N = 8 per-rank
# config-5 step (one 60-min file, the all-reduce every step) and config 4's
# one-file step; then the drop-in timing tool.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r04c
cp audio-fir-filter_amd/liblcfir.so /tmp/lib_product.so
cp abvar/nrmdma5.so audio-fir-filter_amd/liblcfir.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_batch.py -m gpu -k "norm or fused or configs_4_and_5 or rccl" > gpurun_out/r04c/pytest_nrm.log 2>&1
rc=$?; tail -3 gpurun_out/r04c/pytest_nrm.log; cp /tmp/lib_product.so audio-fir-filter_amd/liblcfir.so; [ $rc -eq 0 ] || exit $rc
echo "== config 5, one file + exchange"; bash scripts/gpu_ab_variants.sh "nrmdma0 nrmdma3 nrmdma5" 3 --config 5 --files 1 --force-exchange || exit 1
echo "== config 4, one file"; bash scripts/gpu_ab_variants.sh "nrmdma0" 2 --config 4 --files 1 || exit 1
echo "== config 5, 8 files"; bash scripts/gpu_ab_variants.sh "nrmdma0 nrmdma5" 2 --config 5 || exit 1
echo "== dropin"; timeout -k 10 600 tests/cpp/dropin_bench --threads 1,16,ref --reps 3 > gpurun_out/r04c/dropin.log 2>&1 || { tail -5 gpurun_out/r04c/dropin.log; exit 1; }
cut -c1-400 gpurun_out/r04c/dropin.log
