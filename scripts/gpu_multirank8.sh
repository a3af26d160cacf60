#!/bin/bash
# 8 ranks of bench.py config 2 sharing one GPU (gloo): the driver's N = 8 shape, rehearsed through the
# bare `bench.py --gpus 8` launch (bench.py starts the 8 rank processes itself).
set -u -o pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export LCFIR_BENCH_SHARE_DEVICE=1
timeout -k 10 240 python bench.py --gpus 8 --steps 10 --warmup 2 --preroll-s 1 > gpurun_out/mr_c2_n8.log 2>&1
rc=$?; grep '^{' gpurun_out/mr_c2_n8.log | cut -c1-600; exit $rc
