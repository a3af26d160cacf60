#!/bin/bash
# 8 ranks of bench.py config 2 sharing one GPU (gloo): the driver's N = 8 launch shape, rehearsed.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export LCFIR_BENCH_SHARE_DEVICE=1
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 8 --steps 10 --warmup 2 --preroll-s 1 > gpurun_out/mr_c2_n8.log 2>&1
rc=$?; grep '^{' gpurun_out/mr_c2_n8.log | cut -c1-600; exit $rc
