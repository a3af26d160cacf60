#!/bin/bash
# multi-rank rehearsal (bare --gpus N launches) + drop-in pinned mode + config 1 with the taps-only plan
set -u -o pipefail
cd "${GRAFT_REPO_ROOT}"
bash scripts/gpu_r04d.sh || exit 1
mkdir -p gpurun_out/r04e
echo "== dropin (pageable, pinned)"
timeout -k 10 600 tests/cpp/dropin_bench --threads 1,16,ref --reps 3 --modes pageable,pinned > gpurun_out/r04e/dropin.log 2>&1 || { tail -5 gpurun_out/r04e/dropin.log; exit 1; }
cut -c1-330 gpurun_out/r04e/dropin.log
echo "== config 1 (L = 32768 by the taps-only plan)"
timeout -k 10 300 python bench.py --config 1 --steps 20 --warmup 5 > gpurun_out/r04e/bench_c1.json 2> gpurun_out/r04e/bench_c1.err || { tail -5 gpurun_out/r04e/bench_c1.err; exit 1; }
cut -c1-700 gpurun_out/r04e/bench_c1.json
