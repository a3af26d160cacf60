#!/bin/bash
# GPU box: the fused per-file normalize -- its tests, then config 5 (and 4)
# with and without the fusion, alternating.  Each GPU step has its own time
# limit; the first failure ends the script.
set -u -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
step() { # name timeout cmd...
    local name=$1 t=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    tail -2 "$OUT/$name.log" | cut -c1-1500
    if [ $rc -ne 0 ]; then echo "!! $name failed rc=$rc"; tail -40 "$OUT/$name.log"; exit $rc; fi
}
step pytest_nrm 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_batch.py \
    "tests/test_gpu_parity.py::test_fft_channel_groups" tests/test_gpu_baseline_configs.py
for rep in 1 2; do
    step "c5_fused_$rep" 300 python bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline
    step "c5_sep_$rep" 300 python bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline --no-fuse-normalize
done
step c4_fused 300 python bench.py --config 4 --steps 10 --warmup 2 --no-cpu-baseline
step c4_sep 300 python bench.py --config 4 --steps 10 --warmup 2 --no-cpu-baseline --no-fuse-normalize
echo "== done"
