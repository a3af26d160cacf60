#!/bin/bash
# GPU-box run of BASELINE.json configs 1-5 at N = 1 (bench lines) plus a
# rocprofv3 kernel-stats pass per config.  Every GPU step has its own time
# limit; the first failure ends the script.
# usage (from the repo root, on the GPU box): bash scripts/gpu_configs.sh [tag]
set -u -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-cfg}
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
step() { # name timeout cmd...
    local name=$1 t=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    tail -2 "$OUT/$name.log" | cut -c1-3000
    if [ $rc -ne 0 ]; then echo "!! $name failed rc=$rc"; tail -40 "$OUT/$name.log"; exit $rc; fi
}
step bench_c2 300 python bench.py --steps 20 --warmup 5
step bench_c1 300 python bench.py --config 1 --steps 20 --warmup 5
step bench_c3 300 python bench.py --config 3 --steps 20 --warmup 5
step bench_c4 600 python bench.py --config 4 --steps 20 --warmup 3
step bench_c5 600 python bench.py --config 5 --steps 20 --warmup 3 --no-cpu-baseline
step bench_c5g 600 python bench.py --config 5 --peak-scope global --steps 20 --warmup 3 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
step rocprof_c3 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_${TAG}_c3" -o bench -- \
    python3 "$ROOT/bench.py" --config 3 --no-cpu-baseline --no-parity
step rocprof_c4 600 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_${TAG}_c4" -o bench -- \
    python3 "$ROOT/bench.py" --config 4 --steps 10 --warmup 2 --no-cpu-baseline --no-parity
cp "$OUT/prof_${TAG}_c3/bench_kernel_stats.csv" "$OUT/kernel_stats_${TAG}_c3.csv"
cp "$OUT/prof_${TAG}_c4/bench_kernel_stats.csv" "$OUT/kernel_stats_${TAG}_c4.csv"
echo "== done"
