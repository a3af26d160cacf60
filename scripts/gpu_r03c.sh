#!/bin/bash
# round 3: GPU suite on the tree, then the bench lines: config 2 (driver
# shape), 3, 1, a long filter (config-2 data, 19 201 taps), and the N = 8
# per-rank shapes of configs 4/5 (one file; config 5 with the RCCL exchange).
set -u -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r03c}
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
step() { # name timeout cmd...
    local name=$1 t=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$t" "$@" > "$OUT/${TAG}_$name.log" 2>&1
    local rc=$?
    tail -2 "$OUT/${TAG}_$name.log" | cut -c1-1500
    if [ $rc -ne 0 ]; then echo "!! $name failed rc=$rc"; tail -80 "$OUT/${TAG}_$name.log"; exit $rc; fi
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 1500 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread
step bench_c2 400 python bench.py --steps 20 --warmup 5
step bench_c3 300 python bench.py --config 3 --steps 20 --warmup 5 --no-cpu-baseline
step bench_c1 300 python bench.py --config 1 --steps 20 --warmup 5 --no-cpu-baseline
step bench_t19201 300 python bench.py --ntaps 19201 --steps 20 --warmup 5 --no-cpu-baseline
step bench_c4f1 300 python bench.py --config 4 --files 1 --steps 10 --warmup 3 --no-cpu-baseline
step bench_c5f1x 300 python bench.py --config 5 --files 1 --force-exchange --steps 10 --warmup 3 --no-cpu-baseline
echo "== done"
