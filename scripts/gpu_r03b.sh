#!/bin/bash
# round 3: the L = 32768 segment on the device: its parity tests first, then
# the whole GPU suite, then config 2 / 3 / 1 bench lines.
set -u -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r03b}
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
step() { # name timeout cmd...
    local name=$1 t=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$t" "$@" > "$OUT/${TAG}_$name.log" 2>&1
    local rc=$?
    tail -3 "$OUT/${TAG}_$name.log" | cut -c1-3000
    if [ $rc -ne 0 ]; then echo "!! $name failed rc=$rc"; tail -80 "$OUT/${TAG}_$name.log"; exit $rc; fi
}
step seg32 600 python -u -m pytest tests/test_gpu_parity.py -k "seg32" -x -v --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 1500 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread
step bench_c2 400 python bench.py --steps 20 --warmup 5
step bench_c3 400 python bench.py --config 3 --steps 20 --warmup 5 --no-cpu-baseline
step bench_c1 400 python bench.py --config 1 --steps 20 --warmup 5 --no-cpu-baseline
echo "== done"
