#!/bin/bash
# Round 4, first GPU pass: smoke, the GPU suite, the driver-shaped bench line,
# the drop-in timing tool (config 2's file through ProcessFile.cp's threads),
# and the bare `bench.py --gpus 2` launch.  The first failure ends the script.
set -u -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-r04a}"
mkdir -p "$OUT"
step() { # name timeout cmd...
    local name=$1 t=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    tail -3 "$OUT/$name.log" | cut -c1-2500
    if [ $rc -ne 0 ]; then echo "!! $name failed rc=$rc"; tail -40 "$OUT/$name.log"; exit $rc; fi
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step bench 300 python bench.py --steps 20 --warmup 5
step dropin 600 tests/cpp/dropin_bench --threads 1,16,ref --reps 3
LCFIR_BENCH_SHARE_DEVICE=1 step gpus2 300 python bench.py --gpus 2 --config 5 --files 2 --seconds 600 --steps 10 --warmup 2
echo "== done"
