#!/bin/bash
# GPU-box quick check: smoke -> pytest -m gpu -> bench (one line).
# usage (repo root, on the GPU box): bash scripts/gpu_quick.sh <tag> [bench args...]
set -u -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-run}; shift || true
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
step() { # name timeout cmd...
    local name=$1 t=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$t" "$@" > "$OUT/${TAG}_$name.log" 2>&1
    local rc=$?
    tail -3 "$OUT/${TAG}_$name.log" | cut -c1-3000
    if [ $rc -ne 0 ]; then echo "!! $name failed rc=$rc"; tail -60 "$OUT/${TAG}_$name.log"; exit $rc; fi
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 1500 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread
step bench 600 python bench.py "$@"
echo "== done"
