#!/bin/bash
# GPU-box check: smoke -> pytest -m gpu -> bench -> rocprofv3 kernel stats.
# Every GPU step has its own time limit; the first failure ends the script.
# usage (from the repo root, on the GPU box): bash scripts/gpu_check.sh [bench args...]
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
    tail -5 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then echo "!! $name failed rc=$rc"; tail -40 "$OUT/$name.log"; exit $rc; fi
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 1200 python -m pytest tests -m gpu -x -q
step bench 600 python bench.py --steps 10 --warmup 2 "$@"
cd /tmp && export TMPDIR=/tmp
step rocprof 600 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o bench -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline "$@"
find "$OUT/prof" -name "*kernel_stats*" -exec cp {} "$OUT/" \;
echo "== done"
