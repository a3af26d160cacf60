#!/bin/bash
# GPU-box check: smoke -> pytest -m gpu -> bench -> rocprofv3 kernel stats ->
# PMC HBM traffic (FETCH_SIZE / WRITE_SIZE) and f64 VALU instruction counts,
# each its own rocprofv3 --pmc pass -> pmc summary json.
# Every GPU step has its own time limit; the first failure ends the script.
# usage (from the repo root, on the GPU box): bash scripts/gpu_check.sh [tag] [bench args...]
set -u -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-run}; shift || true
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
step() { # name timeout cmd...
    local name=$1 t=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    tail -3 "$OUT/$name.log" | cut -c1-3000
    if [ $rc -ne 0 ]; then echo "!! $name failed rc=$rc"; tail -40 "$OUT/$name.log"; exit $rc; fi
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step bench 600 python bench.py "$@"
cd /tmp && export TMPDIR=/tmp
step rocprof 600 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_$TAG" -o bench -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline --no-parity --no-ingest "$@"
cp "$OUT/prof_$TAG/bench_kernel_stats.csv" "$OUT/kernel_stats_$TAG.csv"
python3 "$ROOT/scripts/trace_exclusive.py" "$OUT/prof_$TAG/bench_kernel_trace.csv" > "$OUT/exclusive_from_trace_$TAG.json"
i=0
for c in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64"; do
    i=$((i+1))
    step "pmc_$i" 600 rocprofv3 --pmc $c --kernel-include-regex 'fir_' -f csv \
        -d "$OUT/pmc_$TAG/p_$i" -o pmc -- \
        python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-ingest "$@"
done
cd "$ROOT"
python scripts/pmc_summary.py "$OUT/pmc_$TAG" --json "$OUT/pmc_summary_$TAG.json" > /dev/null
echo "== done"
