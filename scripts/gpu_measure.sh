#!/bin/bash
# GPU box: the driver-shaped bench line, the rocprofv3 kernel stats of the same
# command, and the PMC passes bench.py's roofline reads (HBM traffic, f64 and
# VALU instruction counts) plus an issue/LDS diagnosis pass -- each its own
# rocprofv3 run with its own time limit; the first failure ends the script.
# usage (repo root, GPU box): bash scripts/gpu_measure.sh <tag> [bench args...]
set -u -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-run}; shift || true
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
step() { # name timeout cmd...
    local name=$1 t=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    tail -2 "$OUT/$name.log" | cut -c1-2500
    if [ $rc -ne 0 ]; then echo "!! $name failed rc=$rc"; tail -30 "$OUT/$name.log"; exit $rc; fi
}
step bench 300 python bench.py --steps 20 --warmup 5 "$@"
cd /tmp && export TMPDIR=/tmp
step rocprof 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o bench -- \
    python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline "$@"
cp "$OUT"/prof/*/bench_kernel_stats.csv "$OUT/kernel_stats.csv" 2>/dev/null || \
    cp "$OUT"/prof/bench_kernel_stats.csv "$OUT/kernel_stats.csv"
i=0
for c in FETCH_SIZE WRITE_SIZE \
         "SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_INSTS_SALU SQ_WAIT_INST_ANY"; do
    i=$((i+1))
    step "pmc_$i" 180 rocprofv3 --pmc $c --kernel-include-regex 'fir_' -f csv \
        -d "$OUT/pmc/p_$i" -o pmc -- \
        python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-parity --preroll-s 0 "$@"
done
cd "$ROOT"
python scripts/pmc_summary.py "$OUT/pmc" --json "$OUT/pmc_summary.json" > /dev/null
echo "== done"
