#!/bin/bash
# GPU box: segment length A/B on one workload -- bench lines at L = 16384 and
# L = 32768 (alternating), then per-length PMC passes (instruction mix, waits).
# usage (repo root, GPU box): bash scripts/gpu_seg_ab.sh <tag> [bench args...]
set -u -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-segab}; shift || true
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
step() { # name timeout cmd...
    local name=$1 t=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    tail -1 "$OUT/$name.log" | python3 -c "import sys,json
for l in sys.stdin:
    try: d=json.loads(l)
    except Exception: print(l[:300]); continue
    r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], d['config'].get('fft_plan'))" 2>/dev/null
    if [ $rc -ne 0 ]; then echo "!! $name failed rc=$rc"; tail -30 "$OUT/$name.log"; exit $rc; fi
}
for rep in 1 2; do
    for L in 16384 32768; do
        step "bench_L${L}_$rep" 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ingest --seg-len $L "$@"
    done
done
cd /tmp && export TMPDIR=/tmp
for L in 16384 32768; do
    i=0
    for c in "SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64" \
             "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
             "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_INSTS_SALU SQ_WAIT_INST_ANY"; do
        i=$((i+1))
        step "pmc_L${L}_$i" 180 rocprofv3 --pmc $c --kernel-include-regex 'fir_' -f csv \
            -d "$OUT/pmc_L$L/p_$i" -o pmc -- \
            python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-ingest --preroll-s 0 \
            --seg-len $L "$@"
    done
done
cd "$ROOT"
for L in 16384 32768; do
    python scripts/pmc_summary.py "$OUT/pmc_L$L" --json "$OUT/pmc_L$L.json" > /dev/null
done
echo "== done"
