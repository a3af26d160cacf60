#!/bin/bash
# GPU box: PMC passes (each its own rocprofv3 run) over a short config-2 bench,
# once per LCFIR_FFT_WAVES setting given, for a side-by-side kernel diagnosis.
# usage: bash scripts/gpu_pmc_ab.sh <tag> "<waves...>" [bench args...]
set -u -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=$1; WAVES=$2; shift 2
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for wv in $WAVES; do
    i=0
    for c in FETCH_SIZE \
             "SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
             "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM"; do
        i=$((i+1))
        echo "== w$wv pass $i ($(date +%T))"
        LCFIR_FFT_WAVES=$wv timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex 'fir_' -f csv \
            -d "$OUT/w$wv/p_$i" -o pmc -- \
            python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-parity --preroll-s 0 "$@" \
            > "$OUT/w${wv}_p$i.log" 2>&1
        rc=$?
        if [ $rc -ne 0 ]; then echo "!! w$wv pass $i rc=$rc"; tail -20 "$OUT/w${wv}_p$i.log"; exit $rc; fi
    done
    python "$ROOT/scripts/pmc_summary.py" "$OUT/w$wv" --json "$OUT/pmc_w$wv.json" > /dev/null
done
echo "== done"
