#!/bin/bash
# PMC passes (each its own rocprofv3 run, counters only) over a short bench run.
# usage: bash scripts/gpu_pmc.sh <tag> [bench args...]
set -u -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; shift
OUT="$ROOT/gpurun_out/pmc_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
i=0
while read -r counters; do
    [ -z "$counters" ] && continue
    i=$((i+1))
    echo "== pass $i: $counters ($(date +%T))"
    timeout -k 10 300 rocprofv3 --pmc $counters --kernel-include-regex 'fir_' -f csv \
        -d "$OUT/p$i" -o pmc -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline "$@" \
        > "$OUT/p$i.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "!! pass $i rc=$rc"; tail -20 "$OUT/p$i.log"; exit $rc; fi
done <<'LIST'
FETCH_SIZE
WRITE_SIZE
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD TCP_TCC_READ_REQ_sum
SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT
SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INST_LEVEL_LDS SQ_IFETCH
SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE SQ_INSTS_LDS_LOAD_BANDWIDTH SQ_INSTS_LDS_STORE_BANDWIDTH SQ_IFETCH_LEVEL SQ_LEVEL_WAVES
LIST
echo "== done"
