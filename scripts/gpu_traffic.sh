#!/bin/bash
# PMC traffic sidecar for one bench configuration: FETCH_SIZE, WRITE_SIZE and
# the f64 VALU counts, each its own rocprofv3 --pmc pass, then
# scripts/pmc_summary.py + scripts/make_traffic_json.py -> profiles/traffic_<tag>.json.
# usage: bash scripts/gpu_traffic.sh <tag> <ntaps> <samples_per_launch> [bench args...]
# (SEG_LEN=32768 KERNEL=fir_fft32_f64_kernel for the long segment;
#  METHOD=direct KERNEL=fir_direct_f64_kernel with --method direct)
set -u -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1 NTAPS=$2 SPL=$3; shift 3
OUT="$ROOT/gpurun_out/pmc_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for c in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64"; do
    i=$((i+1))
    echo "== pass $i: $c ($(date +%T))"
    timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex 'fir_' -f csv -d "$OUT/p_$i" -o pmc -- \
        python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-parity "$@" > "$OUT/p_$i.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "!! pass $i rc=$rc"; tail -20 "$OUT/p_$i.log"; exit $rc; fi
done
cd "$ROOT"
python scripts/pmc_summary.py "$OUT" --json "$OUT/summary.json" > /dev/null &&
python scripts/make_traffic_json.py "$OUT/summary.json" "$ROOT/gpurun_out/traffic_$TAG.json" --method "${METHOD:-fft}" \
    --ntaps "$NTAPS" --samples-per-launch "$SPL" --kernel "${KERNEL:-fir_fft_f64_kernel}" --seg-len "${SEG_LEN:-16384}"
