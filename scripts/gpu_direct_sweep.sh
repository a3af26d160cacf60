#!/bin/bash
# GPU box: direct vs FFT bench lines (config-2 shape) over a tap sweep on the
# final kernels.  Each GPU step has its own time limit; the first failure ends
# the script.  usage: bash scripts/gpu_direct_sweep.sh <tag> [taps...]
set -u -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-sweep}; shift || true
TAPS=${*:-15 31 47 63 79 95 127 255 1001 4001}
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
for T in $TAPS; do
    for M in direct fft; do
        [ "$M" = direct ] && [ "$T" -gt 1001 ] && steps=5 || steps=20
        timeout -k 10 300 python bench.py --steps $steps --warmup 2 --no-cpu-baseline --no-ingest --method $M --ntaps $T \
            > "$OUT/bench_${M}_T$T.log" 2>&1 || { echo "!! $M $T"; tail -20 "$OUT/bench_${M}_T$T.log"; exit 1; }
        grep '^{' "$OUT/bench_${M}_T$T.log" | tail -1 | python3 -c "import sys,json
d=json.loads(sys.stdin.read()); r=d['roofline']; p=d['parity']
print('$M', $T, d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], p['rms_vs_longdouble'], p['max_ulp'])"
    done
done
