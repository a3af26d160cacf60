#!/bin/bash
# GPU box: direct kernel check -- the GPU tests that run the direct method,
# then bench lines (config 2 shape) for direct and FFT over a tap sweep and a
# rocprofv3 kernel-stats pass of the direct kernel.  Each GPU step has its own
# time limit; the first failure ends the script.
# usage (repo root, GPU box): bash scripts/gpu_direct_ab.sh <tag> [taps...]
set -u -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-direct}; shift || true
TAPS=${*:-15 47 95 255 1001}
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
    r=d['roofline']; p=d.get('parity',{})
    print(d['value'], d['ms_per_step'], r.get('kernel_ms'), r['frac'], r.get('kernel'), p)" 2>/dev/null
    if [ $rc -ne 0 ]; then echo "!! $name failed rc=$rc"; tail -30 "$OUT/$name.log"; exit $rc; fi
}
step pytest_direct 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "alignment or direct or golden or fuzz or tie or edge or config2"
for T in $TAPS; do
    for M in direct fft; do
        step "bench_${M}_T$T" 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ingest \
            --method $M --ntaps $T
    done
done
cd /tmp && export TMPDIR=/tmp
step rocprof_direct 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o bench -- \
    python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-parity --no-ingest --method direct --ntaps 47
echo "== done"
