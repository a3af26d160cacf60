#!/bin/bash
# GPU box: FFT parity suites with the 4-wave kernel (LCFIR_FFT_WAVES=4), then the
# config-2 bench line with the 4-wave and the default 8-wave kernel alternately.
# usage: bash scripts/exp_waves4.sh <tag> [reps] [bench args...]
set -u -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-waves4}; REPS=${2:-2}; shift 2 || shift $#
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
LCFIR_FFT_WAVES=4 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py \
    -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
tail -3 "$OUT/pytest.log"
[ $rc -eq 0 ] || { echo "!! pytest rc=$rc"; grep -E "Error|assert|FAILED" "$OUT/pytest.log" | head -20; exit $rc; }
for r in $(seq 1 "$REPS"); do
    for wv in 4 8; do
        LCFIR_FFT_WAVES=$wv timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" \
            > "$OUT/bench_w${wv}_r$r.json" 2> "$OUT/bench_w${wv}_r$r.err" || { echo "!! bench w$wv"; tail -20 "$OUT/bench_w${wv}_r$r.err"; exit 1; }
        python - "$OUT/bench_w${wv}_r$r.json" "$wv" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][0])
r = d["roofline"]
print(f"waves {sys.argv[2]:>2}: {d['value']:.1f} Ms/s  step {d['ms_per_step']:.4f} ms  kernel {r['kernel_ms']:.4f} ms  "
      f"frac {r['frac']:.4f}  parity {d['parity']['rms_vs_longdouble']}")
PY
    done
done
