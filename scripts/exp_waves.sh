#!/bin/bash
# GPU box: the FFT parity suites on the default (16-wave) kernel, then the
# config-2 bench line with the 16-wave and the 8-wave (LCFIR_FFT_WAVES=8)
# kernel alternately.  The first failing step ends the script.
# usage: bash scripts/exp_waves.sh <tag> [reps] [bench args...]
set -u -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-waves}; REPS=${2:-2}; shift 2 || shift $#
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "!! smoke"; tail -30 "$OUT/smoke.log"; exit 1; }
tail -2 "$OUT/smoke.log"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_baseline_configs.py \
    -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
tail -5 "$OUT/pytest.log"
[ $rc -eq 0 ] || { echo "!! pytest rc=$rc"; grep -E "Error|assert" "$OUT/pytest.log" | head -20; exit $rc; }
for r in $(seq 1 "$REPS"); do
    for wv in 16 8; do
        LCFIR_FFT_WAVES=$wv timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" \
            > "$OUT/bench_w${wv}_r$r.json" 2> "$OUT/bench_w${wv}_r$r.err" || { echo "!! bench w$wv"; tail -20 "$OUT/bench_w${wv}_r$r.err"; exit 1; }
        python - "$OUT/bench_w${wv}_r$r.json" "$wv" <<'EOF'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][0])
r = d["roofline"]
print(f"waves {sys.argv[2]:>2}: {d['value']:.1f} Ms/s  step {d['ms_per_step']:.4f} ms  kernel {r['kernel_ms']:.4f} ms  "
      f"frac {r['frac']:.4f}  parity {d['parity']['rms_vs_longdouble']}")
EOF
    done
done
