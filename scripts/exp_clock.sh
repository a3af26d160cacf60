#!/bin/bash
# Driver-shaped bench runs (--steps 20 --warmup 5) with and without the
# pre-roll, beside longer ones: does the short timed region sit in the
# shader-clock ramp?  Each GPU step has its own time limit; the first failure
# ends the script.
set -u -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/clock"
mkdir -p "$OUT"
run() { # name args...
    local name=$1; shift
    timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "!! $name rc=$?"; tail -20 "$OUT/$name.err"; exit 1; }
    python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
l = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = l["roofline"]
print(sys.argv[2], l["value"], l["ms_per_step"], "kernel", r["kernel_ms"], "ovl", r.get("overlapped_kernel_ms"),
      "frac", r["frac"], "lanes", l["config"].get("lanes"), "pre", l.get("preroll"), "par", l["parity"]["rms_vs_longdouble"], l["parity"].get("max_ulp"))
PY
}
for spec in "${@:-default}"; do :; done
run p0 --steps 20 --warmup 5 --preroll-s 0
run p05 --steps 20 --warmup 5 --preroll-s 0.5
run p1 --steps 20 --warmup 5 --preroll-s 1
run p2 --steps 20 --warmup 5
run p4 --steps 20 --warmup 5 --preroll-s 4
run p2_1lane --steps 20 --warmup 5 --lanes 1
run p2_500 --steps 500 --warmup 5
run p2b --steps 20 --warmup 5
