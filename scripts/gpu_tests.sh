#!/bin/bash
# GPU box: smoke, then the GPU test suite (per-test time limits), then the
# driver-shaped bench line.  The first failing step ends the script.
set -u -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-suite}"
mkdir -p "$OUT"
shift || true
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "!! smoke"; tail -30 "$OUT/smoke.log"; exit 1; }
tail -2 "$OUT/smoke.log"
timeout -k 10 1500 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread "$@" > "$OUT/pytest.log" 2>&1
rc=$?
grep -E "passed|failed|FAILED|ERROR" "$OUT/pytest.log" | tail -15
[ $rc -eq 0 ] || { echo "!! pytest rc=$rc"; exit $rc; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "!! bench"; tail -20 "$OUT/bench.err"; exit 1; }
tail -c 1500 "$OUT/bench.json"
