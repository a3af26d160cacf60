#!/bin/bash
# Round 4, the tree as committed: smoke, GPU suite, driver-shaped config-2 line.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r04w; mkdir -p "$OUT"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail "$OUT/smoke.log"; exit 1; }
tail -2 "$OUT/smoke.log"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/suite.log" 2>&1 || { tail -30 "$OUT/suite.log"; exit 1; }
tail -1 "$OUT/suite.log"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || { tail "$OUT/bench.log"; exit 1; }
grep '^{' "$OUT/bench.log" | cut -c1-400
echo "== done"
