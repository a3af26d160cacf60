#!/bin/bash
# Round 4, final product: configs 1, 3, 4, 5 at N = 1 (config 2 in r04y).
set -u -o pipefail
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r04z; mkdir -p "$OUT"
for c in "1 --steps 20 --warmup 5" "3 --steps 20 --warmup 5" "4 --steps 20 --warmup 3" "5 --steps 20 --warmup 3"; do
  n=$(echo $c | cut -c1)
  timeout -k 10 400 python bench.py --config $c --no-cpu-baseline > "$OUT/bench_c$n.log" 2>&1 || { tail "$OUT/bench_c$n.log"; exit 1; }
  grep '^{' "$OUT/bench_c$n.log" | cut -c1-160
done
echo "== done"
