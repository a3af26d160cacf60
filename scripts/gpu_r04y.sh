#!/bin/bash
# Round 4, final product (pair table's second half entry by entry): smoke,
# GPU suite, config-2 line, rocprofv3 trace + PMC, the config-4 / config-5
# per-rank steps, a seeded fuzz campaign.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT}"
bash scripts/gpu_check.sh r04y --steps 20 --warmup 5 || exit 1
OUT=gpurun_out/r04y; mkdir -p "$OUT"
for c in "4 --files 1" "5 --files 1 --force-exchange"; do
  n=$(echo $c | cut -c1)
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/c${n}f1.log" 2>&1 || { tail "$OUT/c${n}f1.log"; exit 1; }
  grep '^{' "$OUT/c${n}f1.log" | cut -c1-200
done
FUZZ_TIMEOUT=300 bash scripts/gpu_fuzz.sh 60000 3000 800 r04y || exit 1
echo "== all done"
