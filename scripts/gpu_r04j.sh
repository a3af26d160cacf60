#!/bin/bash
# Round 4, final kernel tree: every BASELINE config at N = 1 plus the N = 8
# per-rank steps of configs 4 and 5 (one file, forced exchange), alternated.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r04j; mkdir -p "$OUT"
step() { local name=$1 t=$2; shift 2; echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  tail -1 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "!! $name rc=$rc"; tail -30 "$OUT/$name.log"; exit $rc; fi; }
step bench_c2 300 python bench.py --steps 20 --warmup 5
step bench_c1 300 python bench.py --config 1 --steps 20 --warmup 5 --no-cpu-baseline
step bench_c3 300 python bench.py --config 3 --steps 20 --warmup 5 --no-cpu-baseline
step bench_c4 600 python bench.py --config 4 --steps 20 --warmup 3 --no-cpu-baseline
step bench_c5 600 python bench.py --config 5 --steps 20 --warmup 3 --no-cpu-baseline
for r in 1 2; do
step c4f1_$r 300 python bench.py --config 4 --files 1 --steps 10 --warmup 3 --no-cpu-baseline
step c5f1x_$r 300 python bench.py --config 5 --files 1 --force-exchange --steps 10 --warmup 3 --no-cpu-baseline
done
echo "== done"
