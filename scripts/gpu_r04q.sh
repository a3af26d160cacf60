#!/bin/bash
# Round 4, the late-wait register kernel as the product: every BASELINE
# config at N = 1, the N = 8 per-rank steps of configs 4 and 5 alternated,
# and phase traces (product, timing-only no-store build, fused normalize).
set -u -o pipefail
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r04q; mkdir -p "$OUT"
step() { local name=$1 t=$2; shift 2; echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  tail -1 "$OUT/$name.log" | cut -c1-200
  if [ $rc -ne 0 ]; then echo "!! $name rc=$rc"; tail -30 "$OUT/$name.log"; exit $rc; fi; }
step bench_c1 300 python bench.py --config 1 --steps 20 --warmup 5 --no-cpu-baseline
step bench_c3 300 python bench.py --config 3 --steps 20 --warmup 5 --no-cpu-baseline
step bench_c4 600 python bench.py --config 4 --steps 20 --warmup 3 --no-cpu-baseline
step bench_c5 600 python bench.py --config 5 --steps 20 --warmup 3 --no-cpu-baseline
for r in 1 2; do
step c4f1_$r 300 python bench.py --config 4 --files 1 --steps 10 --warmup 3 --no-cpu-baseline
step c5f1x_$r 300 python bench.py --config 5 --files 1 --force-exchange --steps 10 --warmup 3 --no-cpu-baseline
done
T=audio-fir-filter_amd/tools/fft32r_trace
step trace 60 $T 4001 32768
step trace_nost 60 ${T}_nost 4001 32768
step trace_nrm 60 $T 4001 32768 sym nrm
step trace_8001 60 $T 8001 32768
echo "== done"
