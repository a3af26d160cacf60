#!/bin/bash
# Round 4: config 5 on the register kernel with the 16-block normalize halves
# (a 60-min file's 15 blocks per half were over the 14-block cap, so every
# normalize ran as its own pass): parity tests, then c4f1 / c5f1x alternated.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r04k; mkdir -p "$OUT"
step() { local name=$1 t=$2; shift 2; echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  tail -1 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "!! $name rc=$rc"; tail -30 "$OUT/$name.log"; exit $rc; fi; }
step tests 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_baseline_configs.py tests/test_gpu_batch.py -k "configs_4_and_5 or norm or exchange or defer"
for r in 1 2; do
step c4f1_$r 300 python bench.py --config 4 --files 1 --steps 10 --warmup 3 --no-cpu-baseline
step c5f1x_$r 300 python bench.py --config 5 --files 1 --force-exchange --steps 10 --warmup 3 --no-cpu-baseline
done
step bench_c5 600 python bench.py --config 5 --steps 20 --warmup 3 --no-cpu-baseline
T=audio-fir-filter_amd/tools/fft32r_trace
step trace_4001 120 $T 4001 32768
step trace_4001_nrm 120 $T 4001 32768 sym nrm
step trace_8001 120 $T 8001 32768
cp "$OUT"/trace_*.log "$OUT/.." 2>/dev/null; echo "== done"
