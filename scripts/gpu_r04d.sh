#!/bin/bash
# bare `bench.py --gpus N` launches rehearsed on one GPU (ranks share it over gloo):
# N = 8 config 2 (one file per rank), N = 8 config 5 (8 files, per-file peaks + exchange),
# N = 4 config 4 with 2 files (files split over ranks: the halo windows + peak exchange)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r04d; mkdir -p $OUT
export LCFIR_BENCH_SHARE_DEVICE=1
run() { local name=$1; shift
  timeout -k 10 280 python bench.py "$@" > $OUT/$name.log 2>&1 || { echo "!! $name"; tail -20 $OUT/$name.log; exit 1; }
  grep '^{' $OUT/$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["n_gpus"], c["workload"][:40], c["files"], c["peak_exchange"], d["value"], d["ms_per_step"], d["parity"]["rms_vs_longdouble"])'
}
run c2_n8 --gpus 8 --steps 10 --warmup 2 --preroll-s 1 --no-ingest
run c5_n8 --gpus 8 --config 5 --seconds 600 --steps 5 --warmup 1 --preroll-s 1 --no-ingest
run c4_n4_split --gpus 4 --config 4 --files 2 --seconds 300 --steps 5 --warmup 1 --preroll-s 1 --no-ingest
