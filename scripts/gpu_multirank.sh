#!/bin/bash
# Rehearsal of bench.py's multi-rank path on a one-GPU box: ranks share the
# device (LCFIR_BENCH_SHARE_DEVICE=1 -> gloo), max-over-ranks timing, the
# peak exchange and the fused normalize's multi-file-per-rank case.  Each
# step has its own time limit; the first failure ends the script.
set -u -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
export LCFIR_BENCH_SHARE_DEVICE=1
step() { # name timeout cmd...
    local name=$1 t=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    grep '^{' "$OUT/$name.log" | cut -c1-400
    if [ $rc -ne 0 ]; then echo "!! $name failed rc=$rc"; tail -30 "$OUT/$name.log"; exit $rc; fi
}
run() { # name nproc bench-args...
    local name=$1 np=$2; shift 2
    step "$name" 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$np" \
        --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) bench.py --gpus "$np" "$@"
}
run mr_c2_n2 2 --steps 10 --warmup 2 --preroll-s 0.5
run mr_c4_n2 2 --config 4 --steps 3 --warmup 1 --preroll-s 0.5
run mr_c5_n2 2 --config 5 --steps 3 --warmup 1 --preroll-s 0.5
run mr_c4f1_n2 2 --config 4 --files 1 --steps 3 --warmup 1 --preroll-s 0.5
# round 3: config 5 at one file per rank (the N = 8 shape: exchange every step,
# each rescale deferred into the lane's next launch), and 8 ranks of config 2
run mr_c5f2_n2 2 --config 5 --files 2 --steps 4 --warmup 1 --preroll-s 0.5
run mr_c2_n8 8 --steps 6 --warmup 2 --preroll-s 0.5
echo "== done"
