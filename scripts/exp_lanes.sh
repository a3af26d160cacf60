#!/bin/bash
# bench.py value at --lanes 1 / 2 / 3, alternating, three repetitions (extra args go to bench.py)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for rep in 1 2 3; do
for l in 1 2 3; do
    out=$(timeout -k 10 300 python bench.py --steps 60 --warmup 5 --no-cpu-baseline --no-parity --lanes $l "$@" 2>gpurun_out/lanes_err.log | grep '^{') || { echo "lanes $l failed"; tail -5 gpurun_out/lanes_err.log; exit 1; }
    echo "lanes $l rep$rep $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"])')"
done
done
