#!/bin/bash
# A/B two builds of liblcfir.so on one box (gpurun_variants_A.so / _B.so at the
# repo root), alternating, driver-shaped config 2 lines.  usage: exp_ab_lib.sh [rounds] [bench args...]
set -u -o pipefail
n=${1:-3}; shift || true
mkdir -p gpurun_out
line() { grep "^{" "$1" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["kernel_ms"], r["frac"])'; }
for i in $(seq 1 "$n"); do for v in A B; do
    cp gpurun_variants_$v.so audio-fir-filter_amd/liblcfir.so || exit 1
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ingest "$@" > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
    echo "$v $i: $(line gpurun_out/ab.log)"
done; done
cp gpurun_variants_B.so audio-fir-filter_amd/liblcfir.so
