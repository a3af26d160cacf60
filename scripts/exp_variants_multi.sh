#!/bin/bash
# GPU box: N builds of liblcfir.so (gpurun_var_<name>.so at the repo root),
# alternating, bench lines for each bench-args set.  The first build named is
# restored at the end.
# usage: exp_variants_multi.sh "<names>" <rounds> "<bench args>" ["<bench args>" ...]
set -u -o pipefail
names=$1 rounds=$2; shift 2
mkdir -p gpurun_out
line() { grep "^{" "$1" | tail -1 | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; p=d.get("parity",{}); print(d["value"], d["ms_per_step"], r["kernel_ms"], r["frac"], d["config"].get("fft_plan"), p.get("max_ulp"))'; }
for args in "$@"; do
    echo "== $args"
    for i in $(seq 1 "$rounds"); do for v in $names; do
        cp "gpurun_var_$v.so" audio-fir-filter_amd/liblcfir.so || exit 1
        timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ingest $args > gpurun_out/var.log 2>&1 \
            || { tail -20 gpurun_out/var.log; exit 1; }
        echo "$v $i: $(line gpurun_out/var.log)"
    done; done
done
first=${names%% *}
cp "gpurun_var_$first.so" audio-fir-filter_amd/liblcfir.so
