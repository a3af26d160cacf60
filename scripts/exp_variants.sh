#!/bin/bash
# Time alternative builds of liblcfir.so (abvar/*.so) with bench.py,
# parity leg on (rms vs the long-double oracle is printed per run).  Each
# variant is copied over the package library and the original restored.
set -u -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
cp audio-fir-filter_amd/liblcfir.so /tmp/liblcfir_orig.so
for rep in 1 2; do
for so in abvar/*.so; do
    cp "$so" audio-fir-filter_amd/liblcfir.so
    out=$(timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline "$@" 2>gpurun_out/variant_err.log | grep '^{')
    rc=$?
    if [ $rc -ne 0 ]; then echo "!! $so failed rc=$rc"; tail -5 gpurun_out/variant_err.log; cp /tmp/liblcfir_orig.so audio-fir-filter_amd/liblcfir.so; exit $rc; fi
    echo "$(basename $so) rep$rep $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"], d.get("parity"))')"
done
done
cp /tmp/liblcfir_orig.so audio-fir-filter_amd/liblcfir.so
