#!/bin/bash
# Time alternative builds of liblcfir.so (gpurun_variants/*.so) with bench.py.
# Each variant is copied over the package library in a scratch copy of the
# package dir, so the tree's own liblcfir.so is left alone.
set -u -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
cp audio-fir-filter_amd/liblcfir.so /tmp/liblcfir_orig.so
for so in gpurun_variants/*.so; do
    cp "$so" audio-fir-filter_amd/liblcfir.so
    for rep in 1 2; do
        out=$(timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-parity "$@" 2>/dev/null | grep '^{')
        rc=$?
        if [ $rc -ne 0 ]; then echo "!! $so failed rc=$rc"; cp /tmp/liblcfir_orig.so audio-fir-filter_amd/liblcfir.so; exit $rc; fi
        echo "$(basename $so) rep$rep $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
    done
done
cp /tmp/liblcfir_orig.so audio-fir-filter_amd/liblcfir.so
