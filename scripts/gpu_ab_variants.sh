#!/bin/bash
# A/B of liblcfir.so builds (abvar/<name>.so), alternating on one box, each
# variant through bench.py with the given args; prints value, ms/step,
# exclusive kernel ms, frac and parity per run.  The product library is
# restored at the end.  usage: gpu_ab_variants.sh "<names>" <reps> <bench args...>
set -u -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
names=$1; reps=$2; shift 2
cp audio-fir-filter_amd/liblcfir.so /tmp/liblcfir_orig.so
for rep in $(seq 1 "$reps"); do
for v in $names; do
    cp "abvar/$v.so" audio-fir-filter_amd/liblcfir.so
    out=$(timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ingest "$@" 2>gpurun_out/ab_err.log | grep '^{')
    rc=$?
    if [ $rc -ne 0 ]; then echo "!! $v failed rc=$rc"; tail -5 gpurun_out/ab_err.log; cp /tmp/liblcfir_orig.so audio-fir-filter_amd/liblcfir.so; exit $rc; fi
    echo "$v rep$rep $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["kernel_ms"], r["frac"], d["parity"]["rms_vs_longdouble"], d["parity"]["max_ulp"])')"
done
done
cp /tmp/liblcfir_orig.so audio-fir-filter_amd/liblcfir.so
