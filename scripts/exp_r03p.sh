#!/bin/bash
# round 3: parity + fuzz suites, then config 2 (x3) and 4 003 taps in both pair-table forms
set -u -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/r03p_t.log 2>&1 || { tail -30 gpurun_out/r03p_t.log; exit 1; }
tail -1 gpurun_out/r03p_t.log
line() { grep "^{" "$1" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["kernel_ms"], r["frac"], d["config"]["fft_plan"], d["parity"]["rms_vs_longdouble"])'; }
for i in 1 2 3; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03p_c2_$i.log 2>&1 || exit 1
    echo "c2 $i: $(line gpurun_out/r03p_c2_$i.log)"
done
for f in "" "--general-form"; do
    timeout -k 10 200 python bench.py --ntaps 4003 $f --steps 20 --warmup 5 --no-cpu-baseline --no-ingest > gpurun_out/r03p_4003.log 2>&1 || exit 1
    echo "4003 $f: $(line gpurun_out/r03p_4003.log)"
done
