#!/bin/bash
# Parity + timing of an alternative liblcfir.so build: the FFT parity and fuzz
# tests with abvar/$1 in place, then scripts/exp_variants.sh over
# every abvar/*.so (remaining args go to bench.py).
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
v="$1"; shift
cp audio-fir-filter_amd/liblcfir.so /tmp/orig.so
cp "abvar/$v" audio-fir-filter_amd/liblcfir.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_fft_opt_in.py > gpurun_out/variant_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/variant_pytest.log
cp /tmp/orig.so audio-fir-filter_amd/liblcfir.so
[ $rc -ne 0 ] && exit $rc
bash scripts/exp_variants.sh "$@"
