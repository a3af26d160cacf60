set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
LCFIR_FFT_LOG2M=12 timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "fft or smoke" > gpurun_out/pytest12.log 2>&1; echo "pytest12 rc=$?"; tail -3 gpurun_out/pytest12.log
for m in 12 13 12 13; do
LCFIR_FFT_LOG2M=$m timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_m$m.log 2>&1 || exit 1
echo "m=$m $(grep -o '"value": [0-9.]*' gpurun_out/bench_m$m.log) $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/bench_m$m.log) $(grep -o '"rms_vs_longdouble": [0-9.e-]*' gpurun_out/bench_m$m.log)"
done
