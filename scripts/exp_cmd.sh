set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_exp.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_exp.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_exp$i.log 2>&1 || exit 1
echo "run$i $(grep -o '"value": [0-9.]*' gpurun_out/bench_exp$i.log) $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/bench_exp$i.log) $(grep -o '"rms_vs_longdouble": [0-9.e-]*' gpurun_out/bench_exp$i.log)"
done
