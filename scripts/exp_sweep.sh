set -u -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for s in 60 300 600 1800 3600; do
  timeout -k 10 300 python bench.py --seconds $s --steps 20 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/sweep_$s.log 2>&1 || exit 1
  echo "sec=$s $(grep '^{' gpurun_out/sweep_$s.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["kernel_ms"])')"
done
