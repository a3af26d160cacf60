set -u -o pipefail
for i in 1 2; do for k in 0 4 6; do
  cp gpurun_variants_liblcfir_k$k.so audio-fir-filter_amd/liblcfir.so || exit 1
  for c in "--config 5 --files 1 --force-exchange --steps 10 --warmup 3" "--config 5 --steps 5 --warmup 2" "--config 4 --files 1 --steps 10 --warmup 3"; do
    timeout -k 10 200 python bench.py $c --no-cpu-baseline --no-ingest --no-parity > gpurun_out/nrm.log 2>&1 || { tail -20 gpurun_out/nrm.log; exit 1; }
    echo "k$k $c :: $(grep '^{' gpurun_out/nrm.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"])')"
  done
done; done
