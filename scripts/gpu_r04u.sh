#!/bin/bash
# Round 4: config 2 with 2 / 3 / 4 lanes (streams the consecutive steps
# alternate over), alternating, driver-shaped.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r04u; mkdir -p "$OUT"
for r in 1 2; do for l in 2 3 4; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ingest --lanes $l > "$OUT/c2_l${l}_$r.log" 2>&1 || { tail "$OUT/c2_l${l}_$r.log"; exit 1; }
  echo "lanes $l rep $r $(grep '^{' "$OUT/c2_l${l}_$r.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["kernel_ms"], r["frac_step"])')"
done; done
echo "== done"
