#!/bin/bash
# GPU box: config 2 eager (default) vs HIP-graph replays, alternating, three
# repetitions each; bench lines only (no CPU baseline, no ingest probe).
set -u -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-graphc2}"
mkdir -p "$OUT"
for rep in 1 2 3; do
    for g in off on; do
        timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ingest --graph $g \
            > "$OUT/g${g}_$rep.log" 2>&1 || { echo "!! $g $rep"; tail -20 "$OUT/g${g}_$rep.log"; exit 1; }
        grep '^{' "$OUT/g${g}_$rep.log" | tail -1 | python3 -c "import sys,json
d=json.loads(sys.stdin.read()); r=d['roofline']
print('$g', $rep, d['value'], d['ms_per_step'], r['kernel_ms'], d['config'].get('hip_graph'))"
    done
done
