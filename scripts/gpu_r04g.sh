#!/bin/bash
# chunked two-stream host-pointer pipeline: the drop-in GPU tests, then the timing tool
set -u -o pipefail
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r04g; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_cpp_dropin.py tests/test_abi.py -m gpu > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|ERROR" $OUT/pytest.log | tail -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 tests/cpp/dropin_bench --threads 1,16,ref --reps 3 --modes pageable,pinned,bounce > $OUT/dropin.log 2>&1 || { tail -5 $OUT/dropin.log; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/r04g/dropin.log"):
    if l.startswith("{"):
        d = json.loads(l); sp = d["split_per_call_ms"]
        print(d["mode"], d["threads"], d["msamples_per_s"], d["fanout_msamples_per_s"], d["fanout_h2d_bound_frac"], d["alloc_ms_per_file"], d["fanout_ms_per_file"], sp, d["bit_identical"])
PY
