#!/bin/bash
# Submit one gpurun call; if the pool has no free slot (gpurun's "transient"
# verdict: nothing ran, nothing charged) wait and submit again, at most N
# times (GPURUN_TRIES, default 8).  A call that ran -- whatever its exit status -- is never repeated.
# usage: bash scripts/gpurun_when_free.sh LOG TIMEOUT 'command'
LOG=$1; T=$2; CMD=$3
for i in $(seq 1 ${GPURUN_TRIES:-8}); do
    /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" > "$LOG" 2>&1
    rc=$?
    if grep -q "status=transient" "$LOG" && ! grep -q "status=ok\|status=fail" "$LOG"; then
        echo "try $i $(date +%T): pool busy, waiting" >> "$LOG.tries"
        sleep 150
        continue
    fi
    exit $rc
done
exit 3
