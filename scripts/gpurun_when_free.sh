#!/bin/bash
# Submit one gpurun command, re-submitting only while the pool reports no free box / slot (status=transient: the
# command never started, nothing charged).  Any started run -- pass or fail -- is final.
#   bash scripts/gpurun_when_free.sh <timeout s> <log> '<command>'
T=$1; LOG=$2; CMD=$3
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout $T -- "$CMD" > $LOG 2>&1
  rc=$?
  grep -q "status=transient\|backing off" $LOG || exit $rc
  sleep 150
done
exit $rc
