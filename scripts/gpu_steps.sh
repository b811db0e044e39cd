#!/bin/bash
# Run GPU steps in order, each under its own time limit, each writing gpurun_out/<dir>/<name>.log.  A step that
# fails its checks (exit 1, e.g. a pytest assertion) does not stop the run; a time limit, abort, segfault or any
# other signal exit does (no further GPU step after a fault or a hang).
#   bash scripts/gpu_steps.sh <dir> "<name>|<seconds>|<command>" ...
set -o pipefail
D=gpurun_out/$1
shift
mkdir -p "$D"
export TMPDIR=/tmp
for s in "$@"; do
  name=${s%%|*}; rest=${s#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  echo "== $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "$D/$name.log" 2>&1
  rc=$?
  echo "   rc=$rc; $(tail -1 "$D/$name.log" | cut -c1-300)"
  if [ $rc -ge 2 ] && [ $rc -ne 5 ]; then
    echo "   stopping: rc $rc"
    exit $rc
  fi
done
exit 0
