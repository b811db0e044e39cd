#!/bin/bash
# Round-2 GPU check: gpu tests (new ones first), smoke, bench.  Each GPU step has its own time limit; steps
# are chained so the first failure stops the run.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="${TESTS:-tests}"
timeout -k 10 900 python -u -m pytest $T -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest ok" \
&& timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo "smoke ok" \
&& timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 && echo "bench ok"
rc=$?
grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3; tail -2 gpurun_out/smoke.log; tail -1 gpurun_out/bench.log | cut -c1-600
exit $rc
