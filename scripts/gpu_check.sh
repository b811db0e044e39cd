#!/bin/bash
# GPU-box check: parity tests, smoke, bench, rocprof kernel stats.  Each GPU step
# has its own time limit; steps are chained so the first failure stops the run.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest ok" \
&& timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo "smoke ok" \
&& timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1 && echo "bench ok" \
&& timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1 && echo "prof ok"
rc=$?
tail -3 gpurun_out/pytest_gpu.log; cat gpurun_out/smoke.log | tail -3; tail -2 gpurun_out/bench.log
exit $rc
