#!/bin/bash
# GPU-box run of this round's parity gate and evidence: the new parity tests first (reference-pinned 100-step
# trajectories on both operand paths, the INTEGRATION stub, the headline shapes), then the whole GPU suite, smoke,
# and the default bench line.  Each GPU step has its own time limit; steps are chained so the first failure stops.
#   bash scripts/gpu_round.sh [fast]     (fast: skip the full suite)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -s"
timeout -k 10 600 $T tests/test_traj100.py tests/test_gpu_integration.py tests/test_gpu_headline.py -m gpu > gpurun_out/pytest_new.log 2>&1 && echo "new tests ok" \
&& { [ "$1" = fast ] || { timeout -k 10 1200 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest ok"; }; } \
&& timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo "smoke ok" \
&& timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --full-run 0 > gpurun_out/bench_c2.log 2>&1 && echo "bench ok"
rc=$?
grep -h "identical for\|noise after\|final noise\|round differently" gpurun_out/pytest_new.log
tail -3 gpurun_out/pytest_new.log; tail -3 gpurun_out/pytest_gpu.log 2>/dev/null; tail -1 gpurun_out/smoke.log; tail -1 gpurun_out/bench_c2.log | cut -c1-400
exit $rc
