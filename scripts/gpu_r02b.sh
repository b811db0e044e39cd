#!/bin/bash
# Round-2 state check on a fresh box: GPU tests, smoke, bench config 2 (default line), bench config 5 (bf16),
# rocprof kernel stats of the config-2 and config-5 benches.  Each GPU step has its own time limit; steps are
# chained so the first failure stops the run.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P="${PREFIX:-r02b}"
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest ok" \
&& timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo "smoke ok" \
&& timeout -k 10 600 python bench.py > gpurun_out/bench_c2.log 2>&1 && echo "bench c2 ok" \
&& timeout -k 10 300 python bench.py --config 5 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1 && echo "bench c5 ok" \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --full-run 0 > gpurun_out/prof_c2.log 2>&1 && echo "prof c2 ok" \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run -- python3 bench.py --config 5 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/prof_c5.log 2>&1 && echo "prof c5 ok"
rc=$?
grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3; tail -2 gpurun_out/smoke.log
tail -1 gpurun_out/bench_c2.log | cut -c1-400; tail -1 gpurun_out/bench_c5.log | cut -c1-400
exit $rc
