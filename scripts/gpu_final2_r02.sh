#!/bin/bash
# Round-2 final check: full GPU suite, smoke, default bench line (config 2 with CPU baseline and the full run),
# configs 4 and 5, and a rocprofv3 kernel trace of config 2.  Steps chained, each with its own limit.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest ok" \
&& timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo "smoke ok" \
&& timeout -k 10 600 python bench.py > gpurun_out/bench_c2_final.log 2>&1 && echo "bench c2 ok" \
&& timeout -k 10 300 python bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1 && echo "bench c4 ok" \
&& timeout -k 10 300 python bench.py --config 5 --steps 6 --warmup 2 --no-cpu-baseline --full-run 0 > gpurun_out/bench_c5.log 2>&1 && echo "bench c5 ok" \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --full-run 0 > gpurun_out/prof_c2.log 2>&1 && echo "prof c2 ok"
rc=$?
tail -2 gpurun_out/pytest_gpu.log; tail -1 gpurun_out/smoke.log
for f in bench_c2_final bench_c4 bench_c5; do grep '^{"metric"' gpurun_out/$f.log | tail -1 | cut -c1-260; echo; done
exit $rc
