#!/bin/bash
# cheng2020 on x6 operands: full GPU suite, smoke, config 3 and config 2 benches, rocprofv3 kernel trace of config 3.
# Steps chained, each with its own limit.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest ok" \
&& timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo "smoke ok" \
&& timeout -k 10 300 python bench.py --config 3 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 && echo "bench c3 ok" \
&& timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --full-run 0 > gpurun_out/bench_c2.log 2>&1 && echo "bench c2 ok" \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run -- python3 bench.py --config 3 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c3.log 2>&1 && echo "prof c3 ok"
rc=$?
tail -3 gpurun_out/pytest_gpu.log; for f in c3 c2; do grep -h '^{' gpurun_out/bench_$f.log | cut -c1-300; echo; done
exit $rc
