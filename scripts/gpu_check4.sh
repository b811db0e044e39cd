#!/bin/bash
# Full GPU suite + config 4 / 2 / 5 benches.  Steps chained, each with its own limit.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest ok" \
&& timeout -k 10 300 python bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1 && echo "bench c4 ok" \
&& timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --full-run 0 > gpurun_out/bench_c2.log 2>&1 && echo "bench c2 ok" \
&& timeout -k 10 300 python bench.py --config 5 --steps 6 --warmup 2 --no-cpu-baseline --full-run 0 > gpurun_out/bench_c5.log 2>&1 && echo "bench c5 ok"
rc=$?
tail -3 gpurun_out/pytest_gpu.log; for f in c4 c2 c5; do tail -1 gpurun_out/bench_$f.log | cut -c1-300; echo; done
exit $rc
