#!/bin/bash
# GPU-box run: parity tests (bf16 first), full GPU suite, bench fp32 (config 2) and bf16 (config 5).
# Each GPU step has its own time limit; steps are chained so the first failure stops the run.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_bf16.py -m gpu > gpurun_out/pytest_bf16.log 2>&1 && echo "bf16 tests ok" \
&& timeout -k 10 900 $T tests -m gpu > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest ok" \
&& timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1 && echo "bench ok" \
&& timeout -k 10 300 python bench.py --config 5 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1 && echo "bench c5 ok"
rc=$?
tail -3 gpurun_out/pytest_bf16.log; tail -3 gpurun_out/pytest_gpu.log; tail -1 gpurun_out/bench.log; tail -1 gpurun_out/bench_c5.log
exit $rc
