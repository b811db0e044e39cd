#!/bin/bash
# bf16 kernel experiment on the GPU box: bf16 parity tests, phase trace, per-kernel timings at config-5 shapes,
# config-5 bench.  Each GPU step has its own time limit; steps chained so the first failure stops the run.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_bf16.log 2>&1 && echo "bf16 tests ok" \
&& timeout -k 10 200 python scripts/exp/bf_trace.py run > gpurun_out/bf_trace.log 2>&1 && echo "trace ok" \
&& timeout -k 10 200 python scripts/kbench_bf16.py > gpurun_out/kbench_bf16.log 2>&1 && echo "kbench ok" \
&& timeout -k 10 300 python bench.py --config 5 --steps 6 --warmup 2 --no-cpu-baseline --full-run 0 > gpurun_out/bench_c5.log 2>&1 && echo "bench c5 ok"
rc=$?
tail -3 gpurun_out/pytest_bf16.log; cat gpurun_out/bf_trace.log gpurun_out/kbench_bf16.log | grep -v amdgpu.ids; tail -1 gpurun_out/bench_c5.log | cut -c1-300
exit $rc
