#!/bin/bash
# rocprofv3 kernel-trace summary of the config-5 (bf16, 2048x2048 ROI) and config-2 benches.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python bench.py --config 5 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c5.log 2>&1 && echo "prof c5 ok" \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2 -o run -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c2.log 2>&1 && echo "prof c2 ok" \
&& timeout -k 10 400 python bench.py --config 5 --steps 6 --warmup 2 > gpurun_out/bench_c5_cpu.log 2>&1 && echo "bench c5 (with cpu baseline) ok"
rc=$?
tail -1 gpurun_out/prof_c5.log | cut -c1-300; tail -1 gpurun_out/bench_c5_cpu.log | cut -c1-300
exit $rc
