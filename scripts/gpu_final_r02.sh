#!/bin/bash
# Round-2 evidence on the final code: default bench line (config 2, CPU baseline, full 1001-step run) and rocprofv3
# kernel traces of configs 2, 4 and 5.  Steps chained, each with its own limit.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench_c2_final.log 2>&1 && echo "bench c2 ok" \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --full-run 0 > gpurun_out/prof_c2.log 2>&1 && echo "prof c2 ok" \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o run -- python3 bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c4.log 2>&1 && echo "prof c4 ok" \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run -- python3 bench.py --config 5 --steps 6 --warmup 2 --no-cpu-baseline --full-run 0 > gpurun_out/prof_c5.log 2>&1 && echo "prof c5 ok"
rc=$?
tail -1 gpurun_out/bench_c2_final.log | cut -c1-400
exit $rc
