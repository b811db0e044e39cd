#!/bin/bash
# cheng2020 (configs[2] per-GPU shard) bench + kernel trace on the GPU box.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python bench.py --model cheng2020 --steps 6 --warmup 2 --cpu-seconds 10 > gpurun_out/bench_cheng.log 2>&1 && echo "cheng bench ok" \
&& timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cheng -o run -- python bench.py --model cheng2020 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_cheng.log 2>&1 && echo "cheng prof ok"
rc=$?
tail -2 gpurun_out/bench_cheng.log
exit $rc
