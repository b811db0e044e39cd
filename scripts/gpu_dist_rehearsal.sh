#!/bin/bash
# N > 1 rehearsal on a one-GPU box: two ranks (gloo, both on GPU 0) through the driver's launch line, config 2
# (image shard, no data-path collective) and config 4 (one flat gradient all-reduce per outer step).
set -o pipefail
mkdir -p gpurun_out
export ICA_BENCH_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --full-run 0 > gpurun_out/dist_c2.log 2>&1 && echo "dist c2 ok" \
&& timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --config 4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/dist_c4.log 2>&1 && echo "dist c4 ok"
rc=$?
grep '^{"metric"' gpurun_out/dist_c2.log | cut -c1-300; grep '^{"metric"' gpurun_out/dist_c4.log | cut -c1-300
exit $rc
