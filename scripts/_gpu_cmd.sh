mkdir -p gpurun_out/ab
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests -m gpu > gpurun_out/ab/pytest_all.log 2>&1 && echo all ok \
&& timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ab/smoke.log 2>&1 && echo smoke ok \
&& timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --full-run 0 > gpurun_out/ab/bench_quick.log 2>&1 && echo bench ok && \
ICA_BENCH_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --full-run 0 > gpurun_out/ab/bench_2rank.log 2>&1 && echo 2rank ok
