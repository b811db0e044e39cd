mkdir -p gpurun_out/ab
export TMPDIR=/tmp
bash scripts/gpu_evidence.sh c2 32 512 768 x6 --mixed 40 \
&& timeout -k 10 600 python bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab/bench_c3.log 2>&1 && echo c3 ok \
&& timeout -k 10 600 python bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab/bench_c4.log 2>&1 && echo c4 ok
