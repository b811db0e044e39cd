mkdir -p gpurun_out/ab
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_split.py tests/test_gpu_defend_adv.py tests/test_gpu_bf16.py -m gpu > gpurun_out/ab/pytest_split3.log 2>&1 && echo split ok; \
timeout -k 10 300 $T tests/test_gpu_ar_coding.py -m gpu > gpurun_out/ab/pytest_ar.log 2>&1 && echo ar ok; \
timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab/bench_c5b.log 2>&1 && echo c5 ok \
&& timeout -k 10 300 python bench.py --precision fp32 --steps 10 --warmup 2 --no-cpu-baseline --full-run 0 > gpurun_out/ab/bench_fp32b.log 2>&1 && echo fp32 ok \
&& timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --full-run 0 > gpurun_out/ab/bench_c2b.log 2>&1 && echo c2 ok
