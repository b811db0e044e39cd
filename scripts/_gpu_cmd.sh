mkdir -p gpurun_out/ab
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_split.py tests/test_gpu_x6.py tests/test_gpu_headline.py -m gpu > gpurun_out/ab/pytest_up3.log 2>&1 && echo tests ok \
&& bash scripts/gpu_ab.sh scripts/kbench_x6.py "x6 up3" base > gpurun_out/ab/up3.log 2>&1 && echo kb ok \
&& timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --full-run 0 > gpurun_out/ab/bench_up3.log 2>&1 && echo bench ok
