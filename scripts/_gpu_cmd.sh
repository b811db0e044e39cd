mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -s"
timeout -k 10 600 $T tests/test_gpu_split.py -m gpu > gpurun_out/pytest_split.log 2>&1 && echo split ok \
&& timeout -k 10 900 $T tests/test_gpu_x6.py tests/test_traj100.py tests/test_gpu_headline.py tests/test_gpu_smallgrid.py tests/test_gpu_attack.py -m gpu > gpurun_out/pytest_x6.log 2>&1 && echo x6 tests ok \
&& bash scripts/gpu_ab.sh scripts/kbench_x6.py "x6" base > gpurun_out/kb_split.log 2>&1 && echo kb ok \
&& timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --full-run 0 > gpurun_out/bench_split.log 2>&1 && echo bench ok
