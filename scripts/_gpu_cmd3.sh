mkdir -p gpurun_out/ab
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_cheng.py tests/test_gpu_mbt.py tests/test_gpu_x6.py tests/test_gpu_headline.py -m gpu > gpurun_out/ab/pytest_cheng.log 2>&1 && echo cheng tests ok; \
timeout -k 10 600 python scripts/cheng_seed_sweep.py 24 > gpurun_out/ab/cheng_sweep.log 2>&1 && echo sweep ok; \
timeout -k 10 600 python bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab/bench_c3x.log 2>&1 && echo c3 ok \
&& timeout -k 10 600 python bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab/bench_c4.log 2>&1 && echo c4 ok
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
V=scripts/variants
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
bash scripts/gpu_ab.sh scripts/kbench_x6.py "x6 down" base $V/libpf2022.so $V/libpf1821.so > gpurun_out/ab/down_pf.log 2>&1 && echo ab ok \
&& ICA_HIP_LIB=$V/libpf2022.so timeout -k 10 300 $T tests/test_gpu_x6.py -m gpu > gpurun_out/ab/pytest_pf.log 2>&1 && echo pf tests ok
