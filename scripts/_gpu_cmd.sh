mkdir -p gpurun_out/ab
export TMPDIR=/tmp
V=scripts/variants
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -s"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cheng.py tests/test_gpu_mbt.py -m gpu > gpurun_out/ab/pytest_cheng2.log 2>&1 && echo cheng ok; \
bash scripts/gpu_ab.sh scripts/kbench_x6.py "x6 " base $V/librcp.so > gpurun_out/ab/rcp.log 2>&1 && echo ab ok \
&& ICA_HIP_LIB=$V/librcp.so timeout -k 10 600 $T tests/test_traj100.py tests/test_gpu_x6.py -m gpu > gpurun_out/ab/pytest_rcp.log 2>&1 && echo rcp tests ok; \
timeout -k 10 700 python scripts/cheng_seed_sweep.py 24 > gpurun_out/ab/cheng_sweep.log 2>&1 && echo sweep ok
