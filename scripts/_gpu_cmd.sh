mkdir -p gpurun_out/ab
V=scripts/variants
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
ICA_HIP_LIB=$V/libup3g.so timeout -k 10 400 $T tests/test_gpu_kernels.py tests/test_gpu_split.py tests/test_gpu_x6.py -k "up3 or x6" -m gpu > gpurun_out/ab/pytest_up3g.log 2>&1 && echo tests ok \
&& bash scripts/gpu_ab.sh scripts/kbench_x6.py "up3" base $V/libup3g.so > gpurun_out/ab/up3g.log 2>&1 && echo ab ok
