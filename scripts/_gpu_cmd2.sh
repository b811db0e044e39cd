mkdir -p gpurun_out/ab
export TMPDIR=/tmp
V=scripts/variants
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
bash scripts/gpu_ab.sh scripts/kbench_x6.py "x6 down" base $V/libpf2022.so $V/libpf1821.so > gpurun_out/ab/down_pf.log 2>&1 && echo ab ok \
&& ICA_HIP_LIB=$V/libpf2022.so timeout -k 10 300 $T tests/test_gpu_x6.py -m gpu > gpurun_out/ab/pytest_pf.log 2>&1 && echo pf tests ok
