mkdir -p gpurun_out/ab
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 400 $T -s tests/test_gpu_cheng.py -k float64 -m gpu > gpurun_out/ab/pytest_f64.log 2>&1 && echo f64 ok && timeout -k 10 900 $T tests -m gpu > gpurun_out/ab/pytest_all.log 2>&1 && echo all ok
