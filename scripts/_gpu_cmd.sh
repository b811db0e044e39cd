mkdir -p gpurun_out/ab
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_attack_cli.py -k debug -m gpu > gpurun_out/ab/pytest_cli.log 2>&1 && echo cli ok
