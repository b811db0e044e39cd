mkdir -p gpurun_out/ab
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests -m gpu > gpurun_out/ab/pytest_all.log 2>&1 && echo all ok \
&& timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ab/smoke.log 2>&1 && echo smoke ok
