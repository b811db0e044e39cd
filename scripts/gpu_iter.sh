#!/bin/bash
# One development iteration on the GPU box: the x6 parity subset (kernels, parity-split layout, headline shapes,
# reference-pinned 100-step trajectories), the default bench line and the x6 kernel bench.
#   bash scripts/gpu_iter.sh <tag>     -> gpurun_out/<tag>/{pytest,bench,kb}.log
set -o pipefail
O=gpurun_out/${1:-iter}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_x6.py tests/test_gpu_split.py tests/test_gpu_smallgrid.py tests/test_gpu_attack.py tests/test_gpu_headline.py tests/test_traj100.py -m gpu > $O/pytest.log 2>&1 && echo "pytest ok" \
&& timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --full-run 0 > $O/bench.log 2>&1 && echo "bench ok" \
&& timeout -k 10 300 python scripts/kbench_x6.py --only x6 > $O/kb.log 2>&1 && echo "kb ok"
