#!/bin/bash
# End-of-round evidence run: full GPU suite, smoke, both benches with the CPU baseline, rocprof kernel-trace
# summaries of the same bench commands, PMC traffic passes for config 5.  One time limit per step, chained.
set -o pipefail
mkdir -p gpurun_out/final
export TMPDIR=/tmp
O=gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && echo "pytest ok" \
&& timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo "smoke ok" \
&& timeout -k 10 600 python bench.py > $O/bench_c2.log 2>&1 && echo "bench c2 ok" \
&& timeout -k 10 600 python bench.py --config 5 > $O/bench_c5.log 2>&1 && echo "bench c5 ok" \
&& timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python bench.py --no-cpu-baseline > $O/prof_c2.log 2>&1 && echo "prof c2 ok" \
&& timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python bench.py --config 5 --no-cpu-baseline > $O/prof_c5.log 2>&1 && echo "prof c5 ok" \
&& PMC_TAG=final/pmc_c5 timeout -k 10 900 bash scripts/gpu_pmc.sh --config 5 > $O/pmc_c5.log 2>&1 && echo "pmc c5 ok" \
&& PMC_TAG=final/pmc_c2 timeout -k 10 900 bash scripts/gpu_pmc.sh > $O/pmc_c2.log 2>&1 && echo "pmc c2 ok"
rc=$?
tail -2 $O/pytest_gpu.log; tail -1 $O/bench_c2.log | cut -c1-400; tail -1 $O/bench_c5.log | cut -c1-400
exit $rc
