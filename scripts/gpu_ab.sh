#!/bin/bash
# A/B of two builds of libica_hip.so on one box: GPU parity tests on the candidate, then alternating benches.
# usage: bash scripts/gpu_ab.sh <candidate .so> <baseline .so> [bench args]
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
A=$1; B=$2; shift 2
O=gpurun_out/ab
ICA_HIP_LIB=$A timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && echo "pytest ok" || { tail -30 $O/pytest.log; exit 1; }
for r in 1 2; do
  for L in $A $B; do
    ICA_HIP_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 3 "$@" > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
    echo "$L $(python -c "import json;d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]);print(d['value'],d['roofline']['kernel'],d['roofline']['launch_ms'],json.dumps(d['per_kernel_ms']))")"
  done
done
