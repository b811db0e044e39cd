#!/bin/bash
# A/B of bf16 variant libraries: bf16 parity tests on each, then interleaved kbench_bf16 rounds (GPU box).
# usage: bash scripts/exp/bf_ab.sh <lib.so>...
set -o pipefail
for L in "$@"; do
  ICA_HIP_LIB=$PWD/$L timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1 || { echo "tests FAILED on $L"; tail -20 gpurun_out/ab_pytest.log; exit 1; }
  echo "tests ok on $L"
done
for r in 1 2; do
  for L in "$@"; do
    echo "== $L"
    ICA_HIP_LIB=$PWD/$L timeout -k 10 120 python scripts/kbench_bf16.py --only rgb 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
