#!/bin/bash
# x6 conv_down prefetch variants vs the in-tree library: interleaved kbench rounds (GPU box)
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for L in imagecompression_adversarial_amd/libica_hip.so scripts/exp/lib_pf2.so scripts/exp/lib_tpf16.so scripts/exp/lib_tpf22.so; do
    echo "== $L"
    ICA_HIP_LIB=$PWD/$L timeout -k 10 120 python scripts/kbench_x6.py --only down 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
