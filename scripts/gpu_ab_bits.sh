#!/bin/bash
# A/B of kernel variants with a bit-exactness check: kbench_x6 timings for each library (interleaved, two
# repetitions), then every case's output under each variant compared bit for bit against the product library.
#   bash scripts/gpu_ab_bits.sh <case substring> <lib>...     (lib "base" = the product library)
set -o pipefail
SUB=$1; shift
KB=${KB:-scripts/kbench_x6.py}   # the kbench script (scripts/kbench_k3x6.py: the cheng2020 k3 s1 launches)
mkdir -p gpurun_out/ab
bash scripts/gpu_ab.sh $KB "$SUB" base "$@" || exit 1
ICA_HIP_LIB=imagecompression_adversarial_amd/libica_hip.so timeout -k 10 180 python $KB --only "$SUB" --dump gpurun_out/ab/base.pt > /dev/null || exit 1
for L in "$@"; do
  n=$(basename $L .so)
  ICA_HIP_LIB=$L timeout -k 10 180 python $KB --only "$SUB" --dump gpurun_out/ab/$n.pt > /dev/null || exit 1
  echo "== bits $n vs base"; python scripts/kbench_x6.py --cmp gpurun_out/ab/base.pt gpurun_out/ab/$n.pt
done
rm -f gpurun_out/ab/*.pt
