#!/bin/bash
# A/B of kernel variants: one kernel-bench script run against several libraries (the product library and
# scripts/build_variant.sh builds, loaded through ICA_HIP_LIB), interleaved by library, two repetitions.
#   bash scripts/gpu_ab.sh <kbench script> <case substring> <lib>...     (lib "base" = the product library)
set -o pipefail
KB=$1; SUB=$2; shift 2
for rep in 1 2; do
  for L in "$@"; do
    lib=$L; [ "$L" = base ] && lib=imagecompression_adversarial_amd/libica_hip.so
    echo "== $L (rep $rep)"
    ICA_HIP_LIB=$lib timeout -k 10 180 python $KB --only "$SUB" || exit 1
  done
done
