#!/bin/bash
# PMC counter summaries of kbench_x6 cases for the product library and variant libraries (one pass per counter group
# each, scripts/gpu_pmc_kb.sh), plus their timings.
#   bash scripts/gpu_pmc_ab.sh <case substring> <out dir> <lib>...   (lib "base" = the product library)
set -o pipefail
SUB=$1; OUT=$2; shift 2
mkdir -p $OUT
for L in base "$@"; do
  lib=$L; [ "$L" = base ] && lib=imagecompression_adversarial_amd/libica_hip.so
  n=$(basename $L .so)
  ICA_HIP_LIB=$lib bash scripts/gpu_pmc_kb.sh scripts/kbench_x6.py "$SUB" $OUT/$n > /dev/null 2>&1 || exit 1
  ICA_HIP_LIB=$lib timeout -k 10 180 python scripts/kbench_x6.py --only "$SUB" > $OUT/$n/kb.log 2>&1 || exit 1
done
