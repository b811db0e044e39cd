#!/bin/bash
# A/B of an x6 variant library against the in-tree one: interleaved kbench_x6 rounds (GPU box).
# usage: bash scripts/exp/x6_ab.sh <variant .so> [kbench --only filter]
set -o pipefail
V=$1; F=${2:-}
for r in 1 2 3; do
  for L in imagecompression_adversarial_amd/libica_hip.so $V; do
    echo "== $L"
    ICA_HIP_LIB=$PWD/$L timeout -k 10 120 python scripts/kbench_x6.py ${F:+--only $F} 2>&1 | grep "^x6" || exit 1
  done
done
