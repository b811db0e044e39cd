#!/bin/bash
# Same-box A/B of the working tree against a snapshot package (scripts/variants/<base>/: an older
# imagecompression_adversarial_amd with its own built library), one kernel-bench script, interleaved, two repetitions.
#   bash scripts/gpu_ab_tree.sh <kbench script> <case substring> <base dir> <out log>
set -o pipefail
KB=$(readlink -f $1); SUB=$2; BASE=$3; OUT=$4
mkdir -p $(dirname $OUT)
: > $OUT
for rep in 1 2; do
  echo "== tree (rep $rep)" >> $OUT
  timeout -k 10 240 python $KB --only "$SUB" >> $OUT 2>&1 || exit 1
  echo "== $BASE (rep $rep)" >> $OUT
  (cd $BASE && timeout -k 10 240 python $KB --only "$SUB") >> $OUT 2>&1 || exit 1
done
