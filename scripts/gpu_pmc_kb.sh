#!/bin/bash
# PMC passes over one kernel-bench script's cases (one pass per counter group, each under its own limit):
#   bash scripts/gpu_pmc_kb.sh <kbench script> <case substring> [out dir]   -> <out>/summary.txt
set -o pipefail
KB=$1; SUB=$2; OUT=${3:-gpurun_out/pmckb}
mkdir -p $OUT
export TMPDIR=/tmp
B="python $KB --only $SUB"
i=0
for G in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $G --output-format csv -d $OUT/p$i -o p$i -- $B > $OUT/p$i.log 2>&1 || exit 1
done
python scripts/pmc_summary.py $OUT > $OUT/summary.txt 2>&1; cat $OUT/summary.txt
