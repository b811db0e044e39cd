#!/bin/bash
# PMC passes over kbench_bf16 kernels (one pass per counter group): bash scripts/gpu_pmc_kb.sh <name-substring>
set -o pipefail
mkdir -p gpurun_out/pmckb
export TMPDIR=/tmp
B="python scripts/kbench_bf16.py --only $1"
i=0
for G in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS" \
         "FETCH_SIZE" "WRITE_SIZE" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $G --output-format csv -d gpurun_out/pmckb/p$i -o p$i -- $B > gpurun_out/pmckb/p$i.log 2>&1 || exit 1
done
python scripts/pmc_summary.py gpurun_out/pmckb > gpurun_out/pmckb/summary.txt 2>&1; cat gpurun_out/pmckb/summary.txt
