#!/bin/bash
# PMC passes on a short bench run (separate passes; no tracing domains combined with --pmc).
#   bash scripts/gpu_pmc.sh [extra bench args, e.g. --config 5]  -> gpurun_out/pmc{,_c5}/
set -o pipefail
TAG=${PMC_TAG:-pmc}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
# bench.py writes the (kernel, grid) behind every timed tag here: scripts/pmc_traffic.py matches PMC rows with it
export ICA_LAUNCH_TABLE=gpurun_out/$TAG/launches.json
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline $*"
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/$TAG/p1 -o p1 -- $B > gpurun_out/$TAG/p1.log 2>&1 \
&& timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/$TAG/p2 -o p2 -- $B > gpurun_out/$TAG/p2.log 2>&1 \
&& timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/$TAG/p3 -o p3 -- $B > gpurun_out/$TAG/p3.log 2>&1 \
&& timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/$TAG/p4 -o p4 -- $B > gpurun_out/$TAG/p4.log 2>&1
rc=$?
tail -2 gpurun_out/$TAG/p1.log gpurun_out/$TAG/p4.log
exit $rc
