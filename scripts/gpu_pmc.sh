#!/bin/bash
# PMC passes on a short bench run (separate passes; no tracing domains combined with --pmc).
set -o pipefail
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc/p1 -o p1 -- $B > gpurun_out/pmc/p1.log 2>&1 \
&& timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc/p2 -o p2 -- $B > gpurun_out/pmc/p2.log 2>&1 \
&& timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc/p3 -o p3 -- $B > gpurun_out/pmc/p3.log 2>&1 \
&& timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmc/p4 -o p4 -- $B > gpurun_out/pmc/p4.log 2>&1
rc=$?
ls -R gpurun_out/pmc | head -30
tail -3 gpurun_out/pmc/p1.log gpurun_out/pmc/p4.log
exit $rc
