#!/bin/bash
# One round's bench evidence for a config: the default bench line (CPU baseline included), a rocprofv3
# kernel-trace summary of a short run (kernel stats + per-grid averages; the raw trace stays on the box), and the
# PMC passes (scripts/gpu_pmc.sh) reduced to per-launch traffic (scripts/pmc_traffic.py) and a counter summary.
#   bash scripts/gpu_evidence.sh <tag> <label> [bench args, e.g. --config 3]
set -o pipefail
TAG=$1; LABEL=$2; shift 2
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python bench.py "$@" > $O/bench.log 2>&1 && echo "bench ok" \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt -o kt -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --full-run 0 "$@" > $O/prof.log 2>&1 \
&& cp $(find /tmp/kt -name "kt_kernel_stats.csv") $O/kernel_stats.csv && python scripts/kt_by_grid.py $(find /tmp/kt -name "kt_kernel_trace.csv") $O/kernel_stats_by_grid.csv && echo "rocprof ok" \
&& PMC_TAG=${TAG}_pmc bash scripts/gpu_pmc.sh "$@" > /dev/null 2>&1 \
&& python scripts/pmc_traffic.py gpurun_out/${TAG}_pmc gpurun_out/${TAG}_pmc/launches.json "$LABEL" > $O/pmc_traffic.json && python scripts/pmc_summary.py gpurun_out/${TAG}_pmc > $O/pmc_summary.txt 2>&1 \
&& rm -rf gpurun_out/${TAG}_pmc && echo "pmc ok"
