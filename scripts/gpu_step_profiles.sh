#!/bin/bash
# rocprofv3 kernel traces of the fused (N=1 default) and world-1 row-sharded
# bench steps; per-step breakdowns written to gpurun_out/.
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for mode in ${MODES:-fused sharded1}; do
  extra=""
  [ $mode = sharded1 ] && extra="--sharded 1"
  d=/tmp/kt_$mode
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
    python bench.py --steps 10 --warmup 5 --cpu-baseline 0 --rooflines 0 $extra > gpurun_out/kt_$mode.log 2>&1
  kt=$(find $d -name "*kernel_trace.csv" | head -n 1)
  st=$(find $d -name "*kernel_stats.csv" | head -n 1)
  cp "$st" gpurun_out/kernel_stats_$mode.csv
  python scripts/step_breakdown.py "$kt" k_seq_ranges 5 > gpurun_out/step_breakdown_$mode.txt
  python scripts/step_timeline.py "$kt" k_seq_ranges 2 > gpurun_out/step_timeline_$mode.txt
done
