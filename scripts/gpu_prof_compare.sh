#!/bin/bash
# rocprofv3 kernel traces of the bench step in several modes; per-step breakdowns to gpurun_out/.
# Usage (via gpurun): bash scripts/gpu_prof_compare.sh TAG "mode1args" "mode2args" ...
#   e.g. bash scripts/gpu_prof_compare.sh r3 "--jagged 1" "--jagged 0"
set -e -o pipefail
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
i=0
for args in "$@"; do
  d=/tmp/kt_${TAG}_$i
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
    python bench.py --steps 10 --warmup 5 --cpu-baseline 0 --rooflines 0 $args > gpurun_out/kt_${TAG}_$i.log 2>&1
  kt=$(find $d -name "*kernel_trace.csv" | head -n 1)
  st=$(find $d -name "*kernel_stats.csv" | head -n 1)
  cp "$st" gpurun_out/${TAG}_kernel_stats_$i.csv
  echo "# bench args: $args" > gpurun_out/${TAG}_step_breakdown_$i.txt
  python scripts/step_breakdown.py "$kt" k_seq_ranges 5 >> gpurun_out/${TAG}_step_breakdown_$i.txt
  i=$((i+1))
done
