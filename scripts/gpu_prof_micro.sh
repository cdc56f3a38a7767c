#!/bin/bash
# per-kernel stats of one microbench: bash scripts/gpu_prof_micro.sh <script> <tag>
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pm -o run -- python -u $1 > gpurun_out/prof_$2.log 2>&1
cp $(find /tmp/pm -name "*kernel_stats.csv" | head -1) gpurun_out/prof_$2_stats.csv
