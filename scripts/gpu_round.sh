#!/bin/bash
# One GPU call: gpu tests, default bench line, kernel-trace step profile.
# Usage (via gpurun): bash scripts/gpu_round.sh TAG [tests=1] [bench=1] [prof=1]
set -e -o pipefail
TAG=${1:-r2}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ "${2:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1
fi
if [ "${3:-1}" = 1 ]; then
  timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
fi
if [ "${4:-1}" = 1 ]; then
  MODES=fused bash scripts/gpu_step_profiles.sh
  cp gpurun_out/kernel_stats_fused.csv gpurun_out/${TAG}_kernel_stats.csv
  cp gpurun_out/step_breakdown_fused.txt gpurun_out/${TAG}_step_breakdown.txt
fi
