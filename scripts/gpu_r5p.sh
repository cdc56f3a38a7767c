#!/bin/bash
# r5p: fresh world-1 row-sharded step timeline (where the device idles)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
MODES="sharded1" timeout -k 10 400 bash scripts/gpu_step_profiles.sh > gpurun_out/r5p_profiles.log 2>&1 || { tail -20 gpurun_out/r5p_profiles.log; exit 1; }
head -3 gpurun_out/step_breakdown_sharded1.txt; grep -A12 "idle gaps" gpurun_out/step_breakdown_sharded1.txt
