#!/bin/bash
# Round 4, call q: kernel-trace breakdown of the world-1 row-sharded step, then the
# PMC traffic of every bench roofline (profiles/r4_pmc_*).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4q
mkdir -p $O
MODES="sharded1" timeout -k 10 300 bash scripts/gpu_step_profiles.sh > $O/profiles.log 2>&1
rc=$?; echo "profiles rc=$rc" >> $O/summary.txt
cp gpurun_out/step_breakdown_sharded1.txt gpurun_out/step_timeline_sharded1.txt gpurun_out/kernel_stats_sharded1.csv $O/ 2>/dev/null
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash scripts/gpu_pmc_round.sh r4 > $O/pmc.log 2>&1
echo "pmc rc=$?" >> $O/summary.txt
cat $O/summary.txt; head -30 $O/step_breakdown_sharded1.txt
