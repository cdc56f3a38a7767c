#!/bin/bash
# Round 4, call m: per-step kernel breakdowns of the fused step and of the world-1
# row-sharded step (rocprofv3 kernel traces, timed steps only), then the PMC traffic
# of every bench roofline (profiles/r4_pmc_*, two counter passes).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4m
mkdir -p $O
MODES="fused sharded1" timeout -k 10 500 bash scripts/gpu_step_profiles.sh > $O/profiles.log 2>&1
rc=$?; echo "profiles rc=$rc" >> $O/summary.txt
for m in fused sharded1; do
  cp gpurun_out/step_breakdown_$m.txt $O/ 2>/dev/null; cp gpurun_out/step_timeline_$m.txt $O/ 2>/dev/null
  cp gpurun_out/kernel_stats_$m.csv $O/ 2>/dev/null
done
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash scripts/gpu_pmc_round.sh r4 > $O/pmc.log 2>&1
echo "pmc rc=$?" >> $O/summary.txt
head -3 $O/step_breakdown_fused.txt
