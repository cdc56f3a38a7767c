#!/bin/bash
# Round 4, call c: bench A/B of the opt-ins and build variants, op sites of the
# torch glue, and a kernel-trace step breakdown aligned to the timed steps.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_abflags.sh 1 "default||" "wgrad_reg|GRK_WGRAD_REG=1|" "merge|| --merge-proj 1" \
  "dflat|| --dense-flat 1" "ch64|GRK_LIB=$PWD/abtest/libgrk_ch64.so|" "ch128|GRK_LIB=$PWD/abtest/libgrk_ch128.so|" \
  || exit $?
timeout -k 10 300 python -u scripts/op_sites.py > gpurun_out/op_sites_r4c.txt 2>&1 || exit $?
MODES=fused bash scripts/gpu_step_profiles.sh || exit $?
cp gpurun_out/step_breakdown_fused.txt gpurun_out/r4c_step_breakdown.txt
cp gpurun_out/kernel_stats_fused.csv gpurun_out/r4c_kernel_stats.csv
