#!/bin/bash
# Round 4, call f: the whole default GPU suite (+ the sharded-jagged opt-in),
# the default bench line, the projection-GEMM microbench and a kernel-trace
# step breakdown of the timed steps.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
GRK_SHARDED_JAGGED_TESTS=1 bash scripts/gpu_suite.sh r4f 1 || exit $?
timeout -k 10 120 python -u scripts/microbench/proj_bmm.py > gpurun_out/r4f_proj_bmm.txt 2>&1 || exit $?
MODES=fused bash scripts/gpu_step_profiles.sh || exit $?
cp gpurun_out/step_breakdown_fused.txt gpurun_out/r4f_step_breakdown.txt
cp gpurun_out/kernel_stats_fused.csv gpurun_out/r4f_kernel_stats.csv
