#!/bin/bash
# Round 4, call c: the changed kernels' tests (embedding: fused zero fill +
# row-indexed segments; wgrad LDS ring) and the fixed opt-ins, the jagged-vs-
# padded row diagnostic, bench A/B of opt-ins / build variants, op sites of the
# torch glue, and a kernel-trace step breakdown aligned to the timed steps.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
FAULT='illegal memory access|memory access fault|HSA_STATUS_ERROR|hipErrorIllegalAddress|HW Exception|GPU Hang|page not present'
PYT="python -u -m pytest -v -rs --timeout 200 --timeout-method thread"
env GRK_MERGE_PROJ_TESTS=1 GRK_DENSE_FLAT_TESTS=1 GRK_SHARDED_JAGGED_TESTS=1 timeout -k 10 600 $PYT \
  tests/test_gpu_embedding.py tests/test_gpu_wgrad.py tests/test_gpu_dense_flat.py tests/test_gpu_jagged.py \
  tests/test_gpu_attention.py tests/test_gpu_model.py tests/test_gpu_sharding.py > gpurun_out/r4c_tests.log 2>&1
rc=$?; echo "tests rc=$rc" | tee -a gpurun_out/r4c_tests.log
grep -Eqi "$FAULT" gpurun_out/r4c_tests.log && { echo "GPU fault -- stopping"; exit 3; }
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 120 python -u scripts/diag/jagged_vs_padded.py > gpurun_out/r4c_jagged_diag.txt 2>&1 || exit $?
bash scripts/gpu_abflags.sh 1 "default||" "wgrad_reg|GRK_WGRAD_REG=1|" "merge|| --merge-proj 1" \
  "dflat|| --dense-flat 1" "ch64|GRK_LIB=$PWD/abtest/libgrk_ch64.so|" "ch64merge|GRK_LIB=$PWD/abtest/libgrk_ch64.so| --merge-proj 1" \
  || exit $?
timeout -k 10 300 python -u scripts/op_sites.py > gpurun_out/op_sites_r4c.txt 2>&1 || exit $?
MODES=fused bash scripts/gpu_step_profiles.sh || exit $?
cp gpurun_out/step_breakdown_fused.txt gpurun_out/r4c_step_breakdown.txt
cp gpurun_out/kernel_stats_fused.csv gpurun_out/r4c_kernel_stats.csv
