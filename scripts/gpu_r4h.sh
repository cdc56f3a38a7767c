#!/bin/bash
# Round 4, call h: r4g's failures after the shadow-registry fix and the sharded
# jagged test restructure, the HSTU rounding diagnosis, wgrad / dense-flat tests,
# then the default bench line and a step breakdown.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
FAULT='illegal memory access|memory access fault|HSA_STATUS_ERROR|hipErrorIllegalAddress|HW Exception|GPU Hang|page not present'
timeout -k 10 600 python -u -m pytest -v -rs --timeout 200 --timeout-method thread \
  tests/test_gpu_sharding.py tests/test_gpu_sharding_c3.py tests/test_gpu_dense_flat.py tests/test_gpu_wgrad.py \
  tests/test_gpu_embedding.py tests/test_gpu_jagged.py \
  "tests/test_gpu_model.py::test_hstu_model_matches_oracle" "tests/test_gpu_model.py::test_bench_config_step_matches_oracle_fp32" \
  > gpurun_out/r4h_gputest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r4h_gputest.log
grep -Eqi "$FAULT" gpurun_out/r4h_gputest.log && { echo "GPU fault -- stopping"; exit 3; }
case $rc in 0|1) ;; *) echo "pytest exit $rc -- stopping"; exit $rc ;; esac
timeout -k 10 120 python -u scripts/diag/hstu_rounding.py > gpurun_out/r4h_hstu_rounding.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/r4h_bench.json 2> gpurun_out/r4h_bench.err || exit $?
MODES=fused bash scripts/gpu_step_profiles.sh || exit $?
cp gpurun_out/step_breakdown_fused.txt gpurun_out/r4h_step_breakdown.txt
cp gpurun_out/kernel_stats_fused.csv gpurun_out/r4h_kernel_stats.csv
cp gpurun_out/step_timeline_fused.txt gpurun_out/r4h_step_timeline.txt
tail -3 gpurun_out/r4h_gputest.log
