#!/bin/bash
# Round 4, call g: the tests r4f failed (sharding, bench-config and HSTU model
# bounds) plus the embedding / sort / index tests after the wave-aggregated sort
# histogram fix, then the default bench line and a step breakdown.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
FAULT='illegal memory access|memory access fault|HSA_STATUS_ERROR|hipErrorIllegalAddress|HW Exception|GPU Hang|page not present'
timeout -k 10 600 python -u -m pytest -v -rs --timeout 200 --timeout-method thread \
  tests/test_gpu_sharding.py tests/test_gpu_sharding_c3.py tests/test_gpu_embedding.py tests/test_gpu_index.py \
  "tests/test_gpu_model.py::test_hstu_model_matches_oracle" "tests/test_gpu_model.py::test_bench_config_step_matches_oracle_fp32" \
  > gpurun_out/r4g_gputest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r4g_gputest.log
grep -Eqi "$FAULT" gpurun_out/r4g_gputest.log && { echo "GPU fault -- stopping"; exit 3; }
case $rc in 0|1) ;; *) echo "pytest exit $rc -- stopping"; exit $rc ;; esac
timeout -k 10 300 python -u bench.py > gpurun_out/r4g_bench.json 2> gpurun_out/r4g_bench.err || exit $?
MODES=fused bash scripts/gpu_step_profiles.sh || exit $?
cp gpurun_out/step_breakdown_fused.txt gpurun_out/r4g_step_breakdown.txt
cp gpurun_out/kernel_stats_fused.csv gpurun_out/r4g_kernel_stats.csv
tail -3 gpurun_out/r4g_gputest.log
