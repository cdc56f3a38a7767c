#!/bin/bash
# Round 4, call i: the grouped MFMA projection GEMMs (new) first, then the whole
# default GPU suite (every fused test now runs the grouped projections), the
# default bench line, the bmm-projection A/B line and a step breakdown.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
FAULT='illegal memory access|memory access fault|HSA_STATUS_ERROR|hipErrorIllegalAddress|HW Exception|GPU Hang|page not present'
timeout -k 10 300 python -u -m pytest -v -rs --timeout 120 --timeout-method thread tests/test_gpu_ggemm.py \
  > gpurun_out/r4i_ggemm.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r4i_ggemm.log
grep -Eqi "$FAULT" gpurun_out/r4i_ggemm.log && { echo "GPU fault in the grouped GEMM tests -- stopping"; exit 3; }
case $rc in 0|1) ;; *) echo "pytest exit $rc -- stopping"; exit $rc ;; esac
timeout -k 10 180 python -u scripts/microbench/ggemm_shapes.py > gpurun_out/r4i_ggemm_shapes.txt 2>&1 || exit $?
timeout -k 10 300 python -u scripts/op_sites.py > gpurun_out/r4i_op_sites.txt 2>&1 || exit $?
bash scripts/gpu_suite.sh r4i 1 || exit $?
timeout -k 10 300 python -u bench.py --grouped-proj 0 > gpurun_out/r4i_bench_bmmproj.json 2> gpurun_out/r4i_bench_bmmproj.err || exit $?
MODES=fused bash scripts/gpu_step_profiles.sh || exit $?
cp gpurun_out/step_breakdown_fused.txt gpurun_out/r4i_step_breakdown.txt
cp gpurun_out/kernel_stats_fused.csv gpurun_out/r4i_kernel_stats.csv
cp gpurun_out/step_timeline_fused.txt gpurun_out/r4i_step_timeline.txt
tail -3 gpurun_out/r4i_ggemm.log
