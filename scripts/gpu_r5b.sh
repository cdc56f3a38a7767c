#!/bin/bash
# Round 5, call b: grk's MFMA GEMM -- its tests, then the step shapes against hipBLASLt
# (two ring configurations).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5b
mkdir -p $O
FAULT='illegal memory access|memory access fault|HSA_STATUS_ERROR|hipErrorIllegalAddress|HW Exception|GPU Hang|page not present'
timeout -k 10 300 python -u -m pytest -v -rs --timeout 200 --timeout-method thread -m gpu tests/test_gpu_mgemm.py \
  > $O/mgemm_tests.log 2>&1
rc=$?
echo "mgemm tests rc=$rc" >> $O/summary.txt
grep -Eqi "$FAULT" $O/mgemm_tests.log && { echo "GPU fault -- stopping"; cat $O/summary.txt; exit 3; }
case $rc in 0|1) ;; *) echo "pytest exit $rc -- stopping"; exit $rc ;; esac
timeout -k 10 400 python -u scripts/microbench/mgemm.py > $O/mgemm_bench.txt 2>&1
echo "mgemm bench rc=$?" >> $O/summary.txt
cat $O/summary.txt; cat $O/mgemm_bench.txt; grep -E "passed|failed|Error" $O/mgemm_tests.log | tail -8
