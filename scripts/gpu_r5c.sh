#!/bin/bash
# Round 5, call c: the MFMA GEMM after the loop restructure (tests + shape sweep) and
# grk_wgrad on its K-major mode (tests + A/B against the round-4 kernels).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5c
mkdir -p $O
FAULT='illegal memory access|memory access fault|HSA_STATUS_ERROR|hipErrorIllegalAddress|HW Exception|GPU Hang|page not present'
timeout -k 10 400 python -u -m pytest -v -rs --timeout 200 --timeout-method thread -m gpu tests/test_gpu_mgemm.py \
  tests/test_gpu_wgrad.py tests/test_gpu_linear.py > $O/tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> $O/summary.txt
grep -Eqi "$FAULT" $O/tests.log && { echo "GPU fault -- stopping"; cat $O/summary.txt; exit 3; }
case $rc in 0|1) ;; *) echo "pytest exit $rc -- stopping"; exit $rc ;; esac
timeout -k 10 400 python -u scripts/microbench/mgemm.py > $O/mgemm_bench.txt 2>&1
echo "mgemm bench rc=$?" >> $O/summary.txt
timeout -k 10 400 python -u scripts/microbench/wgrad_ab.py > $O/wgrad_ab.txt 2>&1
echo "wgrad ab rc=$?" >> $O/summary.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
  SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --kernel-include-regex "k_mgemm" --output-format csv \
  -d /tmp/sqm -o run -- python -u scripts/microbench/mgemm.py eager > $O/sq.log 2>&1
echo "sq rc=$?" >> $O/summary.txt
cp $(find /tmp/sqm -name "*counter_collection.csv" | head -1) $O/sq_mgemm.csv 2>/dev/null
cat $O/summary.txt; cat $O/mgemm_bench.txt $O/wgrad_ab.txt; grep -E "passed|failed|Error" $O/tests.log | tail -8
