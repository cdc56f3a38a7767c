#!/bin/bash
# Round 5, call a: the new parity tests (bench configuration at its own size, the
# rebuilt C5 fp8 test), the rolling flush (deferred == dense, lag bound, graph ==
# eager), the ADVICE r4 fixes (sharded dense_flat, shadows), then the bench line at
# --steps 20 and 32 (the rolling flush must make them agree).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5a
mkdir -p $O
FAULT='illegal memory access|memory access fault|HSA_STATUS_ERROR|hipErrorIllegalAddress|HW Exception|GPU Hang|page not present'
# grk's new MFMA GEMM first: its own tests and its timing against hipBLASLt
timeout -k 10 300 python -u -m pytest -v -rs --timeout 200 --timeout-method thread -m gpu tests/test_gpu_mgemm.py \
  > $O/mgemm_tests.log 2>&1
rc=$?
echo "mgemm tests rc=$rc" >> $O/summary.txt
grep -Eqi "$FAULT" $O/mgemm_tests.log && { echo "GPU fault -- stopping"; cat $O/summary.txt; exit 3; }
case $rc in 0|1) ;; *) echo "pytest exit $rc -- stopping"; exit $rc ;; esac
timeout -k 10 300 python -u scripts/microbench/mgemm.py > $O/mgemm_bench.txt 2>&1
echo "mgemm bench rc=$?" >> $O/summary.txt
# the rest on the round-4 GEMM backend (the new kernel is validated above first)
export GRK_GEMM_BACKEND=hipblaslt
timeout -k 10 700 python -u -m pytest -v -rs --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_bench_size.py tests/test_gpu_fp8.py tests/test_gpu_sharding.py tests/test_gpu_dense_flat.py \
  "tests/test_gpu_model.py::test_deferred_table_updates_are_bit_identical_to_dense" \
  "tests/test_gpu_model.py::test_graph_replayed_steps_equal_eager_steps" \
  "tests/test_gpu_model.py::test_eval_predict_and_export_read_flushed_rows" -s > $O/tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/summary.txt
grep -Eqi "$FAULT" $O/tests.log && { echo "GPU fault -- stopping"; cat $O/summary.txt; exit 3; }
case $rc in 0|1) ;; *) echo "pytest exit $rc -- stopping"; exit $rc ;; esac
timeout -k 10 300 python -u bench.py --steps 20 --cpu-baseline 0 > $O/bench20.json 2> $O/bench20.err
echo "bench20 rc=$?" >> $O/summary.txt
timeout -k 10 200 python -u bench.py --steps 32 --cpu-baseline 0 --rooflines 0 > $O/bench32.json 2> $O/bench32.err
echo "bench32 rc=$?" >> $O/summary.txt
cat $O/summary.txt
grep -E "passed|failed|error" $O/tests.log | tail -5
cut -c1-300 $O/bench20.json $O/bench32.json
cat $O/mgemm_bench.txt; grep -E 'passed|failed' $O/mgemm_tests.log | tail -3
