#!/bin/bash
# Round 5, call i: bench-size parity test (table updates per ulp) and a bisect of the C5
# graph == eager failure over the two side-stream overlaps.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5i
mkdir -p $O
FAULT='illegal memory access|memory access fault|HSA_STATUS_ERROR|hipErrorIllegalAddress|HW Exception|GPU Hang|page not present'
PYT="python -u -m pytest -v -rs -s --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 400 $PYT tests/test_gpu_bench_size.py > $O/bench_size.log 2>&1
echo "bench_size rc=$?" >> $O/summary.txt
grep -Eqi "$FAULT" $O/bench_size.log && { echo "GPU fault"; exit 3; }
for w in 1 0; do for sl in 1 0; do
  GRK_WGRAD_SIDE=$w GRK_SLICE_SIDE=$sl timeout -k 10 300 $PYT \
    "tests/test_gpu_fp8.py::test_c5_fp8_trainer_graph_equals_eager" > $O/c5_w${w}_s${sl}.log 2>&1
  echo "c5 graph wgrad_side=$w slice_side=$sl rc=$?" >> $O/summary.txt
  grep -Eqi "$FAULT" $O/c5_w${w}_s${sl}.log && { echo "GPU fault"; cat $O/summary.txt; exit 3; }
done; done
cat $O/summary.txt; grep -E "bench-size|worst|ulp|optimizer|passed|failed" $O/bench_size.log | head; grep -h "At index\|passed\|failed" $O/c5_*.log
