#!/bin/bash
# Round 5, call h: the rolling flush's slice on a side stream (GRK_SLICE_SIDE) -- the
# deferred / graph bitwise tests, fused and sharded bench A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5h
mkdir -p $O
FAULT='illegal memory access|memory access fault|HSA_STATUS_ERROR|hipErrorIllegalAddress|HW Exception|GPU Hang|page not present'
timeout -k 10 700 python -u -m pytest -v -rs --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sharding.py \
  tests/test_gpu_model.py tests/test_gpu_bench_size.py > $O/tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> $O/summary.txt
grep -Eqi "$FAULT" $O/tests.log && { echo "GPU fault -- stopping"; cat $O/summary.txt; tail -30 $O/tests.log; exit 3; }
case $rc in 0|1) ;; *) echo "pytest exit $rc -- stopping"; tail -30 $O/tests.log; exit $rc ;; esac
for v in 1 0; do
  GRK_SLICE_SIDE=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --rooflines 0 \
    > $O/bench_slice$v.json 2> $O/bench_slice$v.err
  echo "bench slice=$v rc=$?" >> $O/summary.txt
  GRK_SLICE_SIDE=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --rooflines 0 \
    --sharded 1 > $O/bench_sharded_slice$v.json 2> $O/bench_sharded_slice$v.err
  echo "bench sharded slice=$v rc=$?" >> $O/summary.txt
done
cat $O/summary.txt; grep -E "passed|failed|Error" $O/tests.log | tail -8
for f in bench_slice1 bench_slice0 bench_sharded_slice1 bench_sharded_slice0; do echo $f; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/$f.json | head -2; done
