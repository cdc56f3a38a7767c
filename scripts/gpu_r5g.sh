#!/bin/bash
# Round 5, call g: weight gradients on a side stream (functional.WGRAD_SIDE) + the
# grk route / packing / remaps of the row-sharded step: GPU tests, fused bench A/B,
# sharded bench, step breakdowns of both.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5g
mkdir -p $O
FAULT='illegal memory access|memory access fault|HSA_STATUS_ERROR|hipErrorIllegalAddress|HW Exception|GPU Hang|page not present'
timeout -k 10 700 python -u -m pytest -v -rs --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sharding.py \
  tests/test_gpu_model.py tests/test_gpu_jagged.py > $O/tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> $O/summary.txt
grep -Eqi "$FAULT" $O/tests.log && { echo "GPU fault -- stopping"; cat $O/summary.txt; tail -30 $O/tests.log; exit 3; }
case $rc in 0|1) ;; *) echo "pytest exit $rc -- stopping"; tail -30 $O/tests.log; exit $rc ;; esac
for v in 1 0; do
  GRK_WGRAD_SIDE=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --rooflines 0 \
    > $O/bench_side$v.json 2> $O/bench_side$v.err
  echo "bench side=$v rc=$?" >> $O/summary.txt
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --rooflines 0 --sharded 1 > $O/bench_sharded1.json 2> $O/bench_sharded1.err
echo "bench sharded1 rc=$?" >> $O/summary.txt
MODES="fused sharded1" timeout -k 10 500 bash scripts/gpu_step_profiles.sh > $O/profiles.log 2>&1
echo "profiles rc=$?" >> $O/summary.txt
for m in fused sharded1; do cp gpurun_out/step_breakdown_$m.txt gpurun_out/step_timeline_$m.txt $O/ 2>/dev/null; done
cat $O/summary.txt; grep -E "passed|failed|Error" $O/tests.log | tail -8
for f in bench_side1 bench_side0 bench_sharded1; do echo $f; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/$f.json | head -2; done
head -12 $O/step_breakdown_fused.txt; head -12 $O/step_breakdown_sharded1.txt
