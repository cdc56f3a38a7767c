#!/bin/bash
# Round 5, call f: the grk route / bucket packing of the row-sharded path -- GPU tests,
# the world-1 sharded and fused bench lines, the sharded step breakdown.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5f
mkdir -p $O
FAULT='illegal memory access|memory access fault|HSA_STATUS_ERROR|hipErrorIllegalAddress|HW Exception|GPU Hang|page not present'
timeout -k 10 400 python -u -m pytest -v -rs --timeout 200 --timeout-method thread -m gpu tests/test_gpu_sharding.py \
  > $O/tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> $O/summary.txt
grep -Eqi "$FAULT" $O/tests.log && { echo "GPU fault -- stopping"; cat $O/summary.txt; tail -30 $O/tests.log; exit 3; }
case $rc in 0|1) ;; *) echo "pytest exit $rc -- stopping"; tail -30 $O/tests.log; exit $rc ;; esac
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --rooflines 0 --sharded 1 > $O/bench_sharded1.json 2> $O/bench_sharded1.err
echo "bench sharded1 rc=$?" >> $O/summary.txt
MODES="sharded1" timeout -k 10 300 bash scripts/gpu_step_profiles.sh > $O/profiles.log 2>&1
echo "profiles rc=$?" >> $O/summary.txt
cp gpurun_out/step_breakdown_sharded1.txt gpurun_out/step_timeline_sharded1.txt $O/ 2>/dev/null
cat $O/summary.txt; grep -E "passed|failed|Error" $O/tests.log | tail -5; tail -c 400 $O/bench_sharded1.json; head -30 $O/step_breakdown_sharded1.txt
