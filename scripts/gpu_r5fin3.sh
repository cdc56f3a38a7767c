#!/bin/bash
# Round 5 profiles: PMC traffic of every bench roofline (two counter passes, profiles/r5_pmc_*),
# the per-step kernel breakdowns (fused, world-1 sharded), and rocprofv3 --kernel-trace --stats
# of the default bench command with its JSON line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5fin3
mkdir -p $O
timeout -k 10 400 python -u -m pytest -v -rs -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bench_size.py \
  > $O/bench_size.log 2>&1
echo "bench_size rc=$?" >> $O/summary.txt
timeout -k 10 700 bash scripts/gpu_pmc_round.sh r5 > $O/pmc.log 2>&1
rc=$?; echo "pmc rc=$rc" >> $O/summary.txt
cp gpurun_out/pmc_r5/* $O/ 2>/dev/null
[ $rc -eq 0 ] || { cat $O/summary.txt; tail -20 $O/pmc.log; exit $rc; }
MODES="fused sharded1" timeout -k 10 500 bash scripts/gpu_step_profiles.sh > $O/profiles.log 2>&1
rc=$?; echo "profiles rc=$rc" >> $O/summary.txt
for m in fused sharded1; do
  cp gpurun_out/step_breakdown_$m.txt gpurun_out/step_timeline_$m.txt gpurun_out/kernel_stats_$m.csv $O/ 2>/dev/null
done
[ $rc -eq 0 ] || { cat $O/summary.txt; exit $rc; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ktb -o run -- python bench.py \
  > $O/bench_default.json 2> $O/bench_default.err
echo "rocprof bench rc=$?" >> $O/summary.txt
cp $(find /tmp/ktb -name "*kernel_stats.csv" | head -1) $O/kernel_stats_bench.csv 2>/dev/null
timeout -k 10 300 python -u scripts/op_sites.py > $O/op_sites.txt 2> $O/op_sites.err
echo "op_sites rc=$?" >> $O/summary.txt
cat $O/summary.txt; grep -h "traffic" $O/summary.txt $O/pmc.log | head -20
head -14 $O/step_breakdown_fused.txt; tail -c 300 $O/bench_default.json
