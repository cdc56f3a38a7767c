#!/bin/bash
# Round 5, call e: why the column-sliced chunked backward (GRK_BWD_SLICED=1) is slower
# in the bench step than in the microbench -- bench kernel traces + FETCH_SIZE and L2
# hit/miss of the chunk kernels for both forms; then the fused and world-1 row-sharded
# step breakdowns (rolling flush) and the sharded bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5e
mkdir -p $O
B="python -u bench.py --steps 3 --warmup 2 --cpu-baseline 0 --rooflines 0"
for v in 1 0; do
  GRK_BWD_SLICED=$v timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_seg_chunks" \
    --output-format csv -d /tmp/pf$v -o run -- $B > $O/pf$v.log 2>&1
  echo "fetch sliced=$v rc=$?" >> $O/summary.txt
  cp $(find /tmp/pf$v -name "*counter_collection.csv" | head -1) $O/bench_fetch_sliced$v.csv 2>/dev/null
  GRK_BWD_SLICED=$v timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --kernel-include-regex "k_seg_chunks" \
    --output-format csv -d /tmp/ph$v -o run -- $B > $O/ph$v.log 2>&1
  echo "hit sliced=$v rc=$?" >> $O/summary.txt
  cp $(find /tmp/ph$v -name "*counter_collection.csv" | head -1) $O/bench_hit_sliced$v.csv 2>/dev/null
done
MODES="fused sharded1" timeout -k 10 500 bash scripts/gpu_step_profiles.sh > $O/profiles.log 2>&1
rc=$?; echo "profiles rc=$rc" >> $O/summary.txt
for m in fused sharded1; do
  cp gpurun_out/step_breakdown_$m.txt $O/ 2>/dev/null; cp gpurun_out/step_timeline_$m.txt $O/ 2>/dev/null
  cp gpurun_out/kernel_stats_$m.csv $O/ 2>/dev/null
done
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --sharded 1 > $O/bench_sharded1.json 2> $O/bench_sharded1.err
echo "bench sharded1 rc=$?" >> $O/summary.txt
cat $O/summary.txt; head -25 $O/step_breakdown_fused.txt; head -25 $O/step_breakdown_sharded1.txt; tail -c 600 $O/bench_sharded1.json
