#!/bin/bash
# Round 4, call z: the C5 bench line (BASELINE configs[4]: HSTU d = 1024, T = 1025, fp8
# attention, B = 16, padded layout), then a world-1 sharded step breakdown.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4z
mkdir -p $O
timeout -k 10 400 python -u bench.py --fp8 1 --hidden 1024 --maxlen 1024 --batch 16 --warmup 3 \
  --cpu-baseline 0 --roofline-reps 3 > $O/bench_c5.json 2> $O/bench_c5.log
rc=$?; echo "bench_c5 rc=$rc" >> $O/summary.txt
[ $rc -eq 0 ] || exit $rc
MODES="sharded1" timeout -k 10 300 bash scripts/gpu_step_profiles.sh > $O/profiles.log 2>&1
echo "profiles rc=$?" >> $O/summary.txt
cp gpurun_out/step_breakdown_sharded1.txt $O/ 2>/dev/null
cat $O/summary.txt; cut -c1-200 $O/bench_c5.json
