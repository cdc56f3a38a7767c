#!/bin/bash
# Round 5, call k: the record form of the column-sliced projected-row backward
# (GRK_BWD_SLICED=2): bit-exact chunk-order tests, microbench + bench A/B against the
# whole-row kernel, FETCH_SIZE / L2 hits of the chunk kernel in the bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5k
mkdir -p $O
FAULT='illegal memory access|memory access fault|HSA_STATUS_ERROR|hipErrorIllegalAddress|HW Exception|GPU Hang|page not present'
PYT="python -u -m pytest -v -rs --timeout 200 --timeout-method thread -m gpu"
timeout -k 10 500 $PYT -s tests/test_gpu_bench_size.py tests/test_gpu_model.py -k "bench_config or deferred or graph_replayed" \
  > $O/parity.log 2>&1
echo "parity rc=$?" >> $O/summary.txt
grep -Eqi "$FAULT" $O/parity.log && { echo "GPU fault"; cat $O/summary.txt; exit 3; }
GRK_BWD_SLICED=2 timeout -k 10 300 $PYT tests/test_gpu_embedding.py tests/test_gpu_jagged.py -k "chunked or merged or projected" \
  > $O/tests2.log 2>&1
rc=$?; echo "tests sliced2 rc=$rc" >> $O/summary.txt
grep -Eqi "$FAULT" $O/tests2.log && { echo "GPU fault"; cat $O/summary.txt; exit 3; }
case $rc in 0|1) ;; *) echo "pytest exit $rc"; exit $rc ;; esac
for v in 2 0; do
  GRK_BWD_SLICED=$v timeout -k 10 200 python -u scripts/microbench/emb_bwd.py > $O/emb_bwd_$v.txt 2>&1
  echo "emb_bwd $v rc=$?" >> $O/summary.txt
done
for v in 2 0; do
  GRK_BWD_SLICED=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 > $O/bench_$v.json 2> $O/bench_$v.err
  echo "bench $v rc=$?" >> $O/summary.txt
done
B="python -u bench.py --steps 3 --warmup 2 --cpu-baseline 0 --rooflines 0"
GRK_BWD_SLICED=2 timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_seg_chunks" \
  --output-format csv -d /tmp/pf2 -o run -- $B > $O/pf2.log 2>&1
echo "fetch rc=$?" >> $O/summary.txt
cp $(find /tmp/pf2 -name "*counter_collection.csv" | head -1) $O/bench_fetch_sliced2.csv 2>/dev/null
GRK_BWD_SLICED=2 timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "k_seg_chunks" \
  --output-format csv -d /tmp/ph2 -o run -- $B > $O/ph2.log 2>&1
echo "hit rc=$?" >> $O/summary.txt
cp $(find /tmp/ph2 -name "*counter_collection.csv" | head -1) $O/bench_hit_sliced2.csv 2>/dev/null
cat $O/summary.txt; grep -E "passed|failed" $O/parity.log $O/tests2.log | tail -4; grep -E "bench-size|table elements|optimizer" $O/parity.log | head -4; cat $O/emb_bwd_*.txt | grep projected
python - <<'PY'
import json
for v in (2, 0):
    try:
        d = json.loads(open(f'gpurun_out/r5k/bench_{v}.json').read().strip().splitlines()[-1])
    except Exception as e:
        print(v, 'no json', e); continue
    pr = [r for r in d.get('rooflines', []) if 'projected' in r['kernel']]
    print(f"sliced={v}: {d['value']} seq/s, {d['ms_per_step']} ms/step, projected call {pr[0]['avg_launch_us'] if pr else None} us")
PY
