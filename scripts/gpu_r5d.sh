#!/bin/bash
# Round 5, call d: the column-sliced chunked embedding backward (k_seg_chunks_sliced):
# bit-exact tests, microbench + bench A/B against the whole-row kernel
# (GRK_BWD_SLICED=0), FETCH_SIZE of both on the microbench; wgrad slice-length A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5d
mkdir -p $O
FAULT='illegal memory access|memory access fault|HSA_STATUS_ERROR|hipErrorIllegalAddress|HW Exception|GPU Hang|page not present'
timeout -k 10 400 python -u -m pytest -v -rs --timeout 200 --timeout-method thread -m gpu tests/test_gpu_embedding.py \
  tests/test_gpu_jagged.py > $O/tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> $O/summary.txt
grep -Eqi "$FAULT" $O/tests.log && { echo "GPU fault -- stopping"; cat $O/summary.txt; exit 3; }
case $rc in 0|1) ;; *) echo "pytest exit $rc -- stopping"; exit $rc ;; esac
for v in 1 0; do
  GRK_BWD_SLICED=$v timeout -k 10 200 python -u scripts/microbench/emb_bwd.py > $O/emb_bwd_sliced$v.txt 2>&1
  echo "emb_bwd sliced=$v rc=$?" >> $O/summary.txt
done
for v in 1 0; do
  GRK_BWD_SLICED=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline 0 \
    > $O/bench_sliced$v.json 2> $O/bench_sliced$v.err
  echo "bench sliced=$v rc=$?" >> $O/summary.txt
done
for v in 1 0; do
  GRK_BWD_SLICED=$v timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_seg_chunks" \
    --output-format csv -d /tmp/pmc_s$v -o run -- python -u scripts/microbench/emb_bwd.py > $O/pmc$v.log 2>&1
  echo "pmc sliced=$v rc=$?" >> $O/summary.txt
  cp $(find /tmp/pmc_s$v -name "*counter_collection.csv" | head -1) $O/pmc_fetch_sliced$v.csv 2>/dev/null
done
timeout -k 10 400 python -u scripts/microbench/wgrad_ab.py > $O/wgrad_ab.txt 2>&1
echo "wgrad ab rc=$?" >> $O/summary.txt
cat $O/summary.txt; cat $O/wgrad_ab.txt | tail -8; cat $O/emb_bwd_sliced*.txt; grep -E "passed|failed|Error" $O/tests.log | tail -8
python - <<'PY'
import json
for v in (1, 0):
    try:
        d = json.loads(open(f'gpurun_out/r5d/bench_sliced{v}.json').read().strip().splitlines()[-1])
    except Exception as e:
        print(v, 'no bench json', e); continue
    pr = [r for r in d.get('rooflines', []) if 'projected' in r['kernel']]
    print(f"sliced={v}: {d['value']} seq/s, {d['ms_per_step']} ms/step, projected call "
          f"{pr[0]['avg_launch_us'] if pr else None} us")
PY
