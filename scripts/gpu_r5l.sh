#!/bin/bash
# Round 5, call l: attention dK/dV A/B builds (oracle checks, then bench round-robin) and
# the jagged capacity quantum (256 vs 512).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5l
mkdir -p $O
FAULT='illegal memory access|memory access fault|HSA_STATUS_ERROR|hipErrorIllegalAddress|HW Exception|GPU Hang|page not present'
PYT="python -u -m pytest -v -rs --timeout 300 --timeout-method thread -m gpu"
for v in nopre fold foldtb; do
  GRK_LIB=$PWD/abvar/libgrk_$v.so timeout -k 10 300 $PYT tests/test_gpu_attention.py \
    -k "c2_shape or precise or determinism or time_bias_c2 or bwd_parts" > $O/attn_$v.log 2>&1
  echo "attn $v rc=$?" >> $O/summary.txt
  grep -Eqi "$FAULT" $O/attn_$v.log && { echo "GPU fault"; cat $O/summary.txt; exit 3; }
done
for i in 1; do
  for v in default nopre fold foldtb; do
    lib=tencent_recommendation_2025_amd/libgrk.so; [ $v = default ] || lib=abvar/libgrk_$v.so
    GRK_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --roofline-reps 5 \
      > $O/ab_${v}_$i.json 2>/dev/null
    echo "ab $v $i rc=$?" >> $O/summary.txt
  done
done
for q in 256 512; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --rooflines 0 --jagged-quantum $q \
    > $O/quantum_$q.json 2>/dev/null
  echo "quantum $q rc=$?" >> $O/summary.txt
done
timeout -k 10 600 bash scripts/gpu_pmc_round.sh r5 > $O/pmc.log 2>&1
echo "pmc rc=$?" >> $O/summary.txt
cp gpurun_out/pmc_r5/r5_pmc_*.json $O/ 2>/dev/null
cat $O/summary.txt; grep -hE "passed|failed" $O/attn_*.log; grep "vs algorithmic" $O/pmc.log
python - <<'PY'
import json, glob
for f in sorted(glob.glob('gpurun_out/r5l/*.json')):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:
        print(f, 'no json'); continue
    ents = [d['roofline']] + d.get('rooflines', []) if 'roofline' in d else []
    dk = [r.get('avg_launch_us') for r in ents if 'dkdv' in r.get('kernel', '')]
    dq = [r.get('avg_launch_us') for r in ents if 'k_attn_dq' in r.get('kernel', '')]
    print(f.split('/')[-1], d['value'], d['ms_per_step'], 'dkdv', dk, 'dq', dq)
PY
