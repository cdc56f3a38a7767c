#!/bin/bash
# Round 5, call j: bench-size parity + C5 graph == eager at the new defaults; the
# attention dK/dV A/B builds (no prologue prefetch; 1/n folded; time-bias split)
# checked against the oracle, then timed in the bench (round-robin).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5j
mkdir -p $O
FAULT='illegal memory access|memory access fault|HSA_STATUS_ERROR|hipErrorIllegalAddress|HW Exception|GPU Hang|page not present'
PYT="python -u -m pytest -v -rs -s --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 500 $PYT tests/test_gpu_bench_size.py tests/test_gpu_model.py -k "bench_config or deferred or graph_replayed" \
  > $O/parity.log 2>&1
echo "parity rc=$?" >> $O/summary.txt
grep -Eqi "$FAULT" $O/parity.log && { echo "GPU fault"; exit 3; }
for v in nopre fold foldtb foldnopre; do
  GRK_LIB=$PWD/abvar/libgrk_$v.so timeout -k 10 300 $PYT tests/test_gpu_attention.py \
    -k "c2_shape or precise or determinism or time_bias_c2 or bwd_parts" > $O/attn_$v.log 2>&1
  echo "attn $v rc=$?" >> $O/summary.txt
  grep -Eqi "$FAULT" $O/attn_$v.log && { echo "GPU fault"; cat $O/summary.txt; exit 3; }
done
timeout -k 10 900 bash scripts/gpu_ab.sh 2 "tencent_recommendation_2025_amd/libgrk.so abvar/libgrk_nopre.so abvar/libgrk_fold.so abvar/libgrk_foldtb.so abvar/libgrk_foldnopre.so" > $O/ab.log 2>&1
echo "ab rc=$?" >> $O/summary.txt
cp gpurun_out/ab.txt $O/ 2>/dev/null
cat $O/summary.txt; grep -E "passed|failed" $O/parity.log $O/attn_*.log | tail -8; grep -E "bench-size|ulp|optimizer" $O/parity.log | head -5; cat $O/ab.txt
