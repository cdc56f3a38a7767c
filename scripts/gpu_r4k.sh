#!/bin/bash
# Round 4, call k: the world-1 row-sharded bench line, then an
# A/B of prepared builds (abtest/: chunked-backward chunk 128, wave pipe 32, attention
# 1/n folded into the dK/dV store scales, + time-bias-free instantiation; norm-gate /
# add-norm backward on 1024 workgroups instead of 512) against the
# product build, one run each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4k
mkdir -p $O
# the N > 1 code path at world 1 (RCCL, row-sharded tables, jagged rows) beside the fused step
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29613 bench.py --sharded 1 --cpu-baseline 0 --roofline-reps 1 > $O/bench_sharded1.json 2> $O/bench_sharded1.err
rc=$?; echo "sharded1 rc=$rc" >> $O/summary.txt
if grep -Eqi 'illegal memory access|memory access fault|HSA_STATUS_ERROR|GPU Hang' $O/bench_sharded1.err || [ $rc -gt 1 ]; then
  echo "sharded1 failed -- stopping" >> $O/summary.txt; exit 3
fi
# every variant must export what the product build exports (built from the same objects)
want=$(nm -D --defined-only tencent_recommendation_2025_amd/libgrk.so | grep -c " T grk_")
for v in abtest/*.so; do
  have=$(nm -D --defined-only $v | grep -c " T grk_")
  [ "$have" = "$want" ] || { echo "$v: $have of $want entry points -- stale variant, stopping" >> $O/summary.txt; exit 4; }
done
timeout -k 10 900 bash scripts/gpu_ab.sh 1 "tencent_recommendation_2025_amd/libgrk.so abtest/libgrk_ch128.so abtest/libgrk_pipe32.so abtest/libgrk_fold.so abtest/libgrk_foldtb.so abtest/libgrk_ngb1024.so" > $O/ab.log 2>&1
echo "ab rc=$?" >> $O/summary.txt
cp gpurun_out/ab.txt $O/ab.txt 2>/dev/null
cat $O/ab.txt
