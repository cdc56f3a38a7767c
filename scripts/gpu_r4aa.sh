#!/bin/bash
# Round 4, call aa: sharded routing on grk_sort_pairs:
# stream (train._sharded_warm_step): the RCCL sharding tests, then the world-1
# row-sharded bench with graph capture (crashed in capture_end in r4k / r4n / r4o).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4aa
mkdir -p $O
timeout -k 10 400 python -u -m pytest -m gpu -v --timeout 240 --timeout-method thread tests/test_gpu_sharding.py \
  tests/test_gpu_sharding_c3.py tests/test_gpu_sharding_world2.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/summary.txt
[ $rc -le 1 ] || exit $rc
PYTHONFAULTHANDLER=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29623 bench.py --sharded 1 --cpu-baseline 0 --roofline-reps 1 \
  > $O/sharded1.json 2> $O/sharded1.err
echo "sharded1 rc=$?" >> $O/summary.txt
cat $O/summary.txt; grep -E "passed|failed" $O/tests.log | tail -1; cut -c1-200 $O/sharded1.json | tail -1
