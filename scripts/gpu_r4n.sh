#!/bin/bash
# Round 4, call n: where the world-1 row-sharded bench step dies (SIGSEGV in the
# first warm-up step, r4k / r4m): one run with Python's fault handler on, so the
# crash prints the Python stack of every thread.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4n
mkdir -p $O
PYTHONFAULTHANDLER=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29617 bench.py --sharded 1 --steps 3 --warmup 2 --cpu-baseline 0 \
  --rooflines 0 > $O/sharded1.json 2> $O/sharded1.err
echo "sharded1 rc=$?" >> $O/summary.txt
grep -A40 "Fatal Python error\|Current thread" $O/sharded1.err | head -80
