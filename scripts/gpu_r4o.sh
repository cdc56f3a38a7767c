#!/bin/bash
# Round 4, call o: the world-1 row-sharded bench step (a) eager (no graph capture)
# and, only if that ran, (b) graph-captured without dropout -- the capture_end crash
# of r4n bisected one switch at a time.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4o
mkdir -p $O
run() {  # name args...
  local n=$1; shift
  PYTHONFAULTHANDLER=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29618 bench.py --sharded 1 --cpu-baseline 0 --rooflines 0 "$@" \
    > $O/$n.json 2> $O/$n.err
  local rc=$?; echo "$n rc=$rc" >> $O/summary.txt; return $rc
}
run eager --graph 0 --steps 10 --warmup 3 && run graph_nodrop --dropout 0 --steps 10 --warmup 3
cat $O/summary.txt
