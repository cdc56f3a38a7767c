#!/bin/bash
# Round 4, call w: the default bench line exactly as the driver runs it (N = 1).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4w
mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.log
echo "bench rc=$?" >> $O/summary.txt
cut -c1-300 $O/bench.json
