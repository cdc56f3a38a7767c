#!/bin/bash
# Round 4, call t: jagged capacity quantum sweep (rows of the captured step rounded up
# to a multiple of the quantum: smaller = less padding, more captured graphs).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4t
mkdir -p $O
for q in 256 512 1024; do
  timeout -k 10 240 python -u bench.py --cpu-baseline 0 --roofline-reps 2 --jagged-quantum $q > $O/q$q.json 2> $O/q$q.err || exit 1
  echo "q=$q $(cut -c1-140 $O/q$q.json)" >> $O/summary.txt
done
cat $O/summary.txt
