#!/bin/bash
# Round 4, call v: quantum 512 vs 1024 at 32 timed steps, alternating, twice each (confirmation of call t).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4v
mkdir -p $O
for i in 1 2; do
  for q in 512 1024; do  # 32 timed steps (default): two segment flushes in every run
    timeout -k 10 240 python -u bench.py --cpu-baseline 0 --roofline-reps 2 --jagged-quantum $q > $O/q$q-$i.json 2> $O/q$q-$i.err || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('q=$q run $i', d['value'], d['ms_per_step'], d['config']['layout'])" $O/q$q-$i.json >> $O/summary.txt
  done
done
cat $O/summary.txt
