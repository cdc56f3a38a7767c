#!/bin/bash
# A/B of builds of libgrk.so on one box: bench.py with each (GRK_LIB), round-robin.
# Usage (via gpurun): bash scripts/gpu_ab.sh ROUNDS "libA.so libB.so ..." [bench args]
set -e -o pipefail
N=$1; LIBS=$2; shift 2
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/ab.txt
for i in $(seq 1 $N); do
  for lib in $LIBS; do
    v=$(basename $lib .so)
    GRK_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --cpu-baseline 0 --roofline-reps 5 "$@" > gpurun_out/ab_$v$i.json 2>/dev/null
    python - "$v" "gpurun_out/ab_$v$i.json" >> gpurun_out/ab.txt <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read())
rl = {r['kernel'][:40]: r.get('avg_launch_us') for r in [d['roofline']] + d['rooflines']}
g = [v for k, v in rl.items() if 'k_gather' in k]
print(sys.argv[1], d['value'], d['ms_per_step'], 'gathers(us)', g)
PY
  done
done
