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
ents = [d['roofline']] + d['rooflines']
def us(*needles):
    return [r.get('avg_launch_us') for r in ents if all(n in r.get('kernel', '') for n in needles)]
print(sys.argv[1], d['value'], d['ms_per_step'], 'gathers(us)', us('k_gather'), 'dkdv(us)', us('dkdv'),
      'emb_bwd(us)', us('grk_embedding_backward'))
PY
  done
done
