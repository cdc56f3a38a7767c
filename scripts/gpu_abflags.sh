#!/bin/bash
# A/B of bench configurations on one box, round-robin: each spec is
# "name|ENV=VAL ...|bench args" (env and args may be empty).  One JSON line per
# run in gpurun_out/abf_<name><round>.json, a summary in gpurun_out/abf.txt.
# Usage (via gpurun): bash scripts/gpu_abflags.sh ROUNDS "spec" "spec" ...
set -o pipefail
N=$1; shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
: > gpurun_out/abf.txt
for i in $(seq 1 $N); do
  for spec in "$@"; do
    name=${spec%%|*}; rest=${spec#*|}; envs=${rest%%|*}; args=${rest#*|}
    env $envs timeout -k 10 200 python -u bench.py --cpu-baseline 0 --roofline-reps 5 --steps 30 --warmup 10 $args \
      > gpurun_out/abf_$name$i.json 2> gpurun_out/abf_$name$i.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "$name round $i: exit $rc" >> gpurun_out/abf.txt; [ $rc -ge 124 ] && exit $rc; continue; fi
    python - "$name" "gpurun_out/abf_$name$i.json" >> gpurun_out/abf.txt <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ents = [d['roofline']] + d.get('rooflines', [])
def us(*needles):
    return [r.get('avg_launch_us') for r in ents if all(n in r.get('kernel', '') for n in needles)]
print(sys.argv[1], round(d['value']), d['ms_per_step'], 'wgrad(us)', us('wgrad'), 'dkdv(us)', us('dkdv'),
      'emb_bwd(us)', us('grk_embedding_backward'))
PY
  done
done
cat gpurun_out/abf.txt
