#!/bin/bash
# A/B of two builds of libgrk.so on one box: bench.py alternately with each (GRK_LIB).
# Usage (via gpurun): bash scripts/gpu_ab.sh libA.so libB.so ROUNDS [bench args]
set -e -o pipefail
A=$1; B=$2; N=$3; shift 3
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/ab.txt
for i in $(seq 1 $N); do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    GRK_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --cpu-baseline 0 --roofline-reps 2 "$@" > gpurun_out/ab_$v$i.json 2>/dev/null
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab_$v$i.json').read()); print('$v', d['value'], d['ms_per_step'])" >> gpurun_out/ab.txt
  done
done
