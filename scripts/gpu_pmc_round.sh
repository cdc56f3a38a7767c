#!/bin/bash
# PMC traffic of every bench roofline: two counter passes (FETCH_SIZE, WRITE_SIZE),
# per-kernel / per-call summaries (scripts/pmc_rooflines.py) copied to gpurun_out/,
# then a bench run that reads them back.
# Usage (via gpurun): bash scripts/gpu_pmc_round.sh TAG [extra bench args]
set -e -o pipefail
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_$TAG
ARGS="--steps 2 --warmup 1 --cpu-baseline 0 --roofline-reps 3 $*"
for c in FETCH_SIZE WRITE_SIZE; do
  d=/tmp/pmc_$c
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $d -o run -- python bench.py $ARGS > gpurun_out/pmc_$TAG/$c.log 2>&1
done
python scripts/pmc_rooflines.py /tmp/pmc_FETCH_SIZE /tmp/pmc_WRITE_SIZE gpurun_out/pmc_$TAG/WRITE_SIZE.log $TAG 3 \
  > gpurun_out/pmc_$TAG/summary.txt 2>&1
cp profiles/${TAG}_pmc_*.json gpurun_out/pmc_$TAG/
timeout -k 10 300 python bench.py --cpu-baseline 0 $* > gpurun_out/pmc_$TAG/bench.json 2> gpurun_out/pmc_$TAG/bench.err
