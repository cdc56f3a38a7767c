#!/bin/bash
# Two rocprofv3 counter passes over a short bench run (FETCH_SIZE, WRITE_SIZE),
# counter CSVs copied to gpurun_out/pmc_{fetch,write}/ for scripts/pmc_rooflines.py.
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
ARGS="--steps 2 --warmup 1 --cpu-baseline 0 --roofline-reps 5"
for c in FETCH_SIZE WRITE_SIZE; do
  d=/tmp/pmc_$c
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $d -o run -- python bench.py $ARGS > gpurun_out/pmc_$c.log 2>&1
  mkdir -p gpurun_out/pmc_$c
  find $d -name "*counter_collection.csv" -exec cp {} gpurun_out/pmc_$c/ \;
done
