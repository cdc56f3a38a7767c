#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes over grk_rq_assign at config 4's shape, summarised
# with the gfx950 corrections (scripts/summarize_profile.py pmc).
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for c in FETCH_SIZE WRITE_SIZE; do
  d=/tmp/rqpmc_$c
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $d -o run -- python scripts/rq_bench.py --first > gpurun_out/rqpmc_$c.log 2>&1
  mkdir -p gpurun_out/rqpmc_$c
  find $d -name "*counter_collection.csv" -exec cp {} gpurun_out/rqpmc_$c/ \;
done
python scripts/summarize_profile.py pmc gpurun_out/rqpmc_FETCH_SIZE/*.csv gpurun_out/rqpmc_WRITE_SIZE/*.csv k_rq_assign gpurun_out/r2s7_pmc_rq_assign.json
