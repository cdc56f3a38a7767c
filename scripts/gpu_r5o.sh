#!/bin/bash
# r5o: host issue time of the row-sharded world-1 step's eager phases (GRK_HOST_TIMES=1)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5o
GRK_HOST_TIMES=1 timeout -k 10 300 python -u bench.py --sharded 1 --cpu-baseline 0 --roofline-reps 3 \
  > gpurun_out/r5o/sharded_host.json 2> gpurun_out/r5o/sharded_host.err || { tail -20 gpurun_out/r5o/sharded_host.err; exit 1; }
grep -E "host issue|fraction of" gpurun_out/r5o/sharded_host.err
python -c "import json; d=json.loads(open('gpurun_out/r5o/sharded_host.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])"
