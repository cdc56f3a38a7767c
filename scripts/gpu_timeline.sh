#!/bin/bash
# Kernel-trace timeline of bench steps: bash scripts/gpu_timeline.sh TAG K [bench args]
set -e -o pipefail
TAG=$1; K=$2; shift 2
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
d=/tmp/kt_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- \
  python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --rooflines 0 "$@" > gpurun_out/kt_$TAG.log 2>&1
kt=$(find $d -name "*kernel_trace.csv" | head -n 1)
python - "$kt" > gpurun_out/${TAG}_markers.txt <<'PY'
import csv, sys
rows = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']) for r in csv.DictReader(open(sys.argv[1])))
m = [r for r in rows if 'k_seq_ranges' in r[2]]
print(len(rows), 'kernels', len(m), 'markers')
for a, b in zip(m, m[1:]):
    print(f'{(b[0] - a[0]) / 1e3:9.1f}')
PY
python scripts/step_timeline.py "$kt" k_seq_ranges +$K > gpurun_out/${TAG}_timeline.txt
python scripts/step_timeline.py "$kt" k_seq_ranges +$((K+1)) > gpurun_out/${TAG}_timeline2.txt
