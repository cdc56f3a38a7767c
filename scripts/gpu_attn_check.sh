#!/bin/bash
# One gpurun call: attention parity tests, then per-kernel timings (rocprofv3
# kernel-trace stats of the microbenchmark).  Every GPU step has its own time
# limit and the chain stops at the first failure.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_attention.py tests/test_gpu_hstu_gate.py -x -q -m gpu > gpurun_out/t_attn.log 2>&1 || { tail -30 gpurun_out/t_attn.log; exit 1; }
tail -1 gpurun_out/t_attn.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for a in "--kind hstu" "--kind hstu --no-drab" "--kind softmax"; do
  rm -rf gpurun_out/prof_attn
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_attn -o run --output-format csv -- python scripts/microbench/attn.py $a --reps 10 > gpurun_out/prof_attn.log 2>&1
  grep -v amdgpu.ids gpurun_out/prof_attn.log | grep "fwd"
  python3 - <<'PY'
import csv, glob
for r in csv.DictReader(open(glob.glob('gpurun_out/prof_attn/*kernel_stats.csv')[0])):
    if 'grk::' in r['Name']:
        print(f"  {float(r['AverageNs']) / 1e3:8.1f} us  {r['Name'][:70]}")
PY
done
