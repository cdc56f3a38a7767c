#!/bin/bash
# r5q: rolling slice with a bounded grid (GRK_SLICE_WGS) -- bitwise tests, then a same-box A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5q
GRK_SLICE_WGS=256 timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  "tests/test_gpu_model.py::test_deferred_table_updates_are_bit_identical_to_dense" \
  tests/test_gpu_bench_size.py > gpurun_out/r5q/tests.log 2>&1 || { tail -30 gpurun_out/r5q/tests.log; exit 1; }
tail -2 gpurun_out/r5q/tests.log
for i in 1 2; do
  for w in 0 256 512 1024; do
    GRK_SLICE_WGS=$w timeout -k 10 200 python -u bench.py --cpu-baseline 0 --roofline-reps 3 \
      > gpurun_out/r5q/ab_${w}_$i.json 2> gpurun_out/r5q/ab_${w}_$i.err || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('wgs', sys.argv[2], d['value'], d['ms_per_step'])" \
      gpurun_out/r5q/ab_${w}_$i.json $w | tee -a gpurun_out/r5q/ab.txt
  done
done
