#!/bin/bash
# r5r: batch-row catch-up on the side stream (GRK_CATCHUP_SIDE) -- bitwise tests, then a same-box A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5r
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  "tests/test_gpu_model.py::test_deferred_table_updates_are_bit_identical_to_dense" \
  "tests/test_gpu_model.py::test_graph_replay_with_dropout_equals_eager" \
  tests/test_gpu_jagged.py tests/test_gpu_bench_size.py tests/test_gpu_fp8.py > gpurun_out/r5r/tests.log 2>&1 || { tail -30 gpurun_out/r5r/tests.log; exit 1; }
tail -2 gpurun_out/r5r/tests.log
for i in 1 2 3; do
  for c in 1 0; do
    GRK_CATCHUP_SIDE=$c timeout -k 10 200 python -u bench.py --cpu-baseline 0 --roofline-reps 3 \
      > gpurun_out/r5r/ab_${c}_$i.json 2> gpurun_out/r5r/ab_${c}_$i.err || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('catchup_side', sys.argv[2], d['value'], d['ms_per_step'])" \
      gpurun_out/r5r/ab_${c}_$i.json $c | tee -a gpurun_out/r5r/ab.txt
  done
done
