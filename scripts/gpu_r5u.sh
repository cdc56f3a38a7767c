#!/bin/bash
# r5u: LDS-tiled dnn-weight kernels -- parity, then a same-box A/B against the torch composition
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5u
GRK_DNNW_KERNEL=1 timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_dnn_weight.py tests/test_gpu_bench_size.py "tests/test_gpu_model.py::test_bench_config_step_matches_oracle_fp32" \
  > gpurun_out/r5u/tests.log 2>&1 || { tail -30 gpurun_out/r5u/tests.log; exit 1; }
tail -2 gpurun_out/r5u/tests.log
for i in 1 2 3; do
  for k in 1 0; do
    GRK_DNNW_KERNEL=$k timeout -k 10 200 python -u bench.py --cpu-baseline 0 --roofline-reps 3 \
      > gpurun_out/r5u/ab_${k}_$i.json 2> gpurun_out/r5u/ab_${k}_$i.err || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('dnnw', sys.argv[2], d['value'], d['ms_per_step'])" \
      gpurun_out/r5u/ab_${k}_$i.json $k | tee -a gpurun_out/r5u/ab.txt
  done
done
