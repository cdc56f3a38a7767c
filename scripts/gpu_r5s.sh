#!/bin/bash
# r5s: the dnn-weight composition kernels -- parity, then a same-box A/B (with the slice grid cap)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5s
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_dnn_weight.py tests/test_gpu_model.py tests/test_gpu_bench_size.py > gpurun_out/r5s/tests.log 2>&1 || { tail -40 gpurun_out/r5s/tests.log; exit 1; }
tail -2 gpurun_out/r5s/tests.log
for i in 1 2; do
  for cfg in "1 512" "0 512" "1 0" "0 0"; do
    set -- $cfg
    GRK_DNNW_KERNEL=$1 GRK_SLICE_WGS=$2 timeout -k 10 200 python -u bench.py --cpu-baseline 0 --roofline-reps 3 \
      > gpurun_out/r5s/ab_$1_$2_$i.json 2> gpurun_out/r5s/ab_$1_$2_$i.err || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('dnnw', sys.argv[2], 'wgs', sys.argv[3], d['value'], d['ms_per_step'])" \
      gpurun_out/r5s/ab_$1_$2_$i.json $1 $2 | tee -a gpurun_out/r5s/ab.txt
  done
done
