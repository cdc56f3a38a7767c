#!/bin/bash
# r5t: key-valid bytes staged in LDS + the jagged row bases in the same one-workgroup launch --
# parity, then a same-box A/B against the build before (abvar/libgrk_base.so)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5t
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  "tests/test_gpu_attention.py::test_seq_ranges" "tests/test_gpu_attention.py::test_seq_ranges_random" \
  "tests/test_gpu_attention.py::test_precomputed_ranges_bitwise_equal" \
  tests/test_gpu_jagged.py tests/test_gpu_bench_size.py > gpurun_out/r5t/tests.log 2>&1 || { tail -30 gpurun_out/r5t/tests.log; exit 1; }
tail -2 gpurun_out/r5t/tests.log
for i in 1 2 3; do
  for v in new base; do
    if [ $v = base ]; then L=$PWD/abvar/libgrk_base.so; else L=$PWD/tencent_recommendation_2025_amd/libgrk.so; fi
    GRK_LIB=$L timeout -k 10 200 python -u bench.py --cpu-baseline 0 --roofline-reps 3 \
      > gpurun_out/r5t/ab_${v}$i.json 2> gpurun_out/r5t/ab_${v}$i.err || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" \
      gpurun_out/r5t/ab_${v}$i.json $v | tee -a gpurun_out/r5t/ab.txt
  done
done
