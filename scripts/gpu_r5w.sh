#!/bin/bash
# r5w: HSTU dK/dV with 1/n folded into the store scales and the time-bias-free instantiation --
# the attention parity tests on that build, then a 3-pair same-box A/B against the product build
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5w
GRK_LIB=$PWD/abvar/libgrk_foldtb.so timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_attention.py tests/test_gpu_jagged.py > gpurun_out/r5w/tests.log 2>&1 || { tail -30 gpurun_out/r5w/tests.log; exit 1; }
tail -2 gpurun_out/r5w/tests.log
for i in 1 2 3; do
  for v in foldtb product; do
    if [ $v = foldtb ]; then L=$PWD/abvar/libgrk_foldtb.so; else L=$PWD/tencent_recommendation_2025_amd/libgrk.so; fi
    GRK_LIB=$L timeout -k 10 200 python -u bench.py --cpu-baseline 0 --roofline-reps 3 \
      > gpurun_out/r5w/ab_${v}$i.json 2> gpurun_out/r5w/ab_${v}$i.err || exit 1
    python -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
dk=[r.get('avg_launch_us') for r in d['rooflines'] if 'dkdv' in r.get('kernel','')]
print(sys.argv[2], d['value'], d['ms_per_step'], 'dkdv us', dk)" gpurun_out/r5w/ab_${v}$i.json $v | tee -a gpurun_out/r5w/ab.txt
  done
done
