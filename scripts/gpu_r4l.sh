#!/bin/bash
# Round 4, call l: the whole GPU suite (no -x: every failure listed) after the
# grk_gemm validation fix (only the [m, n] block of a strided output compared) and
# the pos / neg gradient aliasing fix; C5 model tests with the gate lifted; the default
# bench and the C5 bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4l
mkdir -p $O
FAULT='illegal memory access|memory access fault|HSA_STATUS_ERROR|hipErrorIllegalAddress|HW Exception|GPU Hang|page not present'
check() {  # name rc
  echo "$1 rc=$2" >> $O/summary.txt
  if grep -Eqi "$FAULT" $O/$1.log; then echo "$1: GPU fault -- stopping" >> $O/summary.txt; exit 3; fi
  case $2 in 0|1) return 0 ;; *) echo "$1: exit $2 -- stopping" >> $O/summary.txt; exit $2 ;; esac
}
timeout -k 10 780 python -u -m pytest -m gpu -v -rs --timeout 240 --timeout-method thread tests \
  > $O/tests.log 2>&1; check tests $?
timeout -k 10 200 python -u bench.py --cpu-baseline 0 --roofline-reps 5 > $O/bench.json 2> $O/bench.log; check bench $?
timeout -k 10 200 python -u bench.py --fp8 1 --hidden 1024 --maxlen 1024 --batch 16 --steps 10 --warmup 3 \
  --cpu-baseline 0 --roofline-reps 3 > $O/bench_c5.json 2> $O/bench_c5.log; check bench_c5 $?
grep -E "passed|failed" $O/tests.log | tail -2
