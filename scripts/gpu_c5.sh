#!/bin/bash
# Round 4, call d: config C5 (d = 1024, T = 1025, fp8 attention) on hardware.
#  1. the block-scaled fp8 MFMA probe (operand / scale maps, one wave)
#  2. the C5 projection GEMM alone on the path the model takes (grk_gemm per block)
#  3. the two d = 1024 model tests (opt-in until this run)
#  4. a C5 bench line (B = 16, T = 1025, d = 1024, fp8 q/k/v, padded layout)
#  5. LAST, diagnostic only: torch's batched bf16 GEMM at the projection shape
#     (the round-3 fault), kernel launches logged by the HIP runtime so the
#     faulting kernel is named; expected to fault -- nothing runs after it.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/c5
mkdir -p $O
FAULT='illegal memory access|memory access fault|HSA_STATUS_ERROR|hipErrorIllegalAddress|HW Exception|GPU Hang|page not present'
check() {  # name rc
  echo "$1 rc=$2" >> $O/summary.txt
  if grep -Eqi "$FAULT" $O/$1.log; then echo "$1: GPU fault -- stopping" >> $O/summary.txt; exit 3; fi
  case $2 in 0|1) return 0 ;; *) echo "$1: exit $2 -- stopping" >> $O/summary.txt; exit $2 ;; esac
}
[ -x mbbin/mfma_scale_probe ] && { timeout -k 10 60 mbbin/mfma_scale_probe > $O/probe.log 2>&1; check probe $?; }
timeout -k 10 120 python -u scripts/diag/c5_gemm_isolate.py grk > $O/grk_gemm.log 2>&1; check grk_gemm $?
grep -q "grk: normwise .* ok" $O/grk_gemm.log || { echo "projection GEMM not ok -- stopping" >> $O/summary.txt; exit 4; }
GRK_C5_MODEL_TESTS=1 timeout -k 10 400 python -u -m pytest -v -rs --timeout 300 --timeout-method thread \
  tests/test_gpu_fp8.py > $O/model_tests.log 2>&1; check model_tests $?
timeout -k 10 300 python -u bench.py --fp8 1 --hidden 1024 --maxlen 1024 --batch 16 --steps 10 --warmup 3 \
  --cpu-baseline 0 --roofline-reps 3 > $O/bench_c5.json 2> $O/bench_c5.err; check bench_c5 $?
# diagnostic: the round-3 fault, isolated (HIP logs each kernel launch: LOG_KERN 0x80 at level 4)
AMD_LOG_LEVEL=4 AMD_LOG_MASK=0x80 timeout -k 10 120 python -u scripts/diag/c5_gemm_isolate.py torch_bmm \
  > $O/torch_bmm.log 2>&1; check torch_bmm $?
AMD_LOG_LEVEL=4 AMD_LOG_MASK=0x80 timeout -k 10 120 python -u scripts/diag/c5_gemm_isolate.py torch_bmm_strided \
  > $O/torch_bmm_strided.log 2>&1; check torch_bmm_strided $?
