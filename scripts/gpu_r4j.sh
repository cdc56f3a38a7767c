#!/bin/bash
# Round 4, call j: the fused dnn forms (ReLU epilogue, in-place addend) and the
# GEMM-validation fix under the model / jagged / seqstore / linear tests; config C5
# (d = 1024, T = 1025, fp8 attention): the projection GEMM alone, the d = 1024
# model tests, a C5 bench line; then the default bench and a step breakdown.
# (The round-3 torch.bmm fault is not reproduced: the model no longer issues it.)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4j
mkdir -p $O
FAULT='illegal memory access|memory access fault|HSA_STATUS_ERROR|hipErrorIllegalAddress|HW Exception|GPU Hang|page not present'
check() {  # name rc
  echo "$1 rc=$2" >> $O/summary.txt
  if grep -Eqi "$FAULT" $O/$1.log; then echo "$1: GPU fault -- stopping" >> $O/summary.txt; exit 3; fi
  case $2 in 0|1) return 0 ;; *) echo "$1: exit $2 -- stopping" >> $O/summary.txt; exit $2 ;; esac
}
timeout -k 10 600 python -u -m pytest -v -rs --timeout 200 --timeout-method thread tests/test_gpu_embedding.py tests/test_gpu_linear.py \
  tests/test_gpu_seqstore.py tests/test_gpu_model.py tests/test_gpu_jagged.py tests/test_gpu_ggemm.py tests/test_gpu_emb_combine.py \
  > $O/tests.log 2>&1; check tests $?
timeout -k 10 120 python -u scripts/diag/c5_gemm_isolate.py grk > $O/c5_gemm.log 2>&1; check c5_gemm $?
GRK_C5_MODEL_TESTS=1 timeout -k 10 400 python -u -m pytest -v -rs --timeout 300 --timeout-method thread \
  tests/test_gpu_fp8.py > $O/c5_tests.log 2>&1; check c5_tests $?
timeout -k 10 300 python -u bench.py --fp8 1 --hidden 1024 --maxlen 1024 --batch 16 --steps 10 --warmup 3 \
  --cpu-baseline 0 --roofline-reps 3 > $O/bench_c5.json 2> $O/bench_c5.log; check bench_c5 $?
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.log; check bench $?
# the N = 2 path (row-sharded, jagged rows, lockstep prewarm) rehearsed with two gloo ranks on this one GPU
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 2 --steps 6 --warmup 2 --backend gloo --cpu-baseline 0 --roofline-reps 1 \
  > $O/bench_world2.json 2> $O/bench_world2.log; check bench_world2 $?
MODES=fused bash scripts/gpu_step_profiles.sh || exit $?
cp gpurun_out/step_breakdown_fused.txt $O/step_breakdown.txt
cp gpurun_out/step_timeline_fused.txt $O/step_timeline.txt
tail -3 $O/tests.log
