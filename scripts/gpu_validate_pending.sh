#!/bin/bash
# GPU calls that validate the paths written without hardware at the end of
# round 3 and A/B the prepared build variants.
#
# In the build container first:
#   make
#   bash scripts/build_variant.sh ch64 grk_embedding "-DGRK_CHUNKED_CH=64"
#   bash scripts/build_variant.sh ch128 grk_embedding "-DGRK_CHUNKED_CH=128"
#   bash scripts/build_variant.sh pipe32 grk_embedding "-DGRK_WAVE_PIPE=32"
#   bash scripts/build_variant.sh tbsplit grk_attention_seq "-DGRK_ATTN_TB_SPLIT=1"
#   bash scripts/build_variant.sh foldtb grk_attention_seq "-DGRK_ATTN_FOLD_INVN=1 -DGRK_ATTN_TB_SPLIT=1"
#   mkdir -p mbbin && hipcc --offload-arch=gfx950 -O3 -o mbbin/mfma_scale_probe scripts/microbench/mfma_scale_probe.hip
# then one gpurun call per stage, least risky first:
#   gpurun --timeout 900 -- bash scripts/gpu_validate_pending.sh tests
#   gpurun --timeout 900 -- bash scripts/gpu_validate_pending.sh variants
#   gpurun --timeout 900 -- bash scripts/gpu_validate_pending.sh ab
#   gpurun --timeout 600 -- bash scripts/gpu_c5.sh
#   (c5lib: the torch GEMM forms at the C5 projection shape, diagnostic only)
# Every step has its own time limit.  A step whose tests merely fail (pytest
# exit 1) lets the independent steps after it run; a GPU fault (its message in
# the log -- torch reports an illegal access as an ordinary exception), an
# abort, a crash or a time limit ends the call there.  gpurun_out/pending/
# summary.txt lists each step's exit status.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/pending
mkdir -p $O
PYT="python -u -m pytest -v -rs --timeout 300 --timeout-method thread"
FAULT='illegal memory access|memory access fault|HSA_STATUS_ERROR|hipErrorIllegalAddress|hipErrorLaunchFailure|HW Exception|GPU Hang|page not present'

# step NAME SECONDS CMD...: run CMD under its own limit, output to $O/NAME.log
step() {
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $O/summary.txt
  if grep -Eqi "$FAULT" "$O/$name.log"; then
    echo "$name: GPU fault reported -- stopping" >> $O/summary.txt
    exit 3
  fi
  case $rc in
    0|1|5) return 0 ;;                       # passed / tests failed / none selected
    *) echo "$name: exit $rc -- stopping" >> $O/summary.txt; exit "$rc" ;;
  esac
}

case "${1:-tests}" in
  tests)
    # opt-in tests of the round-3 paths (product library), least new device code first
    step merge_proj 300 env GRK_MERGE_PROJ_TESTS=1 $PYT tests/test_gpu_embedding.py tests/test_gpu_jagged.py \
      -k "bf16_dense or merged_projection"
    step sharded_jagged 300 env GRK_SHARDED_JAGGED_TESTS=1 $PYT tests/test_gpu_sharding.py -k sharded_jagged
    step time_bias 400 env GRK_CHUNKED_TIME_TESTS=1 $PYT tests/test_gpu_attention.py -k time_bias
    step wide_fidelity 400 env GRK_WIDE_FIDELITY_TESTS=1 $PYT tests/test_gpu_attention.py tests/test_gpu_model.py \
      -k wide_fidelity
    step dense_flat 300 env GRK_DENSE_FLAT_TESTS=1 $PYT tests/test_gpu_dense_flat.py
    [ -n "$GRK_PENDING_NO_BENCH" ] && exit 0
    timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --cpu-baseline 0 --roofline-reps 5 --merge-proj 1 \
      > $O/bench_merge_proj.json 2> $O/bench_merge_proj.err
    echo "bench_merge_proj rc=$?" >> $O/summary.txt
    timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --cpu-baseline 0 --roofline-reps 5 --dense-flat 1 \
      > $O/bench_dense_flat.json 2> $O/bench_dense_flat.err
    echo "bench_dense_flat rc=$?" >> $O/summary.txt
    timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --cpu-baseline 0 --roofline-reps 5 \
      > $O/bench_default.json 2> $O/bench_default.err
    echo "bench_default rc=$?" >> $O/summary.txt
    ;;
  variants)
    # the variants' parity (the tests restate the chunk order from the library), then
    # the headline call standalone under each embedding variant
    for v in ch64 ch128 pipe32; do
      [ -f abtest/libgrk_$v.so ] || continue
      step emb_$v 300 env GRK_LIB=$PWD/abtest/libgrk_$v.so $PYT tests/test_gpu_embedding.py
    done
    for v in tbsplit foldtb; do
      [ -f abtest/libgrk_$v.so ] || continue
      step attn_$v 400 env GRK_LIB=$PWD/abtest/libgrk_$v.so $PYT tests/test_gpu_attention.py tests/test_gpu_jagged.py
    done
    for lib in tencent_recommendation_2025_amd/libgrk.so abtest/libgrk_ch64.so abtest/libgrk_ch128.so \
               abtest/libgrk_pipe32.so; do
      [ -f $lib ] || continue
      step micro_$(basename $lib .so) 120 env GRK_LIB=$PWD/$lib python -u scripts/microbench/emb_bwd.py
    done
    ;;
  ab)
    # bench A/B, round-robin (scripts/gpu_ab.sh writes gpurun_out/ab.txt)
    LIBS="tencent_recommendation_2025_amd/libgrk.so"
    for v in ch64 ch128 pipe32 tbsplit foldtb; do
      [ -f abtest/libgrk_$v.so ] && LIBS="$LIBS abtest/libgrk_$v.so"
    done
    bash scripts/gpu_ab.sh 2 "$LIBS" --steps 30 --warmup 10 && cp gpurun_out/ab.txt $O/ab.txt
    ;;
  c5)
    # last: the d = 1024 model step faulted inside torch's batched GEMM in round 3.
    # First the projection shape alone on the path the model now takes (grk_gemm per
    # block), in its own process; the model tests only if it is right.
    # the block-scaled fp8 MFMA's operand and scale maps (one wave), for the C5 kernels
    [ -x mbbin/mfma_scale_probe ] && step mfma_scale_probe 60 mbbin/mfma_scale_probe
    step c5_grk_gemm 120 python -u scripts/diag/c5_gemm_isolate.py grk
    grep -q "grk: normwise .* ok" $O/c5_grk_gemm.log || { echo "c5: projection GEMM not ok -- stopping" >> $O/summary.txt; exit 4; }
    step c5 400 env GRK_C5_MODEL_TESTS=1 $PYT tests/test_gpu_fp8.py
    ;;
  c5lib)
    # which torch GEMM form faults at the C5 projection shape (library behaviour, not the
    # product path): non-batched, batched contiguous, then the round-3 strided call.
    # Expect the call to end at the first fault (one gpurun strike).
    for s in torch_mm torch_bmm torch_bmm_strided; do
      step c5_$s 120 python -u scripts/diag/c5_gemm_isolate.py $s
    done
    ;;
  *)
    echo "usage: $0 tests|variants|ab|c5|c5lib" >&2
    exit 2
    ;;
esac
