#!/bin/bash
# One GPU call that validates the paths written without hardware at the end of
# round 3 and A/Bs the prepared build variants.
#
# In the build container first:
#   make
#   bash scripts/build_variant.sh ch64 grk_embedding "-DGRK_CHUNKED_CH=64"
#   bash scripts/build_variant.sh ch128 grk_embedding "-DGRK_CHUNKED_CH=128"
#   bash scripts/build_variant.sh pipe32 grk_embedding "-DGRK_WAVE_PIPE=32"
#   bash scripts/build_variant.sh tbsplit grk_attention_seq "-DGRK_ATTN_TB_SPLIT=1"
#   bash scripts/build_variant.sh foldtb grk_attention_seq "-DGRK_ATTN_FOLD_INVN=1 -DGRK_ATTN_TB_SPLIT=1"
# then:
#   gpurun --timeout 1200 -- bash scripts/gpu_validate_pending.sh
# Every step has its own time limit; the first failure ends the call.
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pending
O=gpurun_out/pending
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"

# 1) opt-in tests of the round-3 paths (product library)
GRK_CHUNKED_TIME_TESTS=1 timeout -k 10 400 $PYT tests/test_gpu_attention.py -k "time_bias" > $O/time_bias.log 2>&1
GRK_SHARDED_JAGGED_TESTS=1 timeout -k 10 300 $PYT tests/test_gpu_sharding.py -k "sharded_jagged" > $O/sharded_jagged.log 2>&1
GRK_C5_MODEL_TESTS=1 timeout -k 10 400 $PYT tests/test_gpu_fp8.py > $O/c5.log 2>&1
GRK_WIDE_FIDELITY_TESTS=1 timeout -k 10 400 $PYT tests/test_gpu_attention.py tests/test_gpu_model.py \
  -k "wide_fidelity or 256_fidelity" > $O/wide_fidelity.log 2>&1
GRK_MERGE_PROJ_TESTS=1 timeout -k 10 300 $PYT tests/test_gpu_embedding.py tests/test_gpu_jagged.py \
  -k "bf16_dense or merged_projection" > $O/merge_proj.log 2>&1
timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --cpu-baseline 0 --roofline-reps 5 --merge-proj 1 \
  > $O/bench_merge_proj.json 2> $O/bench_merge_proj.err

# 2) the variants' parity (the tests restate the chunk order from the library)
for v in ch64 ch128 pipe32; do
  [ -f abtest/libgrk_$v.so ] || continue
  GRK_LIB=$PWD/abtest/libgrk_$v.so timeout -k 10 300 $PYT tests/test_gpu_embedding.py > $O/emb_$v.log 2>&1
done
for v in tbsplit foldtb; do
  [ -f abtest/libgrk_$v.so ] || continue
  GRK_LIB=$PWD/abtest/libgrk_$v.so timeout -k 10 400 $PYT tests/test_gpu_attention.py tests/test_gpu_jagged.py \
    > $O/attn_$v.log 2>&1
done

# 3) the headline call standalone under each embedding variant
for lib in tencent_recommendation_2025_amd/libgrk.so abtest/libgrk_ch64.so abtest/libgrk_ch128.so abtest/libgrk_pipe32.so; do
  [ -f $lib ] || continue
  echo "== $lib" >> $O/emb_bwd_micro.txt
  GRK_LIB=$PWD/$lib timeout -k 10 120 python -u scripts/microbench/emb_bwd.py >> $O/emb_bwd_micro.txt 2>&1
done

# 4) bench A/B, round-robin (scripts/gpu_ab.sh writes gpurun_out/ab.txt)
LIBS="tencent_recommendation_2025_amd/libgrk.so"
for v in ch64 ch128 pipe32 tbsplit foldtb; do
  [ -f abtest/libgrk_$v.so ] && LIBS="$LIBS abtest/libgrk_$v.so"
done
bash scripts/gpu_ab.sh 2 "$LIBS" --steps 30 --warmup 10
cp gpurun_out/ab.txt $O/ab.txt
