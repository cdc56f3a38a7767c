# Attention parity tests, then per-call timings at the bench's C2 shape.
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/diag/hstu_repeat.py > gpurun_out/diag_repeat.txt 2>&1
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_attention.py tests/test_gpu_hstu_gate.py > gpurun_out/attn_quick_test.log 2>&1
: > gpurun_out/attn_quick.txt
for cfg in "--kind hstu --precise" "--kind softmax --act none --precise" "--kind hstu --precise --T 101" ; do
  timeout -k 10 120 python -u scripts/microbench/attn.py $cfg --reps 50 2>/dev/null >> gpurun_out/attn_quick.txt
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/pa && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pa -o run -- python3 scripts/microbench/attn.py --kind hstu --precise --reps 50 > gpurun_out/attn_quick_prof.log 2>&1
cp $(find /tmp/pa -name "*kernel_stats.csv" | head -1) gpurun_out/attn_quick_stats.csv
