# Wide-head attention: parity tests, then per-call timings against the narrow
# kernels at the same hidden width.
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_attention.py tests/test_gpu_model.py -k wide > gpurun_out/wide_test.log 2>&1
: > gpurun_out/wide_bench.txt
for cfg in "--kind softmax --act none --T 101 --H 1 --hd 512" "--kind softmax --act none --T 101 --H 8 --hd 64" "--kind hstu --T 201 --H 1 --hd 512" "--kind hstu --T 201 --H 2 --hd 256" "--kind hstu --T 201 --H 8 --hd 64"; do
  timeout -k 10 120 python -u scripts/microbench/attn.py $cfg --precise 2>/dev/null >> gpurun_out/wide_bench.txt
done
