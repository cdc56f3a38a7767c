set -e -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_hstu_gate.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/attn_test.log 2>&1
timeout -k 10 400 python -u bench.py --cpu-baseline 0 > gpurun_out/attn_bench.json 2> gpurun_out/attn_bench.err
