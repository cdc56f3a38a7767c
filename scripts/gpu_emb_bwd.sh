#!/bin/bash
# Embedding-backward GPU check: kernel tests, microbench, per-launch kernel trace.
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_embedding.py -x -v --timeout 120 --timeout-method thread > gpurun_out/emb_test.log 2>&1
timeout -k 10 120 python -u scripts/microbench/emb_bwd.py > gpurun_out/emb_bwd.log 2>&1
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d /tmp/ebp -o run -- python -u scripts/microbench/emb_bwd.py > gpurun_out/emb_bwd_prof.log 2>&1
python scripts/microbench/emb_bwd_trace.py $(find /tmp/ebp -name "*kernel_trace.csv" | head -1) > gpurun_out/emb_bwd_trace.txt
