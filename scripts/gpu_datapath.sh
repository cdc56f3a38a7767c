#!/bin/bash
# data path on the GPU box: seqstore GPU tests + throughput (reference path, SeqStore, + device negatives)
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_seqstore.py tests/test_gpu_sampler.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/seqstore_test.log 2>&1
timeout -k 10 600 python -u scripts/bench_datapath.py --users 2048 --events 300 --device cuda > gpurun_out/datapath.json 2> gpurun_out/datapath.err
