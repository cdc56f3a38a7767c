#!/bin/bash
# Config 4 on the GPU: RQ-VAE tests, the config-4 bench line, and a kernel-trace
# profile of it.   usage (via gpurun): bash scripts/gpu_rqvae.sh TAG
set -e -o pipefail
TAG=${1:-r2s7}
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rqvae.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_rqvae_test.log 2>&1
timeout -k 10 400 python -u bench.py --semantic-ids 3 --cpu-baseline 0 > gpurun_out/${TAG}_bench_c4.json \
  2> gpurun_out/${TAG}_bench_c4.err
d=/tmp/kt_c4
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python bench.py --steps 10 \
  --warmup 5 --cpu-baseline 0 --roofline-reps 5 --semantic-ids 3 > gpurun_out/kt_c4.log 2>&1
cp $(find $d -name "*kernel_stats.csv" | head -n 1) gpurun_out/${TAG}_kernel_stats_c4.csv
