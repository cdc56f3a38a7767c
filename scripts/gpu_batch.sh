#!/bin/bash
# GPU batch: selected tests (or all), bench lines (BCE, sampled softmax), SS step profile.
# usage: bash scripts/gpu_batch.sh TAG "pytest selection"
set -e -o pipefail
TAG=${1:-r2}
SEL=${2:-tests}
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1
timeout -k 10 300 python -u bench.py --cpu-baseline 0 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
timeout -k 10 300 python -u bench.py --cpu-baseline 0 --loss sampled_softmax > gpurun_out/${TAG}_bench_ss.json 2> gpurun_out/${TAG}_bench_ss.err
d=/tmp/kt_ss
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python bench.py --steps 10 --warmup 5 --cpu-baseline 0 --roofline-reps 5 --loss sampled_softmax > gpurun_out/kt_ss.log 2>&1
python scripts/step_breakdown.py $(find $d -name "*kernel_trace.csv" | head -n 1) k_seq_ranges 5 > gpurun_out/${TAG}_step_breakdown_ss.txt
