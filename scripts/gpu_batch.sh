#!/bin/bash
# GPU batch: tests, bench lines (BCE, sampled softmax), step profiles of both.
# usage: bash scripts/gpu_batch.sh TAG "pytest selection" [cpu_baseline 0|1]
set -e -o pipefail
TAG=${1:-r2}
SEL=${2:-tests}
CPU=${3:-0}
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
if [ "$SEL" != none ]; then
  timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1
fi
timeout -k 10 400 python -u bench.py --cpu-baseline $CPU > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
timeout -k 10 300 python -u bench.py --cpu-baseline 0 --loss sampled_softmax > gpurun_out/${TAG}_bench_ss.json 2> gpurun_out/${TAG}_bench_ss.err
for loss in bce sampled_softmax; do
  d=/tmp/kt_$loss
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python bench.py --steps 10 --warmup 5 --cpu-baseline 0 --roofline-reps 5 --loss $loss > gpurun_out/kt_$loss.log 2>&1
  python scripts/step_breakdown.py $(find $d -name "*kernel_trace.csv" | head -n 1) k_seq_ranges 5 > gpurun_out/${TAG}_step_breakdown_$loss.txt
  cp $(find $d -name "*kernel_stats.csv" | head -n 1) gpurun_out/${TAG}_kernel_stats_$loss.csv
done
