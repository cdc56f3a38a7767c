#!/bin/bash
# quick GPU microbenches: bash scripts/gpu_micro.sh "<pytest selection or none>" <script> [<script> ...]
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
SEL=$1; shift
if [ "$SEL" != none ]; then
  timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/micro_test.log 2>&1
fi
: > gpurun_out/micro.log
for s in "$@"; do
  timeout -k 10 180 python -u $s >> gpurun_out/micro.log 2>&1
done
