#!/bin/bash
# SQ counters of one microbench's kernels: bash scripts/gpu_sq_micro.sh <script> <kernel-regex> <tag>
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --kernel-include-regex "$2" --output-format csv -d /tmp/sq -o run -- python -u $1 > gpurun_out/sq_$3.log 2>&1
cp $(find /tmp/sq -name "*counter_collection.csv" | head -1) gpurun_out/sq_$3.csv
