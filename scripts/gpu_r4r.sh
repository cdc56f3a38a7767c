#!/bin/bash
# Round 4, call r: PMC traffic of every bench roofline under the r4 tag (FETCH_SIZE and
# WRITE_SIZE in separate passes), then the bench reading them back.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 700 bash scripts/gpu_pmc_round.sh r4
echo "pmc rc=$?"
tail -12 gpurun_out/pmc_r4/summary.txt
