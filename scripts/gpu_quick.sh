#!/bin/bash
# One GPU call: selected GPU test files (or all), then optionally the default bench line.
# Usage (via gpurun): bash scripts/gpu_quick.sh TAG "tests/test_a.py tests/test_b.py|all" [bench=1] [bench args...]
set -e -o pipefail
TAG=${1:-q}
TESTS=${2:-all}
BENCH=${3:-1}
shift 3 || true
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ "$TESTS" = all ]; then TESTS=tests; fi
if [ "$TESTS" != none ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1
fi
if [ "$BENCH" = 1 ]; then
  timeout -k 10 400 python -u bench.py "$@" > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
fi
