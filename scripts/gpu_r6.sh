#!/bin/bash
# Round-6 GPU call: the default GPU suite (no -x), the default bench line, then
# optional extra steps named on the command line (each a script under scripts/diag
# or a bench variant), each under its own time limit; a GPU fault ends the call.
# Usage (via gpurun): bash scripts/gpu_r6.sh TAG [suite=1] [bench=1] [extra commands...]
set -o pipefail
TAG=${1:-r6}
SUITE=${2:-1}
BENCH=${3:-1}
shift 3 2>/dev/null
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$TAG
FAULT='illegal memory access|memory access fault|HSA_STATUS_ERROR|hipErrorIllegalAddress|HW Exception|GPU Hang|page not present'
if [ "$SUITE" = 1 ]; then
  timeout -k 10 780 python -u -m pytest tests -m gpu -v -rs --durations=25 --timeout 200 --timeout-method thread \
    > gpurun_out/$TAG/gputest.log 2>&1
  rc=$?
  echo "pytest rc=$rc" >> gpurun_out/$TAG/gputest.log
  tail -3 gpurun_out/$TAG/gputest.log
  grep -Eqi "$FAULT" gpurun_out/$TAG/gputest.log && { echo "GPU fault in the suite -- stopping"; exit 3; }
  case $rc in 0|1) ;; *) echo "pytest exit $rc -- stopping"; exit $rc ;; esac
fi
if [ "$BENCH" = 1 ]; then
  timeout -k 10 400 python -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
  rc=$?
  echo "bench rc=$rc"
  [ $rc = 0 ] || exit $rc
fi
i=0
for cmd in "$@"; do
  i=$((i+1))
  echo "extra $i: $cmd"
  timeout -k 10 400 bash -c "$cmd" > gpurun_out/$TAG/extra$i.log 2>&1
  rc=$?
  echo "extra $i rc=$rc"
  grep -Eqi "$FAULT" gpurun_out/$TAG/extra$i.log && { echo "GPU fault -- stopping"; exit 3; }
  case $rc in 0|1) ;; *) exit $rc ;; esac
done
