#!/bin/bash
# One GPU call: the whole default GPU suite WITHOUT -x (every test runs and
# reports), then the default bench line.  A GPU fault in the suite's log ends
# the call before the bench.
# Usage (via gpurun): bash scripts/gpu_suite.sh TAG [bench=1]
set -o pipefail
TAG=${1:-r4}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
FAULT='illegal memory access|memory access fault|HSA_STATUS_ERROR|hipErrorIllegalAddress|HW Exception|GPU Hang|page not present'
timeout -k 10 780 python -u -m pytest tests -m gpu -v -rs --durations=25 --timeout 200 --timeout-method thread \
  > gpurun_out/${TAG}_gputest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${TAG}_gputest.log
grep -Eqi "$FAULT" gpurun_out/${TAG}_gputest.log && { echo "GPU fault in the suite -- stopping"; exit 3; }
case $rc in 0|1) ;; *) echo "pytest exit $rc -- stopping"; exit $rc ;; esac
if [ "${2:-1}" = 1 ]; then
  timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
  echo "bench rc=$?"
fi
tail -3 gpurun_out/${TAG}_gputest.log
