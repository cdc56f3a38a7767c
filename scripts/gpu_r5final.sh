#!/bin/bash
# round-5 final: profiles on the final build (PMC, step breakdowns, rocprof bench), then the
# whole GPU suite, the default bench line and smoke()
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_r5fin3.sh > gpurun_out/r5fin3.log 2>&1 || { tail -30 gpurun_out/r5fin3.log; exit 1; }
tail -16 gpurun_out/r5fin3.log
bash scripts/gpu_suite.sh r5final 1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5final_smoke.log 2>&1
echo "smoke rc=$?"
