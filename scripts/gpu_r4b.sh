#!/bin/bash
# Round 4, call b: the default GPU suite (fixes of r4a), then the opt-in paths'
# tests (scripts/gpu_validate_pending.sh tests, without its bench lines).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_suite.sh r4b 0 || exit $?
GRK_PENDING_NO_BENCH=1 bash scripts/gpu_validate_pending.sh tests
