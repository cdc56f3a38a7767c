#!/bin/bash
# Round-6 bench lines beside the default one (each its own process and time limit):
# sampled-softmax loss, row-sharded world 1, BASELINE config 4 (RQ-VAE semantic ids)
# and config 5 (fp8, d = 1024, T = 1025).  Outputs gpurun_out/TAG/bench_<name>.json.
# Usage (via gpurun): bash scripts/gpu_lines.sh TAG [names...]
set -o pipefail
TAG=${1:-r6lines}
shift
NAMES=${@:-default sampled_softmax sharded1 c4 c5}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$TAG
for n in $NAMES; do
  case $n in
    default) args="" ;;
    sampled_softmax) args="--loss sampled_softmax --cpu-baseline 0" ;;
    sharded1) args="--sharded 1 --cpu-baseline 0" ;;
    c4) args="--semantic-ids 3 --cpu-baseline 0" ;;
    c5) args="--fp8 1 --hidden 1024 --maxlen 1024 --batch 16 --cpu-baseline 0 --steps 12" ;;
    *) echo "unknown line $n"; exit 2 ;;
  esac
  echo "line $n: bench.py $args"
  timeout -k 10 500 python -u bench.py $args > gpurun_out/$TAG/bench_$n.json 2> gpurun_out/$TAG/bench_$n.err
  rc=$?
  echo "line $n rc=$rc"
  [ $rc = 0 ] || exit $rc
done
