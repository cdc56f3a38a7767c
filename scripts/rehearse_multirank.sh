#!/usr/bin/env bash
# Rehearse the N-rank row-sharded training path on ONE GPU: N processes share
# cuda:0 and talk over gloo (collectives staged through host memory).  The
# real multi-GPU run uses RCCL ("nccl"), one process per GPU:
#   python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
#       --master-addr 127.0.0.1 --master-port 29500 bench.py --gpus 8
set -euo pipefail
N=${1:-2}
cd "$(dirname "$0")/.."
python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
    --master-port "${PORT:-29531}" bench.py --gpus "$N" --backend gloo --steps 3 --warmup 1 \
    --cpu-baseline 0 --roofline-reps 2 "${@:2}"
