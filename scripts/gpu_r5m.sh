#!/bin/bash
# Round 5, call m: where the flush slice overlaps (GRK_SLICE_AT forward / backward) and
# the capture stream's priority (GRK_MAIN_PRIORITY=-1); bitwise deferred / graph tests with the backward fork.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5m
mkdir -p $O
FAULT='illegal memory access|memory access fault|HSA_STATUS_ERROR|hipErrorIllegalAddress|HW Exception|GPU Hang|page not present'
python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())" > $O/prio.txt 2>&1
GRK_SLICE_AT=backward timeout -k 10 500 python -u -m pytest -v -rs --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_model.py -k "deferred or graph_replayed" "tests/test_gpu_fp8.py::test_c5_fp8_trainer_graph_equals_eager" \
  > $O/tests.log 2>&1
echo "tests rc=$?" >> $O/summary.txt
grep -Eqi "$FAULT" $O/tests.log && { echo "GPU fault"; cat $O/summary.txt; exit 3; }
for i in 1; do
  for cfg in "forward 0" "backward 0" "forward -1" "backward -1"; do
    set -- $cfg
    if [ "$2" = 0 ]; then unset GRK_MAIN_PRIORITY; else export GRK_MAIN_PRIORITY=$2; fi
    GRK_SLICE_AT=$1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 \
      --rooflines 0 > $O/bench_${1}_$2_$i.json 2>/dev/null
    echo "bench $1 $2 $i rc=$?" >> $O/summary.txt
  done
done
timeout -k 10 600 bash scripts/gpu_pmc_round.sh r5 > $O/pmc.log 2>&1
echo "pmc rc=$?" >> $O/summary.txt
cp gpurun_out/pmc_r5/r5_pmc_*.json gpurun_out/pmc_r5/summary.txt $O/ 2>/dev/null
cat $O/summary.txt $O/prio.txt; grep -E "passed|failed" $O/tests.log | tail -3
for f in $O/bench_*.json; do echo "$(basename $f) $(grep -o '"ms_per_step": [0-9.]*' $f | head -1)"; done
