#!/bin/bash
# Round 4, call ab (final check after the sharded routing-sort change): the whole GPU suite as the driver runs it (-x), smoke(), the
# default bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4ab
mkdir -p $O
timeout -k 10 780 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/summary.txt; tail -3 $O/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> $O/summary.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.log
echo "bench rc=$?" >> $O/summary.txt
cat $O/summary.txt; cut -c1-160 $O/bench.json
