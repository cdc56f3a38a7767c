#!/usr/bin/env python
"""Per-step kernel breakdown of a rocprofv3 kernel trace of bench.py, over the
last `steps` training steps (delimited by the one k_pair_logits launch per step).

    python scripts/kernel_window.py <run_kernel_trace.csv> [steps] [top]
"""
import collections
import csv
import sys

path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'k_pair_logits<' in r['Kernel_Name']]
a, b = idx[-steps - 1], idx[-1]
win = rows[a:b]
span = (int(rows[b]['Start_Timestamp']) - int(rows[a]['Start_Timestamp'])) / 1e6 / steps
busy = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in win) / 1e6 / steps
print(f'step span {span:.2f} ms, kernel busy {busy:.2f} ms, {len(win) / steps:.0f} launches/step')
agg = collections.defaultdict(lambda: [0, 0])
for r in win:
    k = r['Kernel_Name'][:84]
    agg[k][0] += int(r['End_Timestamp']) - int(r['Start_Timestamp'])
    agg[k][1] += 1
for k, (t, c) in sorted(agg.items(), key=lambda x: -x[1][0])[:top]:
    print(f'{t / 1e6 / steps:7.3f} ms {c / steps:5.1f}/step {t / c / 1e3:8.1f} us  {k}')
