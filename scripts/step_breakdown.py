#!/usr/bin/env python
"""Per-step kernel breakdown of the timed region of a rocprofv3 kernel trace.

    python scripts/step_breakdown.py <kernel_trace.csv> [marker] [last_n_steps]

Steps are delimited by the marker kernel (default grk::k_seq_ranges, launched
once per training step); the last N steps are summarised (ms/step by category,
busy time, wall span), so first-use GEMM tuning and warmup are excluded.
"""
import csv
import sys
from collections import defaultdict

from summarize_profile import category


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else 'k_seq_ranges'
    last = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if marker in r[2]]
    if len(starts) < last + 1:
        sys.exit(f'only {len(starts)} marker launches')
    lo, hi = starts[-last - 1], starts[-1]
    sel = rows[lo:hi]
    cat = defaultdict(float)
    top = defaultdict(lambda: [0.0, 0])
    busy = 0.0
    for s, e, n in sel:
        d = (e - s) / 1e6
        busy += d
        cat[category(n)] += d
        top[n[:90]][0] += d
        top[n[:90]][1] += 1
    span = (sel[-1][1] - sel[0][0]) / 1e6
    print(f'# {last} steps: busy {busy / last:.3f} ms/step, span {span / last:.3f} ms/step, '
          f'{len(sel) / last:.0f} launches/step')
    for k, v in sorted(cat.items(), key=lambda kv: -kv[1]):
        print(f'  {v / last:8.3f}  {100 * v / busy:5.1f}%  {k}')
    gaps = sorted(((sel[i + 1][0] - sel[i][1], sel[i][2][:60], sel[i + 1][2][:60]) for i in range(len(sel) - 1)
                   if sel[i + 1][0] > sel[i][1]), reverse=True)
    print(f'# idle gaps: {sum(g[0] for g in gaps) / 1e6 / last:.3f} ms/step; largest (us, after -> before):')
    for g, a, b in gaps[:12]:
        print(f'  {g / 1e3:8.1f}  {a}  ->  {b}')
    print('# top kernels (ms/step, launches/step, avg us)')
    for k, (v, c) in sorted(top.items(), key=lambda kv: -kv[1][0])[:40]:
        print(f'  {v / last:8.3f} {c / last:5.1f} {1e3 * v / c:8.1f}  {k}')


if __name__ == '__main__':
    main()
