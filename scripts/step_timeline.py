#!/usr/bin/env python
"""Dump one training step of a rocprofv3 kernel trace as a timeline.

    python scripts/step_timeline.py <kernel_trace.csv> [marker] [steps_from_end | +k]

One line per kernel: start (us, relative to the step's marker kernel),
duration (us), queue / stream ids, name -- which stream a kernel ran on and
what it waited behind."""
import csv
import sys


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else 'k_seq_ranges'
    arg = sys.argv[3] if len(sys.argv) > 3 else '2'
    back = int(arg)
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r.get('Queue_Id', '?'),
                         r.get('Stream_Id', '?'), r['Kernel_Name']))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if marker in r[4]]
    if arg.startswith('+'):   # '+k': the k-th marker from the start
        lo, hi = starts[back], starts[back + 1]
    else:
        lo, hi = starts[-back - 1], starts[-back]
    t0 = rows[lo][0]
    for s, e, q, st, n in rows[lo:hi]:
        print(f'{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f}  q{q:>3} s{st:>3}  {n[:90]}')


if __name__ == '__main__':
    main()
