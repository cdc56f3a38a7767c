#!/usr/bin/env python
"""Summarise rocprofv3 output into profiles/ (committed evidence).

    python scripts/summarize_profile.py stats  <run_kernel_stats.csv> <steps> <out.txt>
    python scripts/summarize_profile.py pmc    <fetch counter csv> <write counter csv> <kernel substring> <out.json>

`pmc` applies the gfx950 corrections of MI355X_MICROARCH.md §HBM: FETCH_SIZE
(KiB) reads exactly half the bytes of a wide coalesced stream -> x2;
WRITE_SIZE (KiB) reads the bytes exactly for 16-B-per-lane stores.  Counters
come from separate --pmc passes (FETCH_SIZE and WRITE_SIZE do not fit one).
"""
import csv
import json
import re
import sys


def category(name):
    if 'grk::' in name:
        m = re.search(r'grk::(?:\(anonymous namespace\)::)?(\w+)', name)
        return 'grk:' + (m.group(1) if m else name)
    if name.startswith('Cijk') or name.startswith('Custom_Cijk'):
        return 'GEMM (hipBLASLt)'
    if 'elementwise' in name:
        return 'torch elementwise'
    if 'layer_norm' in name or 'GammaBeta' in name:
        return 'torch layernorm'
    if 'reduce_kernel' in name:
        return 'torch reduce'
    if 'rocprim' in name:
        return 'rocprim (sort/scan)'
    return 'other: ' + name[:60]


def stats(path, steps, out):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r['TotalDurationNs']) for r in rows)
    cats = {}
    for r in rows:
        c = category(r['Name'])
        cats[c] = cats.get(c, 0.0) + float(r['TotalDurationNs'])
    lines = [f'# rocprofv3 --kernel-trace --stats summary ({path})',
             f'# total kernel time {tot / 1e6:.2f} ms over {steps} step-equivalents -> {tot / 1e6 / steps:.3f} ms/step',
             '', '## by category (ms per step, share)']
    for c, t in sorted(cats.items(), key=lambda x: -x[1]):
        lines.append(f'{t / 1e6 / steps:9.3f}  {100 * t / tot:5.1f}%  {c}')
    lines += ['', '## top kernels (total ms, calls, avg us)']
    for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:40]:
        lines.append(f"{float(r['TotalDurationNs']) / 1e6:9.3f} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.1f}  "
                     f"{r['Name'][:140]}")
    open(out, 'w').write('\n'.join(lines) + '\n')
    print('\n'.join(lines[:30]))


def pmc(fetch_csv, write_csv, kernel, out, last=5):
    def read(p, counter):
        rows = [r for r in csv.DictReader(open(p)) if kernel in r['Kernel_Name'] and r['Counter_Name'] == counter]
        # the largest grid = the seq-side launch (bench.py's roofline replays); keep the last replays
        big = max(int(r['Grid_Size']) for r in rows)
        rows = [r for r in rows if int(r['Grid_Size']) == big][-last:]
        return rows
    f = read(fetch_csv, 'FETCH_SIZE')
    w = read(write_csv, 'WRITE_SIZE')
    fetch_b = 2 * 1024 * sum(float(r['Counter_Value']) for r in f) / len(f)
    write_b = 1024 * sum(float(r['Counter_Value']) for r in w) / len(w)
    res = {'kernel': kernel, 'grid_size': int(f[0]['Grid_Size']), 'launches_averaged': len(f),
           'fetch_bytes_per_launch': fetch_b, 'write_bytes_per_launch': write_b,
           'traffic_bytes_per_launch': fetch_b + write_b,
           'method': 'rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; FETCH_SIZE x2 (gfx950 '
                     'wide-stream correction, MI355X_MICROARCH.md HBM), KiB -> bytes'}
    json.dump(res, open(out, 'w'), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    if sys.argv[1] == 'stats':
        stats(sys.argv[2], float(sys.argv[3]), sys.argv[4])
    else:
        pmc(sys.argv[2], sys.argv[3], sys.argv[4], sys.argv[5])
