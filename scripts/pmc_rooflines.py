#!/usr/bin/env python
"""HBM traffic per launch of the bench's roofline kernels from two rocprofv3
counter passes (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950),
written to profiles/ for bench.py's `traffic` field.

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d <F> -o run -- python bench.py --steps 2 --warmup 1 --cpu-baseline 0
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d <W> -o run -- python bench.py ... > <bench.log>
    python scripts/pmc_rooflines.py <F> <W> <bench.log> <round tag, e.g. r1>

Corrections (MI355X_MICROARCH.md, HBM / rocprofv3): FETCH_SIZE (KiB) counts
half the bytes of a wide coalesced stream on gfx950 -> x2; WRITE_SIZE (KiB)
is exact for 16-B-per-lane stores.  The last `--reps` launches of each kernel
(bench.py's roofline replays, same shapes as the training launches) are
averaged; the workload the bench printed is stored with them so bench.py only
uses the numbers for the same workload.
"""
import csv
import glob
import json
import os
import sys

fdir, wdir, log, tag = sys.argv[1:5]
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 5
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counter_rows(d, counter):
    path = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)[0]
    return [r for r in csv.DictReader(open(path)) if r['Counter_Name'] == counter]


def per_launch(rows, needle, pick_largest_grid):
    rows = [r for r in rows if needle in r['Kernel_Name']]
    if pick_largest_grid:
        big = max(int(r['Grid_Size']) for r in rows)
        rows = [r for r in rows if int(r['Grid_Size']) == big]
    # one row per dispatch (a counter may be reported per XCD / instance: sum them)
    key = next(k for k in ('Dispatch_Id', 'Correlation_Id', 'Kernel_Id') if k in rows[0])
    by = {}
    for r in rows:
        by.setdefault(r[key], 0.0)
        by[r[key]] += float(r['Counter_Value'])
    vals = [by[k] for k in sorted(by, key=int)][-reps:]
    return sum(vals) / len(vals), len(vals)


line = [ln for ln in open(log) if ln.startswith('{"metric"')][-1]
bench = json.loads(line)
entries = [bench['roofline']] + bench.get('rooflines', [])
fetch, write = counter_rows(fdir, 'FETCH_SIZE'), counter_rows(wdir, 'WRITE_SIZE')
def traffic(needle, pick_largest_grid=False):
    f, nf = per_launch(fetch, needle, pick_largest_grid)
    w, nw = per_launch(write, needle, pick_largest_grid)
    return 2 * f * 1024, w * 1024, min(nf, nw)


def dispatches(rows):
    """[(dispatch id, kernel name, value)] in dispatch order (per-instance rows summed)."""
    key = next(k for k in ('Dispatch_Id', 'Correlation_Id', 'Kernel_Id') if k in rows[0])
    by, names = {}, {}
    for r in rows:
        by[r[key]] = by.get(r[key], 0.0) + float(r['Counter_Value'])
        names[r[key]] = r['Kernel_Name']
    return [(int(k), names[k], by[k]) for k in sorted(by, key=int)]


def call_windows(rows, start, members, lead=()):
    """Counter totals of each multi-launch call: a call opens at a `start`
    kernel (with the `lead` kernels right before it, e.g. its zero fills) and
    takes every following `members` kernel until the next call."""
    calls, pending = [], 0.0
    for _, name, v in dispatches(rows):
        if any(m in name for m in lead):
            pending += v
        elif start in name:
            calls.append(pending + v)
            pending = 0.0
        elif any(m in name for m in members) and calls:
            calls[-1] += v
        else:
            pending = 0.0
    return calls


BWD = dict(start='k_build_keys', lead=('k_zero_fill',),
           members=('k_sort_', 'k_head_', 'k_segments', 'k_seg_'))
SS = dict(start='k_ss_compact', members=('k_ss_',))


def window_traffic(family, group, calls):
    """Traffic of entry `group` of a family whose entries made calls[i] calls
    each, in order, at the very end of the run (bench.py's `pmc_calls`): the
    last `reps` calls of the entry are averaged."""
    out = []
    for rows in (fetch, write):
        w = call_windows(rows, **family)
        end = len(w) - sum(calls[group + 1:])
        mine = w[end - calls[group]:end][-reps:]
        out.append(sum(mine) / len(mine))
    return 2 * out[0] * 1024, out[1] * 1024, reps


bwd_entries = [e for e in entries if e['kernel'].startswith('grk_embedding_backward')]
ss_entries = [e for e in entries if e['kernel'].startswith('grk::k_ss_')]
for e in entries:
    k = e['kernel'].split()[0].replace('grk::', '')
    if k == 'grk_embedding_backward':
        fb, wb, n = window_traffic(BWD, bwd_entries.index(e), [x['pmc_calls'] for x in bwd_entries])
        name = f"{tag}_pmc_emb_bwd_{e['workload']['table']}.json"
    elif k.startswith('k_ss_'):
        fb, wb, n = window_traffic(SS, ss_entries.index(e), [x['pmc_calls'] for x in ss_entries])
        name = f"{tag}_pmc_ss_{e['workload']['pass']}.json"
    elif k.startswith('k_attn') and 'pmc_name' in e:
        fb, wb, n = traffic(e['pmc_kernel'])
        name = e['pmc_name']
    elif k.startswith('k_attn'):
        fb, wb, n = traffic(k + '<')
        name = f"{tag}_pmc_attn_{k[len('k_attn_'):-len('_seq')]}_{e['workload']['kind']}.json"
    elif k == 'k_gather' and 'item-table' in e['kernel']:
        # k_gather< or k_gather_wave< (rows of 64 x 16 B): the last launches of the run are the roofline's
        fb, wb, n = traffic('k_gather')
        name = f'{tag}_pmc_gather_item.json'
    elif k == 'k_gather':
        fb, wb, n = traffic('k_gather', True)  # widest launch: the seq-side fused lookup
        name = f'{tag}_pmc_gather.json'
    elif k.startswith('k_wgrad'):
        # one grk_wgrad call = the ring kernel (k_wgrad_lds<, k_wgrad< before round 4) + k_wgrad_reduce;
        # round 5: the entry is the whole family, the PMC is the uvqk shape's (the 8-wave 256 x 128 ring,
        # the largest reduce grid)
        big = 'k_wgrad_lds<true, 4, 2, '   # the 256 x 128 ring (<..., 6> to round 5, <..., 3, 2> since round 6)
        if any(big in r['Kernel_Name'] for r in fetch):
            f1, w1, n1 = traffic(big)
            f2, w2, n2 = traffic('k_wgrad_reduce', True)
        else:
            f1, w1, n1 = traffic('k_wgrad_lds<' if any('k_wgrad_lds<' in r['Kernel_Name'] for r in fetch) else 'k_wgrad<')
            f2, w2, n2 = traffic('k_wgrad_reduce')
        fb, wb, n = f1 + f2, w1 + w2, min(n1, n2)
        name = f'{tag}_pmc_wgrad.json'
        if 'alg_bytes_per_launch' not in e:   # the family entry: the uvqk shape's operands + outputs
            w = e['workload']
            e = dict(e, alg_bytes_per_launch=int(2 * w['K'] * (w['M'] + w['N']) + 4 * w['M'] * (w['N'] + 1)))
    elif k.startswith('k_adamw_catchup'):
        # the rolling flush's slice launches of the roofline replays (the run's last catch-ups;
        # bench.py times the batch-row catch-up before them)
        fb, wb, n = traffic('k_adamw_catchup')
        name = f'{tag}_pmc_catchup.json'
        e = dict(e, alg_bytes_per_launch=e['slice']['alg_bytes_per_launch']) if 'slice' in e else e
    else:
        continue
    out = {'kernel': k, 'workload': e['workload'], 'launches_averaged': n,
           'fetch_bytes_per_launch': fb, 'write_bytes_per_launch': wb,
           'traffic_bytes_per_launch': fb + wb,
           'alg_bytes_per_launch': e['alg_bytes_per_launch'],
           'method': 'rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; FETCH_SIZE x2 '
                     '(gfx950 wide-stream correction, MI355X_MICROARCH.md HBM), KiB -> bytes'}
    with open(os.path.join(REPO, 'profiles', name), 'w') as fh:
        json.dump(out, fh, indent=1)
    print(f"{name}: traffic {out['traffic_bytes_per_launch'] / 1e6:.1f} MB vs algorithmic "
          f"{e['alg_bytes_per_launch'] / 1e6:.1f} MB per launch")
