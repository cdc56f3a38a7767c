"""Per-kernel durations of each grk_embedding_backward call in a rocprofv3
kernel trace of emb_bwd.py (calls delimited by k_build_keys launches)."""
import csv
import re
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
calls, cur = [], None
for r in rows:
    name = r['Kernel_Name']
    if 'k_build_keys' in name:
        cur = defaultdict(float)
        cur['_start'] = int(r['Start_Timestamp'])
        calls.append(cur)
    if cur is None:
        continue
    m = re.search(r'grk::(?:\(anonymous namespace\)::)?(\w+)', name)
    key = m.group(1) if m else ('rocprim' if 'rocprim' in name else name[:30])
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    cur[key] += d
    cur['_end'] = int(r['End_Timestamp'])
for i, c in enumerate(calls):
    span = (c.pop('_end') - c.pop('_start')) / 1e3
    print(f'call {i:2d} span {span:7.1f} us: ' + ', '.join(f'{k} {v:.1f}' for k, v in sorted(c.items(), key=lambda x: -x[1])))
