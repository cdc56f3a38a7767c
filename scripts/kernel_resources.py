#!/usr/bin/env python
"""Per-kernel register / LDS / occupancy table for one HIP source (gfx950).

    python scripts/kernel_resources.py tencent_recommendation_2025_amd/csrc/grk_attention.hip [name-filter] [hipcc flags...]
"""
import re
import subprocess
import sys
import tempfile

src = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ''
extra = sys.argv[3:]
with tempfile.TemporaryDirectory() as d:
    r = subprocess.run(['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '-Iinclude', '-x', 'hip',
                        '-c', src, '-o', f'{d}/k.o', '-Rpass-analysis=kernel-resource-usage'] + extra,
                       capture_output=True, text=True)
rows, cur = [], None
for line in r.stderr.splitlines():
    m = re.search(r'remark: +(.*?): (.*?) \[-Rpass', line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == 'Function Name':
        cur = {'name': v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
print(f"{'kernel':70s} {'VGPR':>5s} {'AGPR':>5s} {'spill':>5s} {'occ':>4s} {'LDS':>6s}")
for c in rows:
    n = subprocess.run(['c++filt'], input=c['name'], capture_output=True, text=True).stdout.strip()
    if filt and filt not in n:
        continue
    print(f"{n[:70]:70s} {c.get('VGPRs', '?'):>5s} {c.get('AGPRs', '?'):>5s} {c.get('VGPRs Spill', '?'):>5s} "
          f"{c.get('Occupancy [waves/SIMD]', '?'):>4s} {c.get('LDS Size [bytes/block]', '?'):>6s}")
if r.returncode:
    print(r.stderr[-2000:])
