#!/usr/bin/env python
"""Instruction mix of every basic block inside loops of one kernel (gfx950 ISA).

    python scripts/isa_loops.py <src.hip> <mangled-kernel-substring> [extra hipcc flags...]
"""
import collections
import re
import subprocess
import sys
import tempfile

src, kern, extra = sys.argv[1], sys.argv[2], sys.argv[3:]
with tempfile.TemporaryDirectory() as d:
    r = subprocess.run(['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '-Iinclude', '-x', 'hip',
                        '--cuda-device-only', '-S', src, '-o', f'{d}/k.s'] + extra, capture_output=True, text=True)
    if r.returncode:
        sys.exit(r.stderr[-3000:])
    s = open(f'{d}/k.s').read()
names = [m.group(1) for m in re.finditer(r"^(\S+):", s, re.M) if kern in m.group(1) and not m.group(1).startswith(".")]
name = names[0]
i = s.index(name + ':')
j = s.index('.Lfunc_end', i)
blocks, cur = [], None
for ln in s[i:j].splitlines():
    t = ln.strip()
    if t.startswith('.LBB') or t.startswith('; %bb'):
        cur = [' '.join(t.split()), []]
        blocks.append(cur)
        continue
    if not t or t.startswith(';') or t.startswith('.'):
        continue
    if cur is None:
        cur = ['entry', []]
        blocks.append(cur)
    cur[1].append(t.split()[0])
tot = collections.Counter()
print(name)
depth = lambda nm: int(re.search(r'Depth=(\d+)', nm).group(1)) if 'Depth=' in nm else 0
maxd = max(depth(nm) for nm, _ in blocks)
for nm, ins in blocks:
    if depth(nm) < maxd:
        continue
    c = collections.Counter(ins)
    tot.update(c)
    grp = lambda f: sum(v for k, v in c.items() if f(k))
    print(f"{nm.split()[0 if nm[0] == '.' else 1][:12]:12s} n={len(ins):4d} mfma={grp(lambda k: 'mfma' in k):2d} valu={grp(lambda k: k.startswith('v_') and 'mfma' not in k and 'accvgpr' not in k):4d} "
          f"accmov={grp(lambda k: 'accvgpr' in k):3d} ds={grp(lambda k: k.startswith('ds_')):3d} salu={grp(lambda k: k.startswith('s_') and k != 's_waitcnt' and k != 's_nop'):3d} "
          f"wait={c['s_waitcnt']:2d} nop={c['s_nop']:2d} trans={grp(lambda k: k.startswith(('v_exp', 'v_rcp'))):3d} branch={grp(lambda k: 'cbranch' in k):2d}")
grp = lambda f: sum(v for k, v in tot.items() if f(k))
print(f"innermost total: n={sum(tot.values())} mfma={grp(lambda k: 'mfma' in k)} accmov={grp(lambda k: 'accvgpr' in k)} "
      f"ds={grp(lambda k: k.startswith('ds_'))} wait={tot['s_waitcnt']} trans={grp(lambda k: k.startswith(('v_exp', 'v_rcp')))}")
