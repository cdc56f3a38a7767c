#!/usr/bin/env python
"""Reject a code object with an MFMA whose destination overlaps its srcA/srcB.

A multi-pass MFMA must not write registers it still reads as A/B operands.
The VGPR-form build of the whole-sequence attention kernels once produced such
instructions (a literal-zero srcC leaves vdst untied, and the allocator reused
a dying source's registers): the HSTU forward then gave timing-dependent wrong
rows.  `make` runs this on every
object before linking libgrk.so.

    python scripts/check_mfma_overlap.py build/obj/grk_*.o   (the .hip objects)
"""
import re
import subprocess
import sys

OBJDUMP = '/opt/rocm/lib/llvm/bin/llvm-objdump'
BUNDLER = '/opt/rocm/lib/llvm/bin/clang-offload-bundler'


def _regs(op):
    m = re.match(r'([va])\[(\d+):(\d+)\]', op)
    if m:
        return {(m.group(1), r) for r in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.match(r'([va])(\d+)$', op)
    return {(m.group(1), int(m.group(2)))} if m else set()


def overlapping_mfmas(disasm_text):
    """[(kernel, instruction)] of MFMAs with vdst & (srcA | srcB) != {}."""
    bad, fn = [], None
    for line in disasm_text.splitlines():
        m = re.match(r'^[0-9a-f]+ <(\S+)>:', line)
        if m:
            fn = m.group(1)
            continue
        s = line.split('//')[0].strip()
        if not s.startswith('v_mfma'):
            continue
        parts = s.split(None, 1)
        if len(parts) < 2:
            continue
        ops = [o.strip() for o in parts[1].split(',')]
        if len(ops) >= 3 and _regs(ops[0]) & (_regs(ops[1]) | _regs(ops[2])):
            bad.append((fn, s))
    return bad


def disassemble(obj):
    """Disassembly of the gfx950 code object in one hipcc object file (its
    .hip_fatbin section, unbundled)."""
    import os
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, 'fb.bin'), os.path.join(d, 'dev.co')
        subprocess.run(['objcopy', '--dump-section', f'.hip_fatbin={fb}', obj, os.path.join(d, 'x.o')],
                       check=True, capture_output=True)
        subprocess.run([BUNDLER, '--type=o', '--unbundle', f'--input={fb}', f'--output={co}',
                        '--targets=hipv4-amdgcn-amd-amdhsa--gfx950'], check=True, capture_output=True)
        return subprocess.run([OBJDUMP, '-d', '--mcpu=gfx950', co], check=True, capture_output=True,
                              text=True).stdout


def main(objs):
    total, bad = 0, []
    for obj in objs:
        text = disassemble(obj)
        total += text.count('v_mfma')
        bad += [(obj, fn, ins) for fn, ins in overlapping_mfmas(text)]
    if total == 0:
        print('check_mfma_overlap: no gfx950 MFMA code found', file=sys.stderr)
        return 1
    for obj, fn, ins in bad[:20]:
        print(f'check_mfma_overlap: {obj}: {fn}: {ins}', file=sys.stderr)
    if bad:
        print(f'check_mfma_overlap: {len(bad)} MFMA(s) with vdst overlapping srcA/srcB', file=sys.stderr)
        return 1
    print(f'check_mfma_overlap: ok ({total} MFMAs in {len(objs)} object(s))')
    return 0


if __name__ == '__main__':
    sys.exit(main(sys.argv[1:]))
