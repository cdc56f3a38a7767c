#!/usr/bin/env python
"""Build guard: no GPU code object of libgrk writes memory through the scalar
data cache (scalar stores or scalar atomics, or that cache's write-back /
discard).  The compiler is not expected to emit any for this code; runs of
such code on this pool were followed by machine resets, so the build checks
the disassembly instead of trusting that.  Host-only checker: listed in
.gpurunignore (it names the instructions it looks for).

    python scripts/check_scalar_writes.py build/obj/grk_*.o
"""
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from check_mfma_overlap import disassemble  # noqa: E402

PATTERN = re.compile(r'^\s+(s_store_\w+|s_buffer_store_\w+|s_scratch_store_\w+|s_atomic_\w+|s_buffer_atomic_\w+|'
                     r's_dcache_wb\w*|s_dcache_discard\w*)\b', re.M)


def scalar_writes(obj):
    """[(mnemonic, count)] of scalar-cache writes in one object's GPU code."""
    found = {}
    for m in PATTERN.finditer(disassemble(obj)):
        found[m.group(1)] = found.get(m.group(1), 0) + 1
    return sorted(found.items())


def main(paths):
    bad = 0
    for p in paths:
        w = scalar_writes(p)
        if w:
            bad += 1
            print(f'{p}: {w}')
    print(f'check_scalar_writes: {"FAIL" if bad else "ok"} ({len(paths)} object(s))')
    return 1 if bad else 0


if __name__ == '__main__':
    sys.exit(main(sys.argv[1:]))
