#!/usr/bin/env python
"""Scan gfx950 code for MFMA register hazards with too few wait states between
the two instructions (straight-line order inside each function; a wait state
= one issued instruction, `s_nop N` = N + 1).  Rules (cdna_hip_programming.md
§5.7 item 2, for the 8-pass `v_mfma_f32_32x32x16_bf16` / 4-pass `16x16x32`):

  D-RAW/WAW   an MFMA's vdst read or written by anything but the next MFMA
              taking the whole range as srcC: 12 states after an 8-pass MFMA
              (8 after a 4-pass one);
  OPERAND     a VALU / VMEM / DS write of a register an MFMA then reads as
              srcA / srcB / srcC: 2 states before the MFMA;
  TRANS-USE   (reported) a transcendental's result (v_exp / v_rcp / v_log /
              v_sqrt / v_rsq / v_sin / v_cos) read by the next VALU
              instruction with no state between (packed v_pk_* listed apart);
  SRC-WAR     (reported, not a documented rule) a write to a register an
              MFMA issued fewer than 12 states earlier reads as srcC (srcA /
              srcB are read at issue: hipcc reuses them the next cycle).

The compiler's hazard recognizer is meant to pad all of these; this checks
what it emitted.

    python scripts/isa_hazards.py build/obj/grk_attention_seq.o [kernel-substring]
    python scripts/isa_hazards.py --source tencent_recommendation_2025_amd/csrc/grk_attention_seq.hip [hipcc flags]
"""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from check_mfma_overlap import disassemble  # noqa: E402


def regs(op):
    op = op.strip()
    m = re.match(r'([vas])\[(\d+):(\d+)\]', op)
    if m:
        return {(m.group(1), r) for r in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.match(r'([vas])(\d+)$', op)
    return {(m.group(1), int(m.group(2)))} if m else set()


def parse(text):
    """{function: [(mnemonic, [operands])]} in address order."""
    out, fn = {}, None
    for line in text.splitlines():
        m = re.match(r'^[0-9a-f]+ <(\S+)>:', line)
        if m:
            fn = m.group(1)
            out[fn] = []
            continue
        if fn is None:
            continue
        s = line.split('//')[0].strip()
        if not s or s.endswith(':'):
            continue
        parts = s.split(None, 1)
        ops = [o.strip() for o in parts[1].split(',')] if len(parts) > 1 else []
        out[fn].append((parts[0], ops))
    return out


def passes(mn):
    if '32x32' in mn:
        return 8
    if '16x16' in mn:
        return 4
    return 4


def dst_src(mn, ops):
    """(written registers, read registers) of one instruction (VGPR/AGPR only)."""
    rd = set()
    if not ops:
        return set(), set()
    if mn.startswith(('global_store', 'buffer_store', 'flat_store', 'scratch_store')):
        for o in ops:
            rd |= {r for r in regs(o) if r[0] in 'va'}
        return set(), rd
    if mn.startswith('ds_write') or mn.startswith('ds_store'):
        for o in ops:
            rd |= {r for r in regs(o) if r[0] in 'va'}
        return set(), rd
    if mn.startswith(('s_', 'v_cmp')) and not mn.startswith('v_cmp'):
        return set(), set()
    wr = {r for r in regs(ops[0]) if r[0] in 'va'}
    for o in ops[1:]:
        rd |= {r for r in regs(o) if r[0] in 'va'}
    return wr, rd


def states(mn, ops):
    if mn == 's_nop':
        try:
            return int(ops[0], 0) + 1
        except (ValueError, IndexError):
            return 1
    return 1


def scan(fns, filt=''):
    found = []
    for fn, ins in fns.items():
        if filt and filt not in fn:
            continue
        trans = []     # [(state, regs, text)] recent transcendental writes
        inflight = []  # [(issue state, passes, dst regs, src regs, text)]
        writes = []    # [(state, regs, text)] recent non-MFMA writes
        t = 0
        for mn, ops in ins:
            is_mfma = mn.startswith('v_mfma')
            wr, rd = dst_src(mn, ops)
            if is_mfma:
                d = regs(ops[0])
                a, b, c = (regs(ops[k]) if len(ops) > k else set() for k in (1, 2, 3))
                # OPERAND: a recent write feeding this MFMA
                for ws, wregs, wtxt in writes:
                    if t - ws < 2 and wregs & (a | b | c):
                        found.append(('OPERAND', fn, t - ws, wtxt, f'{mn} {",".join(ops)}'))
                # D-RAW/WAW from an earlier MFMA (the accumulate chain is exempt)
                for s0, p, dd, ss, txt in inflight:
                    need = 12 if p == 8 else 8
                    if t - s0 < need and dd & (a | b | d) and not (dd == c and dd == d):
                        found.append(('D-RAW/WAW(mfma)', fn, t - s0, txt, f'{mn} {",".join(ops)}'))
                inflight.append((t, passes(mn), d, c, f'{mn} {",".join(ops)}'))
            else:
                if mn.startswith('v_'):
                    for ts, tregs, ttxt in trans:
                        if t - ts < 2 and tregs & rd:
                            kind = 'TRANS-USE(packed)' if mn.startswith('v_pk_') else 'TRANS-USE'
                            found.append((kind, fn, t - ts, ttxt, f'{mn} {",".join(ops)}'))
                    if re.match(r'v_(exp|rcp|log|sqrt|rsq|sin|cos)_f(32|16)', mn):
                        trans.append((t, wr, f'{mn} {",".join(ops)}'))
                touched = wr | rd
                for s0, p, dd, ss, txt in inflight:
                    need = 12 if p == 8 else 8
                    if t - s0 < need and dd & touched:
                        found.append(('D-RAW/WAW', fn, t - s0, txt, f'{mn} {",".join(ops)}'))
                    if t - s0 < 12 and wr & ss:
                        found.append(('SRC-WAR', fn, t - s0, txt, f'{mn} {",".join(ops)}'))
                if wr:
                    writes.append((t, wr, f'{mn} {",".join(ops)}'))
            t += states(mn, ops)
            inflight = [x for x in inflight if t - x[0] < 16]
            writes = [x for x in writes if t - x[0] < 4]
            trans = [x for x in trans if t - x[0] < 4]
            if mn.startswith('s_cbranch') or mn in ('s_branch', 's_setpc_b64', 's_endpgm'):
                # straight-line only: a branch target's history is unknown here
                inflight, writes, trans = [], [], []
    return found


def main(argv):
    if argv and argv[0] == '--source':
        src, flags = argv[1], argv[2:]
        with tempfile.TemporaryDirectory() as d:
            obj = os.path.join(d, 'k.o')
            subprocess.run(['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '-Iinclude', '-c',
                            src, '-o', obj] + flags, check=True)
            text = disassemble(obj)
        filt = ''
    else:
        text = disassemble(argv[0])
        filt = argv[1] if len(argv) > 1 else ''
    fns = parse(text)
    found = scan(fns, filt)
    kinds = {}
    for k, fn, dist, a, b in found:
        kinds.setdefault(k, []).append((fn, dist, a, b))
    n_mfma = sum(1 for f in fns.values() for mn, _ in f if mn.startswith('v_mfma'))
    print(f'{n_mfma} MFMAs in {len(fns)} functions')
    for k, v in sorted(kinds.items()):
        print(f'{k}: {len(v)}')
        for fn, dist, a, b in v[:6]:
            print(f'    {dist} states  {a}  ->  {b}   [{fn[:60]}]')
    return 0


if __name__ == '__main__':
    sys.exit(main(sys.argv[1:]))
