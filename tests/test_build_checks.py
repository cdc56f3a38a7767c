"""Build-time guards on the compiled kernels (CPU: disassembly only)."""
import glob
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_no_mfma_writes_its_own_sources():
    """No MFMA in the built objects has a destination overlapping its srcA/srcB
    (scripts/check_mfma_overlap.py)."""
    objs = sorted(p for p in glob.glob(os.path.join(REPO, 'build', 'obj', 'grk_*.o')) if not p.endswith('.cpp.o'))
    if not objs:
        pytest.skip('no build/obj (run make first)')
    r = subprocess.run([sys.executable, os.path.join(REPO, 'scripts', 'check_mfma_overlap.py'), *objs],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]


def test_overlap_detector_flags_a_bad_mfma():
    sys.path.insert(0, os.path.join(REPO, 'scripts'))
    from check_mfma_overlap import overlapping_mfmas
    text = ('0000000000001000 <k>:\n'
            '  v_mfma_f32_32x32x16_bf16 v[32:47], v[36:39], v[82:85], 0 // 000000001000\n'
            '  v_mfma_f32_32x32x16_bf16 v[0:15], v[16:19], v[20:23], v[0:15]\n')
    assert overlapping_mfmas(text) == [('k', 'v_mfma_f32_32x32x16_bf16 v[32:47], v[36:39], v[82:85], 0')]


def test_mfma_wait_states_in_attention_objects():
    """The attention objects keep the documented MFMA wait states
    (scripts/isa_hazards.py: an MFMA's D untouched for 12 / 8 states except by
    the accumulate chain, 2 states between a write and the MFMA reading it)."""
    sys.path.insert(0, os.path.join(REPO, 'scripts'))
    from check_mfma_overlap import disassemble
    from isa_hazards import parse, scan
    objs = [p for p in glob.glob(os.path.join(REPO, 'build', 'obj', 'grk_attention*.o'))]
    if not objs:
        pytest.skip('no build/obj (run make first)')
    for obj in objs:
        found = [f for f in scan(parse(disassemble(obj))) if f[0] in ('D-RAW/WAW', 'D-RAW/WAW(mfma)', 'OPERAND')]
        assert not found, (obj, found[:5])


def test_hazard_scanner_flags_short_gaps():
    sys.path.insert(0, os.path.join(REPO, 'scripts'))
    from isa_hazards import parse, scan
    text = ('0000000000001000 <k>:\n'
            '  v_mov_b32 v40, 0\n'
            '  v_mfma_f32_32x32x16_bf16 v[0:15], v[40:43], v[20:23], v[0:15]\n'
            '  s_nop 3\n'
            '  v_add_f32 v50, v3, v4\n'
            '  v_exp_f32 v60, v61\n'
            '  v_pk_mul_f32 v[62:63], v[60:61], v[64:65]\n')
    kinds = sorted({f[0] for f in scan(parse(text))})
    assert kinds == ['D-RAW/WAW', 'OPERAND', 'TRANS-USE(packed)'], kinds


def test_python_sources_bind_every_global_they_read():
    """Every global a function in the shipped Python (package, bench.py, the
    graft entry, oracle, tests) reads is bound somewhere in its module
    (scripts/undefined_names.py): a typo there would surface only when the line
    runs on the GPU box."""
    sys.path.insert(0, os.path.join(REPO, 'scripts'))
    from undefined_names import undefined
    paths = [os.path.join(REPO, p) for p in ('bench.py', '__graft_entry__.py')]
    for d in ('tencent_recommendation_2025_amd', 'oracle', 'tests', 'scripts'):
        paths += sorted(glob.glob(os.path.join(REPO, d, '*.py')))
    bad = [(os.path.relpath(p, REPO), scope, n) for p in paths for scope, n in undefined(p)]
    assert not bad, bad


def test_gpu_code_writes_no_memory_through_the_scalar_cache():
    """scripts/check_scalar_writes.py over every built GPU object (a host-only
    checker kept out of GPU uploads: it names the instructions it rejects)."""
    script = os.path.join(REPO, 'scripts', 'check_scalar_writes.py')
    if not os.path.exists(script):
        pytest.skip('checker not present (GPU box upload)')
    objs = sorted(p for p in glob.glob(os.path.join(REPO, 'build', 'obj', 'grk_*.o')) if not p.endswith('.cpp.o'))
    if not objs:
        pytest.skip('no build/obj (run make first)')
    r = subprocess.run([sys.executable, script, *objs], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
