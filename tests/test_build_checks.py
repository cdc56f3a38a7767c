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
