"""Per-row error of the HSTU forward at the C2 test shape (diagnostic)."""
import sys, os
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..', 'tests'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
import test_gpu_attention as t
from tencent_recommendation_2025_amd import kernels as K, _lib
_lib.lib()
for act in ('silu', None):
    res, want, valid = t.run(K, 1, B=128, T=201, H=8, hd=64, lens=t.C2_LENS, precise=True, seed=11,
                             out_dtype=torch.float32, act=act)
    for key in ('out', 'dq', 'dk', 'dv', 'drab'):
        print(act, key, t.nrel(res[key], want[key]))
    o, w = res['out'], np.asarray(want['out'])
    err = np.linalg.norm(o - w, axis=1) / (np.linalg.norm(w, axis=1) + 1e-30)
    bad = np.argsort(-err)[:10]
    B, T = 128, 201
    for r in bad:
        b, q = divmod(int(r), T)
        print(f'row b={b} q={q} len={t.C2_LENS[b]} start={T - t.C2_LENS[b]} err={err[r]:.3e} |w|={np.linalg.norm(w[r]):.3e}')
