"""HSTU forward at the C2 test shape, repeated: error vs oracle and run-to-run equality (diagnostic)."""
import sys, os
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..', 'tests'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
import test_gpu_attention as t
from tencent_recommendation_2025_amd import kernels as K, _lib
_lib.lib()
print('lib', _lib.LIB_PATH)
for act in (None, 'silu'):
    outs = []
    for rep in range(4):
        res, want, valid = t.run(K, 1, B=128, T=201, H=8, hd=64, lens=t.C2_LENS, precise=True, seed=11,
                                 out_dtype=torch.float32, act=act, oracle=(rep == 0))
        if rep == 0:
            w = want
        outs.append(res)
        print(act, rep, {k: f'{t.nrel(res[k], w[k]):.2e}' for k in ('out', 'dq', 'dk', 'dv', 'drab')})
    for k in ('out', 'dq', 'dk', 'dv'):
        print(act, k, 'repeatable', all(np.array_equal(outs[0][k], o[k]) for o in outs[1:]))
