"""Attention precision + timing at the full C2 shape (B=128, T=201, H=8, hd=64,
ragged left-padded lengths U{32..201}): normwise error vs the fp64 oracle
(same bf16-rounded inputs) for fast (PREC=0) and precise (PREC=1) kernels,
fp32 and bf16 outputs, and the per-kernel launch time of each mode."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'tests'))
from oracle.embedding import to_bf16_f32  # noqa: E402
from test_gpu_attention import nrel, run  # noqa: E402

from tencent_recommendation_2025_amd import _lib as L  # noqa: E402
from tencent_recommendation_2025_amd import kernels as K  # noqa: E402

L.lib()
B, T, H, hd = 128, 201, 8, 64
lens = np.random.default_rng(3).integers(32, 202, B).tolist()
for kind in (1, 0):
    for precise in (False, True):
        for odt in (torch.float32, torch.bfloat16):
            act = 'silu' if kind == 1 else None
            res, want, _ = run(K, kind, B, T, H, hd, lens, precise, seed=11, out_dtype=odt, act=act)
            errs = {}
            for key in ('out', 'dq', 'dk', 'dv') + (('drab',) if kind == 1 else ()):
                w = want[key] if odt == torch.float32 or key == 'drab' else to_bf16_f32(want[key].astype(np.float32))
                errs[key] = nrel(res[key], w)
            print(f"kind={'hstu' if kind else 'softmax'} precise={int(precise)} out={str(odt)[6:]}: " +
                  ' '.join(f'{k}={v:.2e}' for k, v in errs.items()), flush=True)

# timing, bench layout (u|v|q|k pre-activations, SiLU on load, bf16 out)
dev = 'cuda'
D = H * hd
kv = torch.zeros(B, T, dtype=torch.uint8, device=dev)
for b, n in enumerate(lens):
    kv[b, T - n:] = 1
pre = torch.randn(B * T, 4 * D, device=dev).bfloat16()
do = torch.randn(B * T, D, device=dev).bfloat16()
dpre = torch.empty(B * T, 4 * D, dtype=torch.bfloat16, device=dev)
o = torch.empty(B * T, D, dtype=torch.bfloat16, device=dev)
lse = torch.empty(B, H, T, device=dev)
delta = torch.empty(B, H, T, device=dev)


def tm(fn, reps=50):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for kind in (1, 0):
    for precise in (False, True):
        hstu = kind == 1
        extra = dict(rab=0.1 * torch.randn(H, T, device=dev), inv_n=1.0 / T, act='silu') if hstu else {}
        drab = torch.zeros(H, T, device=dev) if hstu else None
        args = K.attn_args(kind, pre[:, 2 * D:3 * D], pre[:, 3 * D:], pre[:, D:2 * D], B, T, H, hd, key_valid=kv,
                           scale=hd ** -0.5, out_dtype=torch.bfloat16, seq_range=K.seq_ranges(kv), precise=precise,
                           **extra)
        K.attention_fwd(args, o, lse)
        K.attention_bwd(args, o, do, lse, delta, dpre[:, 2 * D:3 * D], dpre[:, 3 * D:], dpre[:, D:2 * D], drab)
        tf = tm(lambda: K.attention_fwd(args, o, lse))
        tq = tm(lambda: K.attention_bwd(args, o, do, lse, delta, dpre[:, 2 * D:3 * D], None, None, drab,
                                        parts=L.ATTN_BWD_DQ))
        tk = tm(lambda: K.attention_bwd(args, o, do, lse, delta, None, dpre[:, 3 * D:], dpre[:, D:2 * D], None,
                                        parts=L.ATTN_BWD_DKDV))
        print(f"time kind={'hstu' if hstu else 'softmax'} precise={int(precise)}: fwd {tf:.1f} us, dq {tq:.1f} us, "
              f"dkdv {tk:.1f} us", flush=True)
