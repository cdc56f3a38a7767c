"""Which rounding points explain the grk HSTU core's distance from the fp32 oracle?

The fp32 HSTU model test (tests/test_gpu_model.py) measured logits 1.6e-3 from
the fp32 oracle and 1.3e-3 from the oracle with the core's bf16 storage points
(RefHSTU.bf16_core) -- before the gate's bf16 SiLU(u) (k_ng_fwd) was added to
them; round 4 run (gpurun_out/r4h_hstu_rounding.txt) found the remaining 2.4e-3.  Here one layer core (functional.hstu_core: y from a bf16-
exact pre-activation) against a float64 restatement with each candidate rounding
switched on or off, normwise errors printed per variant.

    python scripts/diag/hstu_rounding.py
"""
import itertools
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def rb(x):
    return x.to(torch.bfloat16).to(x.dtype)


def core(pre, rab, ln_w, ln_b, B, T, H, hd, round_qkv, round_p, round_o, round_y, scale_q):
    D = H * hd
    x = pre.double().view(B, T, 4 * D)
    u, v, q, k = torch.split(F.silu(x), D, dim=-1)
    if round_qkv:
        u, v, q, k = rb(u), rb(v), rb(q), rb(k)
    sh = lambda t: t.reshape(B, T, H, hd).transpose(1, 2)
    q, k, v = sh(q), sh(k), sh(v)
    if scale_q:
        q = rb(q * hd ** -0.5) if round_qkv else q * hd ** -0.5
        s = q @ k.transpose(-1, -2)
    else:
        s = (q @ k.transpose(-1, -2)) * hd ** -0.5
    i = torch.arange(T)[:, None]
    j = torch.arange(T)[None, :]
    s = s + rab.double()[:, (i - j).clamp(0, rab.shape[1] - 1)][None]
    a = F.silu(s) / T * (j <= i).double()
    if round_p:
        a = rb(a)
    o = (a @ v).transpose(1, 2).reshape(B, T, D)
    if round_o:
        o = rb(o)
    y = F.layer_norm(o, (D,), ln_w.double(), ln_b.double(), eps=1e-8) * u
    if round_y:
        y = rb(y)
    return y.reshape(B * T, D)


def main():
    from tencent_recommendation_2025_amd import functional as G
    torch.manual_seed(0)
    for (B, T, H, hd) in ((8, 21, 2, 16), (16, 201, 8, 64)):
        D = H * hd
        pre = rb(torch.randn(B * T, 4 * D)).float()
        rab = 0.3 * torch.randn(H, T)
        ln_w = 1 + 0.1 * torch.randn(D)
        ln_b = 0.02 * torch.randn(D)
        kv = torch.ones(B, T, dtype=torch.uint8)
        y = G.hstu_core(pre.cuda(), rab.cuda(), ln_w.cuda(), ln_b.cuda(), kv.cuda(), B, T, H, hd, 1.0 / T).double().cpu()
        print(f'B={B} T={T} H={H} hd={hd}', flush=True)
        for flags in itertools.product((0, 1), repeat=5):
            ref = core(pre, rab, ln_w, ln_b, B, T, H, hd, *flags)
            e = float((y - ref).norm() / ref.norm())
            print(f'  round qkv={flags[0]} p={flags[1]} o={flags[2]} y={flags[3]} scale_q={flags[4]}: {e:.3e}', flush=True)


if __name__ == '__main__':
    main()
