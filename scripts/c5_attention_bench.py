"""Config C5 attention (BASELINE.json configs[4]: HSTU d=1024, seq_len 1024 + 1,
fp8 MFMA attention): one layer's attention forward + backward at B=16, T=1025,
H=8, hd=128 with bf16 and with fp8 e4m3 q/k/v, timed with HIP events on the
stream the kernels run on.  Prints one JSON line per variant with ms and the
causal algorithmic rate (2 B D T (T+1) FLOP forward, 2.5x that
backward) against the dense bf16 MFMA peak (2.5 PFLOP/s; the non-scaled fp8
MFMA the kernels use runs at the bf16 rate, MI355X_MICROARCH.md)."""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=16)
    ap.add_argument('--seq', type=int, default=1025)
    ap.add_argument('--heads', type=int, default=8)
    ap.add_argument('--hd', type=int, default=128)
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--kind', default='hstu', choices=['hstu', 'softmax'])
    a = ap.parse_args()
    from tencent_recommendation_2025_amd import _lib as L
    from tencent_recommendation_2025_amd import kernels as K
    B, T, H, hd = a.batch, a.seq, a.heads, a.hd
    D = H * hd
    kind = L.ATTN_HSTU if a.kind == 'hstu' else L.ATTN_SOFTMAX
    g = torch.Generator(device='cuda').manual_seed(0)
    x32 = torch.randn(B * T, 3 * D, device='cuda', generator=g)
    lens = torch.randint(T // 2, T + 1, (B,), generator=g, device='cuda')
    kv = (torch.arange(T, device='cuda')[None, :] >= (T - lens)[:, None]).to(torch.uint8).contiguous()
    rab = 0.1 * torch.randn(H, T, device='cuda', generator=g)
    dout = torch.randn(B * T, D, device='cuda', generator=g).bfloat16()
    fwd_flop = 2.0 * B * D * T * (T + 1)
    for name, dt in (('bf16', torch.bfloat16), ('fp8_e4m3', torch.float8_e4m3fn)):
        x = x32.to(dt)
        extra = dict(rab=rab, inv_n=1.0 / T, scale=hd ** -0.5) if kind == L.ATTN_HSTU else {}
        args = K.attn_args(kind, x[:, :D], x[:, D:2 * D], x[:, 2 * D:], B, T, H, hd, key_valid=kv, precise=1,
                           seq_range=K.seq_ranges(kv), **extra)
        out = torch.empty(B * T, D, device='cuda', dtype=torch.bfloat16)
        lse = torch.empty(B, H, T, device='cuda')
        dq, dk, dv = (torch.empty(B * T, D, device='cuda', dtype=torch.bfloat16) for _ in range(3))
        delta = torch.empty(B, H, T, device='cuda')
        drab = torch.zeros(H, T, device='cuda') if kind == L.ATTN_HSTU else None

        def fwd():
            K.attention_fwd(args, out, lse)

        def bwd():
            K.attention_bwd(args, out, dout, lse, delta, dq, dk, dv, drab)

        res = {}
        for part, fn in (('fwd', fwd), ('bwd', bwd)):
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(a.reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[part] = e0.elapsed_time(e1) / a.reps
        flop = fwd_flop * 3.5
        ms = res['fwd'] + res['bwd']
        print(json.dumps({'config': 'C5 attention', 'kind': a.kind, 'qkv': name, 'B': B, 'T': T, 'H': H, 'hd': hd,
                          'fwd_ms': round(res['fwd'], 4), 'bwd_ms': round(res['bwd'], 4), 'ms': round(ms, 4),
                          'tflops': round(flop / ms / 1e9, 1), 'mfma_frac': round(flop / ms / 1e9 / 2500.0, 4),
                          'seq_per_s_layer': round(B / ms * 1e3, 1)}), flush=True)


if __name__ == '__main__':
    main()
