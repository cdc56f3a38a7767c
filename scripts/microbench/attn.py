"""Time the grk attention kernels alone at the bench's HSTU shape.

    python scripts/microbench/attn.py [--kind hstu|softmax] [--B 128 --T 201 --H 8 --hd 64] [--reps 20]

Reports per-call forward / backward time (HIP events on the launch stream),
and TFLOP/s by the SURVEY §8(d) formula (fwd 2*B*D*T*(T+1) per layer,
causal half counted once for QK^T and once for PV) and by the pairs that
are actually valid (left-padded lengths, causal).
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tencent_recommendation_2025_amd import _lib as L  # noqa: E402
from tencent_recommendation_2025_amd import kernels as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--kind', default='hstu')
    ap.add_argument('--B', type=int, default=128)
    ap.add_argument('--T', type=int, default=201)
    ap.add_argument('--H', type=int, default=8)
    ap.add_argument('--hd', type=int, default=64)
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--full', action='store_true', help='every sequence full length (no padding)')
    ap.add_argument('--precise', action='store_true')
    ap.add_argument('--act', default='silu', help="'silu' (HSTU pre-activations) or 'none'")
    ap.add_argument('--no-ranges', action='store_true', help='do not pass precomputed seq_range')
    ap.add_argument('--no-drab', action='store_true', help='HSTU: skip the rab gradient')
    a = ap.parse_args()
    B, T, H, hd = a.B, a.T, a.H, a.hd
    D = H * hd
    dev = 'cuda'
    g = torch.Generator(device=dev).manual_seed(0)
    pre = torch.randn(B * T, 4 * D, device=dev, generator=g).bfloat16()
    lens = torch.full((B,), T, device=dev) if a.full else torch.randint(32, T + 1, (B,), device=dev, generator=g)
    kv = (torch.arange(T, device=dev)[None, :] >= (T - lens)[:, None]).to(torch.uint8).contiguous()
    kind = L.ATTN_HSTU if a.kind == 'hstu' else L.ATTN_SOFTMAX
    extra = dict(rab=(0.1 * torch.randn(H, T, device=dev, generator=g)).contiguous(), inv_n=1.0 / T,
                 act=None if a.act == 'none' else 'silu') if kind == L.ATTN_HSTU else {}
    args = K.attn_args(kind, pre[:, 2 * D:3 * D], pre[:, 3 * D:], pre[:, D:2 * D], B, T, H, hd, key_valid=kv,
                       precise=a.precise, out_dtype=torch.bfloat16,
                       seq_range=None if a.no_ranges else K.seq_ranges(kv), **extra)
    o = torch.empty(B * T, D, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(B, H, T, device=dev)
    do = torch.randn(B * T, D, device=dev, generator=g).bfloat16()
    dpre = torch.empty(B * T, 4 * D, dtype=torch.bfloat16, device=dev)
    delta = torch.empty(B, H, T, device=dev)
    drab = torch.zeros(H, T, device=dev) if kind == L.ATTN_HSTU and not a.no_drab else None

    def fwd():
        K.attention_fwd(args, o, lse)

    def bwd():
        K.attention_bwd(args, o, do, lse, delta, dpre[:, 2 * D:3 * D], dpre[:, 3 * D:], dpre[:, D:2 * D], drab)

    def timeit(fn):
        for _ in range(3):
            fn()
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(a.reps):
            fn()
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.reps * 1e3  # us

    tf = timeit(fwd)
    tb = timeit(bwd)
    formula = 2.0 * B * D * T * (T + 1)
    L_ = lens.double()
    valid_pairs = float((L_ * (L_ + 1) / 2).sum()) * H
    actual = 4.0 * hd * valid_pairs
    print(f'{a.kind} act={a.act} B={B} T={T} H={H} hd={hd} {"full" if a.full else "ragged"} precise={a.precise}: '
          f'fwd {tf:8.1f} us  bwd {tb:8.1f} us | fwd {formula / tf / 1e6:6.1f} TF/s (formula) '
          f'{actual / tf / 1e6:6.1f} TF/s (valid pairs) | bwd {2.5 * formula / tb / 1e6:6.1f} TF/s (formula x2.5)')


if __name__ == '__main__':
    main()
