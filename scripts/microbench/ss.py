"""Microbench of the in-batch sampled softmax (grk_sampled_softmax_fwd / _bwd)
at BASELINE config 2: M = 128 x 201 positions, D = 512, ~53 % valid.

    python scripts/microbench/ss.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
from tencent_recommendation_2025_amd import kernels as K  # noqa: E402


def time_call(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    dev = torch.device('cuda', 0)
    g = torch.Generator(device=dev).manual_seed(0)
    M, D = 128 * 201, int(os.environ.get('SS_D', 512))
    h = (torch.randn(M, D, device=dev, generator=g) * 0.05).bfloat16()
    e = (torch.randn(M, D, device=dev, generator=g) * 0.05).bfloat16()
    ids = torch.randint(1, 1_000_000, (M,), device=dev, generator=g)
    valid = (torch.rand(M, device=dev, generator=g) < 0.53).to(torch.uint8)
    nv = int(valid.sum().item())
    loss, lse2, cnt = K.sampled_softmax_fwd(h, e, ids, valid, 0.05)
    tf = time_call(lambda: K.sampled_softmax_fwd(h, e, ids, valid, 0.05))
    tb = time_call(lambda: K.sampled_softmax_bwd(h, e, ids, valid, 0.05, lse2))
    unit = 2.0 * nv * nv * D
    print(f'M {M} D {D} valid {nv}: fwd {tf:.1f} us ({unit / tf / 1e6:.0f} TF/s on nv^2 D), '
          f'bwd {tb:.1f} us ({5 * unit / tb / 1e6:.0f} TF/s: S twice + hi/lo G E + hi/lo G^T H)')


if __name__ == '__main__':
    main()
