"""Time grk_gemm (in-process hipBLASLt plans) at the bench's dense-layer shapes.

    GRK_GEMM_LOG=1 python scripts/microbench/grk_gemm.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tencent_recommendation_2025_amd import kernels as K  # noqa: E402

M, d = 128 * 201, 512


def bench(name, fn, flops, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    print(f'{name:50s} {us:8.1f} us  {flops / us / 1e6:7.1f} TF/s', flush=True)


for N, Kd, tag in ((4 * d, d, 'uvqk'), (d, d, 'out_linear'), (d, d + 40, 'itemdnn')):
    x = torch.randn(M, Kd, device='cuda').bfloat16()
    w = torch.randn(N, Kd, device='cuda').bfloat16()
    gy = torch.randn(M, N, device='cuda').bfloat16()
    f = 2.0 * M * N * Kd
    bench(f'{tag} fwd', lambda: K.gemm(x, w, trans_b=True), f)
    bench(f'{tag} dX', lambda: K.gemm(gy, w), f)
    bench(f'{tag} dW fp32', lambda: K.gemm(gy, x, trans_a=True, out_dtype=torch.float32), f)
    bench(f'{tag} dW bf16', lambda: K.gemm(gy, x, trans_a=True), f)
