"""Weight-gradient GEMM at the bench's shapes: grk_wgrad (split-K MFMA) vs grk_gemm (hipBLASLt, trans_a).

    python scripts/microbench/wgrad.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tencent_recommendation_2025_amd import kernels as K  # noqa: E402


def bench(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for k, m, n in [(25728, 2048, 512), (25728, 512, 512), (51456, 512, 560), (25728, 512, 520), (25728, 1024, 512)]:
    dy = torch.randn(k, m, device='cuda').bfloat16()
    x = torch.randn(k, n, device='cuda').bfloat16()
    flop = 2.0 * k * m * n
    t1 = bench(lambda: K.wgrad(dy, x, want_db=True))
    t0 = bench(lambda: (K.gemm(dy, x, trans_a=True, out_dtype=torch.float32), dy.sum(0, dtype=torch.float32)))
    print(f'K={k} M={m} N={n}: grk_wgrad+db {t1 * 1e3:7.1f} us ({flop / t1 / 1e9:6.0f} TF/s)   '
          f'hipBLASLt+sum {t0 * 1e3:7.1f} us ({flop / t0 / 1e9:6.0f} TF/s)', flush=True)
