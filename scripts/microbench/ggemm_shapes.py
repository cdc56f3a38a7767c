"""grk_grouped_gemm (one group) against grk_gemm (hipBLASLt, tuned plans) on the
dense-layer shapes of the C2 step, device time per call (HIP events):

  uvqk forward      C [M, 2048] = X [M, 512] . W^T      (layout 0)
  out_linear fwd    C [M, 512]  = Y [M, 512] . W^T      (layout 0)
  uvqk dgrad        C [M, 512]  = dY [M, 2048] . W      (layout 1)
  projection fwd    C [10001, 512] = E . W_f^T           (layout 0)

    python scripts/microbench/ggemm_shapes.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

M = 14336


def timed(fn, reps=50):
    """Device time per call: `reps` calls captured in one HIP graph (host launch cost
    out of the measurement), replayed between events."""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=side):
        for _ in range(reps):
            fn()
    graph.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    graph.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    from tencent_recommendation_2025_amd import kernels as K
    dev = torch.device('cuda')
    g = torch.Generator(device=dev).manual_seed(0)
    shapes = [('uvqk fwd', M, 2048, 512, 0), ('out_linear fwd', M, 512, 512, 0), ('uvqk dgrad', M, 512, 2048, 1),
              ('projection fwd', 10001, 512, 512, 0)]
    for name, m, n, k, lay in shapes:
        A = torch.randn(m, k, generator=g, device=dev).bfloat16()
        W = (0.05 * torch.randn(n, k, generator=g, device=dev)).bfloat16() if lay == 0 else \
            (0.05 * torch.randn(k, n, generator=g, device=dev)).bfloat16()
        C = torch.empty(m, n, dtype=torch.bfloat16, device=dev)
        ref = A.float() @ (W.float().t() if lay == 0 else W.float())
        K.grouped_gemm([(A, W, C)], n=n, k=k, b_layout=lay)
        torch.cuda.synchronize()
        err = float((C.float() - ref).norm() / ref.norm())
        t_g = timed(lambda: K.grouped_gemm([(A, W, C)], n=n, k=k, b_layout=lay))
        t_h = timed(lambda: K.gemm(A, W, trans_b=(lay == 0)))
        fl = 2 * m * n * k
        print(f'{name:15s} M={m} N={n} K={k}: grouped {t_g:6.1f} us ({fl / t_g / 1e6:5.0f} TF/s, err {err:.1e}) | '
              f'grk_gemm {t_h:6.1f} us ({fl / t_h / 1e6:5.0f} TF/s)', flush=True)


if __name__ == '__main__':
    main()
