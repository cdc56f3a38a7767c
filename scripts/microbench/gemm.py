"""Time the bench step's GEMM shapes in isolation (torch -> hipBLASLt / rocBLAS), bf16.

    python scripts/microbench/gemm.py

M = B*T tokens (128 x 201), d = 512: HSTU uvqk [d -> 4d] and out_linear
[d -> d] forward / dX / dW, itemdnn-style K = d + 40.  dW alternatives:
transposed product, and split-K (S partial products as one bmm + a
fixed-order fp32 sum: deterministic).
"""
import torch

M, d = 128 * 201, 512
dev = 'cuda'


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
    print(f'{name:62s} {us:8.1f} us  {flops / us / 1e6:7.1f} TF/s', flush=True)


def splitk(gy, x, S):
    Mp = gy.shape[0] // S * S
    a = gy[:Mp].view(S, -1, gy.shape[1]).transpose(1, 2)      # [S, N, M/S]
    b = x[:Mp].view(S, -1, x.shape[1])                         # [S, M/S, K]
    part = torch.bmm(a, b, out_dtype=torch.float32) if False else torch.bmm(a, b).float()
    out = part.sum(0)
    if Mp < gy.shape[0]:
        out += gy[Mp:].t().float() @ x[Mp:].float()
    return out


for backend in ('hipblaslt', 'rocblas'):
    try:
        torch.backends.cuda.preferred_blas_library('cublaslt' if backend == 'hipblaslt' else 'cublas')
    except Exception as e:  # noqa: BLE001
        print('backend switch failed:', e)
        continue
    print(f'--- {backend}: {torch.backends.cuda.preferred_blas_library()}')
    for N, K, tag in ((4 * d, d, 'uvqk d->4d'), (d, d, 'out_linear d->d'), (d, d + 40, 'itemdnn (d+40)->d')):
        x = torch.randn(M, K, device=dev).bfloat16()
        w = torch.randn(N, K, device=dev).bfloat16()
        gy = torch.randn(M, N, device=dev).bfloat16()
        f = 2.0 * M * N * K
        bench(f'{tag}: fwd x @ w.t()', lambda: x @ w.t(), f)
        bench(f'{tag}: dX = gy @ w', lambda: gy @ w, f)
        bench(f'{tag}: dW = gy.t() @ x', lambda: gy.t() @ x, f)
        bench(f'{tag}: dW = (x.t() @ gy).t()', lambda: (x.t() @ gy).t(), f)
        for S in (4, 8, 16):
            bench(f'{tag}: dW split-K S={S} (bmm + fp32 sum)', lambda: splitk(gy, x, S), f)
