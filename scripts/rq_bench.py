"""grk_rq_assign alone at config 4's tokenisation size (1M rows, latent 64, 3 x 256
codes; plus latent 32 / 128), HIP events on its stream.  One JSON line per shape:
avg launch ms and TFLOP/s (3 * levels * codes * latent FLOP per row)."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    from tencent_recommendation_2025_amd.rqvae import rq_assign
    shapes = ((64, 3, 256), (32, 3, 256), (128, 3, 256), (64, 4, 1024))
    if '--first' in sys.argv:   # config 4's shape only (PMC passes)
        shapes = shapes[:1]
    for d, lv, k in shapes:
        n = 1_000_000
        g = torch.Generator(device='cuda').manual_seed(0)
        z = torch.randn(n, d, device='cuda', generator=g)
        cb = torch.randn(lv, k, d, device='cuda', generator=g)
        for _ in range(2):
            rq_assign(z, cb, want_quant=False)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 10
        e0.record()
        for _ in range(reps):
            rq_assign(z, cb, want_quant=False)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        print(json.dumps({'rows': n, 'latent': d, 'levels': lv, 'codes': k, 'ms': round(ms, 3),
                          'tflops': round(3.0 * n * lv * k * d / (ms * 1e-3) / 1e12, 1)}), flush=True)


if __name__ == '__main__':
    main()
