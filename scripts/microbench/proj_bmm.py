"""The projected feature tables' GEMMs of the C2 step (model._projection:
P = E W^T per table group, and its backward dE = dP W, dW = dP^T E) -- torch.bmm
as the model issues them vs grk_gemm per block, device time per call.

    python scripts/microbench/proj_bmm.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

D = 512
# (tables, rows) per equal-row-count group at C2: item 3x10001, 3x1001, 4x101, 4x11; user 8x1001
GROUPS = [(3, 10001), (3, 1001), (4, 101), (4, 11), (8, 1001)]


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    from tencent_recommendation_2025_amd import kernels as K
    dev = torch.device('cuda')
    g = torch.Generator(device=dev).manual_seed(0)
    tot = {'bmm': 0.0, 'grk': 0.0}
    for G, R in GROUPS:
        E = (0.02 * torch.randn(G, R, D, device=dev, generator=g)).bfloat16()
        W = (0.02 * torch.randn(D, G, D, device=dev, generator=g)).bfloat16().permute(1, 0, 2)   # [G, d_out, d_in], strided
        dP = torch.randn(G, R, D, device=dev, generator=g).bfloat16()
        fl = 2 * G * R * D * D
        t_f = timed(lambda: torch.bmm(E, W.transpose(1, 2)))
        t_de = timed(lambda: torch.bmm(dP, W))
        t_dw = timed(lambda: torch.bmm(dP.transpose(1, 2), E))
        Wc = W.contiguous()
        t_gf = timed(lambda: [K.gemm(E[i], Wc[i], trans_b=True) for i in range(G)])
        t_gde = timed(lambda: [K.gemm(dP[i], Wc[i]) for i in range(G)])
        t_gdw = timed(lambda: [K.wgrad(dP[i], E[i], out_dtype=torch.bfloat16) for i in range(G)])
        tot['bmm'] += t_f + t_de + t_dw
        tot['grk'] += t_gf + t_gde + t_gdw
        print(f'G={G} rows={R}: bmm fwd {t_f:.1f} dE {t_de:.1f} dW {t_dw:.1f} us ({3 * fl / (t_f + t_de + t_dw) / 1e6:.0f} '
              f'TF/s) | grk fwd {t_gf:.1f} dE {t_gde:.1f} dW(wgrad) {t_gdw:.1f} us', flush=True)
    print(f'total per step: torch.bmm {tot["bmm"]:.1f} us, grk per block {tot["grk"]:.1f} us')


if __name__ == '__main__':
    main()
