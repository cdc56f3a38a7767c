"""grk_wgrad (split-K MFMA weight gradient + bias gradient) against a torch
fp64 reference of the same bf16 operands, on the bench's shapes (K = B*T
tokens, the HSTU projections) and on ragged edges; run-to-run bitwise
determinism (in-order slice reduction, no atomics).  K a multiple of 32 takes
the LDS-DMA ring kernels (k_wgrad_lds: 128 x 128 tiles, or 256 x 128 tiles at
M >= 1024), other K the register-staged one."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def nrel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / max(b.norm(), 1e-30))


@pytest.mark.parametrize('K,M,N', [(25728, 2048, 512), (25728, 512, 512), (51456, 512, 560), (1000, 136, 72),
                                   (3, 8, 8), (0, 16, 24), (777, 264, 1032),
                                   (5000, 1032, 1288), (25728, 1024, 1024), (300, 2048, 520),
                                   # K % 32 == 0: the LDS-DMA ring kernel, ragged M / N tiles, short slices
                                   (14336, 2048, 512), (1024, 136, 72), (3200, 264, 1032), (32, 8, 8), (96, 520, 2048),
                                   # M >= 1024: the 256 x 128-tile ring (ragged M / N tiles, short slices)
                                   (3200, 1032, 1288), (64, 1024, 8), (28672, 4096, 512)])
def test_wgrad_matches_fp64(K, M, N):
    from tencent_recommendation_2025_amd import kernels as Kn
    g = torch.Generator(device=DEV).manual_seed(K + M + N)
    dy = torch.randn(K, M, device=DEV, generator=g).bfloat16()
    x = torch.randn(K, N, device=DEV, generator=g).bfloat16()
    dw, db = Kn.wgrad(dy, x, want_db=True)
    ref = dy.double().t() @ x.double()
    refb = dy.double().sum(0)
    if K == 0:
        assert not dw.any() and not db.any()
        return
    assert nrel(dw, ref) < 2e-6, nrel(dw, ref)
    assert nrel(db, refb) < 2e-6, nrel(db, refb)
    dw2, db2 = Kn.wgrad(dy, x, want_db=True)
    assert torch.equal(dw, dw2) and torch.equal(db, db2)
    dwb, none = Kn.wgrad(dy, x, out_dtype=torch.bfloat16)
    assert none is None and dwb.dtype == torch.bfloat16
    assert nrel(dwb, ref) < 4e-3


def test_wgrad_strided_views():
    """Column blocks of wider activations (row stride > width), as the fused gather hands them out."""
    from tencent_recommendation_2025_amd import kernels as Kn
    g = torch.Generator(device=DEV).manual_seed(9)
    big = torch.randn(4096, 1024, device=DEV, generator=g).bfloat16()
    dy, x = big[:, 256:512], big[:, 512:1000]
    assert Kn.wgrad_ok(dy, x)
    dw, db = Kn.wgrad(dy, x, want_db=True)
    assert nrel(dw, dy.double().t() @ x.double()) < 2e-6
    assert nrel(db, dy.double().sum(0)) < 2e-6
