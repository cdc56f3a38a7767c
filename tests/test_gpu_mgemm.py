"""grk's MFMA GEMM (csrc/grk_mgemm.hip), which grk_gemm runs for the dense layers'
forward and input-gradient products (replacing hipBLASLt there): every epilogue
and layout against torch fp32 on the same bf16 operands, K / M / N tails, operands
that are column blocks of wider buffers (whose columns past K hold NaN: the tail
must be masked, not multiplied), in-place accumulation, run-to-run bitwise
repeatability."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def nrel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp(min=1e-30))


def _operands(m, n, k, layout, g, pad=0):
    """A [m, k] as a column block of an [m, k + pad] buffer (NaN past k), B [n, k] (layout 0)
    or [k, n] (layout 1) likewise."""
    abuf = torch.full((m, k + pad), float('nan'), device=DEV).bfloat16()
    abuf[:, :k] = torch.randn(m, k, device=DEV, generator=g).bfloat16()
    a = abuf[:, :k]
    if layout == 0:
        bbuf = torch.full((n, k + pad), float('nan'), device=DEV).bfloat16()
        bbuf[:, :k] = torch.randn(n, k, device=DEV, generator=g).bfloat16()
        b = bbuf[:, :k]
        ref = a.float() @ b.float().t()
    else:
        bbuf = torch.full((k, n + pad), float('nan'), device=DEV).bfloat16()
        bbuf[:, :n] = torch.randn(k, n, device=DEV, generator=g).bfloat16()
        b = bbuf[:, :n]
        ref = a.float() @ b.float()
    return a, b, ref


@pytest.mark.parametrize('m,n,k', [(14336, 2048, 512), (14336, 512, 2048), (14336, 512, 552), (14336, 552, 512),
                                   (1000, 136, 72), (257, 8, 8), (3, 512, 64), (25728, 512, 512)])
@pytest.mark.parametrize('layout', [0, 1])
def test_mgemm_matches_torch(m, n, k, layout):
    from tencent_recommendation_2025_amd import _lib as L
    from tencent_recommendation_2025_amd import kernels as K
    g = torch.Generator(device=DEV).manual_seed(m + 7 * n + 13 * k + layout)
    a, b, ref = _operands(m, n, k, layout, g, pad=24)
    assert L.lib().grk_gemm_mfma_supported(0, layout, m, n, k, a.stride(0), b.stride(0), n, L.GRK_BF16, 1.0, 0.0)
    bias = torch.randn(n, device=DEV, generator=g)
    mm = K.gemm_mfma
    y = mm(a, b, trans_b=layout == 0)
    assert torch.isfinite(y).all()
    assert nrel(y.float(), ref) < 4e-3
    y2 = mm(a, b, trans_b=layout == 0)
    assert torch.equal(y, y2)                                              # deterministic
    yr = mm(a, b, trans_b=layout == 0, bias=bias, relu=True)               # bias + ReLU in the store
    assert nrel(yr.float(), torch.relu(ref + bias)) < 4e-3
    yb = mm(a, b, trans_b=layout == 0, bias=bias.bfloat16())
    assert nrel(yb.float(), ref + bias.bfloat16().float()) < 4e-3
    y32 = mm(a, b, trans_b=layout == 0, out_dtype=torch.float32)           # fp32 C: only the accumulation order
    assert nrel(y32, ref) < 1e-5
    # accumulate in place into a column block of a wider bf16 buffer (functional.linear in_place)
    cbuf = torch.randn(m, n + 16, device=DEV, generator=g).bfloat16()
    c = cbuf[:, :n]
    keep = cbuf[:, n:].clone()
    want = c.float() + ref
    mm(a, b, trans_b=layout == 0, out=c, c_in=c)
    assert nrel(c.float(), want) < 4e-3
    assert torch.equal(cbuf[:, n:], keep)                                  # columns past n untouched
    # a separate addend
    add = torch.randn(m, n, device=DEV, generator=g).bfloat16()
    ya = mm(a, b, trans_b=layout == 0, c_in=add, relu=True)
    assert nrel(ya.float(), torch.relu(ref + add.float())) < 4e-3
    # grk_gemm's routing: the forward at K % 64 != 0 runs here (the dnn layers), bitwise the same
    if layout == 0 and k % 64:
        assert torch.equal(K.gemm(a, b, trans_b=True, bias=bias, relu=True), yr)


def test_mgemm_rows_past_m_untouched():
    """Output rows past M (a view into a taller buffer) are never written."""
    from tencent_recommendation_2025_amd import kernels as K
    g = torch.Generator(device=DEV).manual_seed(3)
    a, b, ref = _operands(300, 256, 128, 0, g)
    big = torch.full((512, 256), 7.0, device=DEV).bfloat16()
    K.gemm_mfma(a, b, trans_b=True, out=big[:300])
    assert nrel(big[:300].float(), ref) < 4e-3
    assert bool((big[300:] == 7.0).all())
