"""CPU checks of the autograd wiring of round 4's fused forms, with the device
kernels replaced by torch restatements of their documented semantics (the
kernels themselves are checked on the GPU: tests/test_gpu_linear.py,
tests/test_gpu_emb_combine.py).  What is checked here is the Python side:
which tensors the Functions save, which gradients they return in which slot,
and that the in-place linear's output lives in its addend's storage while
autograd still routes the addend's gradient to its producer."""
import pytest
import torch

from tencent_recommendation_2025_amd import functional as G
from tencent_recommendation_2025_amd import kernels as K


def _fake_gemm(a, b, trans_a=False, trans_b=False, out=None, out_dtype=torch.bfloat16, alpha=1.0, beta=0.0,
               bias=None, addend=None, relu=False):
    """kernels.gemm's contract (grk_gemm_ex) in torch: alpha op(a) op(b) + beta C (+ bias), relu."""
    A = a.float().t() if trans_a else a.float()
    B = b.float().t() if trans_b else b.float()
    r = alpha * (A @ B)
    if beta != 0.0:
        r = r + beta * (addend if addend is not None else out).float()
    if bias is not None:
        r = r + bias.float()
    if relu:
        r = torch.relu(r)
    if out is None:
        out = torch.empty(r.shape, dtype=addend.dtype if addend is not None else out_dtype)
    out.copy_(r)
    return out


class _Producer(torch.autograd.Function):
    """Two column blocks of ONE buffer, as the fused gather returns them."""

    @staticmethod
    def forward(ctx, xs, ps):
        buf = torch.empty(xs.shape[0], xs.shape[1] + ps.shape[1] + 8, dtype=torch.bfloat16)
        k = xs.shape[1]
        buf[:, :k] = xs
        buf[:, k:k + ps.shape[1]] = ps
        return buf[:, :k], buf[:, k:k + ps.shape[1]]

    @staticmethod
    def backward(ctx, gx, gp):
        return (None if gx is None else gx.float()), (None if gp is None else gp.float())


def test_in_place_relu_linear_routes_every_gradient(monkeypatch):
    monkeypatch.setattr(K, 'gemm', _fake_gemm)
    monkeypatch.setattr(K, 'wgrad_ok', lambda *a: False)
    g = torch.Generator().manual_seed(0)
    M, Kd, N = 40, 24, 16
    xs = torch.randn(M, Kd, generator=g).bfloat16().float().requires_grad_(True)
    ps = torch.randn(M, N, generator=g).bfloat16().float().requires_grad_(True)
    w = (0.3 * torch.randn(N, Kd, generator=g)).requires_grad_(True)
    b = torch.randn(N, generator=g).requires_grad_(True)
    xv, pv = _Producer.apply(xs, ps)
    y = G.linear(xv, w, b, addend=pv, relu=True, in_place=True)
    assert y.untyped_storage().data_ptr() == pv.untyped_storage().data_ptr()    # accumulated where it lies
    gy = torch.randn(M, N, generator=g)
    (y.float() * gy).sum().backward()
    xr, pr = xs.detach().requires_grad_(True), ps.detach().requires_grad_(True)
    wr, br = w.detach().bfloat16().float().requires_grad_(True), b.detach().requires_grad_(True)
    yr = torch.relu(xr @ wr.t() + br + pr)
    (yr * gy).sum().backward()
    assert torch.allclose(y.float(), yr, rtol=1e-2, atol=1e-2)
    for name, got, want in (('x', xs.grad, xr.grad), ('p', ps.grad, pr.grad), ('w', w.grad, wr.grad),
                            ('b', b.grad, br.grad)):
        assert got is not None, name
        assert float((got - want).norm() / want.norm()) < 2e-2, name


def _fake_combine_fwd(a, b, pos, scale, relu=True, dropout_p=0.0, seed=0):
    act = torch.relu if relu else (lambda t: t)
    s = act(a.float()) + (act(b.float()) if b is not None else 0)
    s = s * scale + (pos.float() if pos is not None else 0)
    return s.bfloat16()


def _fake_combine_bwd(gy, a, b, scale, relu=True, dropout_p=0.0, seed=0, want=(True, True, True), has_b=None):
    g = gy.float()
    has_b = b is not None if has_b is None else has_b
    ga = (g * scale * ((a.float() > 0) if relu else 1)).bfloat16() if want[0] else None
    gb = (g * scale * ((b.float() > 0) if relu else 1)).bfloat16() if want[1] and has_b else None
    gp = g.bfloat16() if want[2] else None
    return ga, gb, gp


@pytest.mark.parametrize('relu', [True, False])
def test_emb_combine_returns_gradients_in_input_order(monkeypatch, relu):
    monkeypatch.setattr(K, 'emb_combine_fwd', _fake_combine_fwd)
    monkeypatch.setattr(K, 'emb_combine_bwd', _fake_combine_bwd)
    g = torch.Generator().manual_seed(1)
    N, D = 30, 16
    a, b, p = (torch.randn(N, D, generator=g).bfloat16().requires_grad_(True) for _ in range(3))
    y = G.emb_combine(a, b, p, 3.0, relu=relu)
    gy = torch.randn(N, D, generator=g).bfloat16()
    y.backward(gy)
    af, bf, pf = (t.detach().float().requires_grad_(True) for t in (a, b, p))
    act = torch.relu if relu else (lambda t: t)
    yr = (act(af) + act(bf)) * 3.0 + pf
    yr.backward(gy.float())
    assert torch.allclose(y.float(), yr, rtol=1e-2, atol=1e-2)
    for name, got, want in (('a', a.grad, af.grad), ('b', b.grad, bf.grad), ('pos', p.grad, pf.grad)):
        assert got is not None and got.dtype == torch.bfloat16, name
        assert torch.allclose(got.float(), want, rtol=1e-2, atol=1e-2), name
