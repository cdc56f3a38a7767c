"""functional.dnn_weight: the composed itemdnn weight of the projection restatement
as one autograd node on grk_dnn_weight_fwd / _bwd (round 5; round 4: torch ops in one
node), against the eager composition it replaces (model._dnn_weight's torch form,
run by torch on the same device) -- values and every input's gradient.  Tolerances:
the kernels sum the K = kk products in k order, torch's GEMM in its own order."""
import pytest
import torch

from tencent_recommendation_2025_amd import functional as G

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _eager(blocks, bias, mms, width):
    cols, b = list(blocks), bias[:, None]
    for Wk, Wt, bt in mms:
        Mk = Wk @ torch.cat([Wt, bt[:, None]], 1)
        cols.append(Mk[:, :-1])
        b = b + Mk[:, -1:]
    cols.append(b)
    Wc = torch.cat(cols, 1)
    return torch.nn.functional.pad(Wc, (0, width - Wc.shape[1]))


def nrel(a, b):
    return float((a.double() - b.double()).norm() / max(float(b.double().norm()), 1e-30))


def _inputs(d=64, nb=3, mm=(32, 16)):
    g = torch.Generator().manual_seed(0)
    W = torch.randn(d, nb * d + len(mm) * d, generator=g).to(DEV).requires_grad_(True)
    blocks = [W[:, j * d:(j + 1) * d] for j in range(nb)]
    mms = []
    for i, k in enumerate(mm):
        Wk = W[:, (nb + i) * d:(nb + i + 1) * d]
        mms.append((Wk, torch.randn(d, k, generator=g).to(DEV).requires_grad_(True),
                    torch.randn(d, generator=g).to(DEV).requires_grad_(True)))
    bias = torch.randn(d, generator=g).to(DEV).requires_grad_(True)
    width = nb * d + sum(mm) + 1 + 7
    return W, blocks, bias, mms, width


@pytest.fixture(params=[True, False], ids=['kernels', 'torch'])
def path(request, monkeypatch):
    """Both forms of the node: grk_dnn_weight_fwd / _bwd (GRK_DNNW_KERNEL=1) and torch ops."""
    monkeypatch.setattr(G, 'DNNW_KERNEL', request.param)
    return request.param


@pytest.mark.parametrize('d,nb,mm', [(64, 3, (32, 16)), (512, 1, (32,)), (96, 2, ())])
def test_dnn_weight_matches_eager_composition(path, d, nb, mm):
    W, blocks, bias, mms, width = _inputs(d, nb, mm)
    got = G.dnn_weight(blocks, bias, mms, width, torch.float32)
    want = _eager(blocks, bias, mms, width)
    assert got.shape == want.shape
    # normwise: the K = kk sums (512 terms at d = 512) in two summation orders
    assert nrel(got, want) < 2e-6
    gy = torch.randn(got.shape, generator=torch.Generator().manual_seed(1)).to(DEV)
    leaves = [W, bias] + [t for m in mms for t in m[1:]]
    ga = torch.autograd.grad(got, leaves, gy)
    gb = torch.autograd.grad(want, leaves, gy)
    for a, b in zip(ga, gb):
        assert nrel(a, b) < 1e-5


def test_dnn_weight_casts_once_and_returns_fp32_gradients(path):
    W, blocks, bias, mms, width = _inputs(mm=(8,))
    got = G.dnn_weight(blocks, bias, mms, width, torch.bfloat16)
    assert got.dtype == torch.bfloat16
    want = _eager(blocks, bias, mms, width).detach()
    assert torch.allclose(got.float(), want.to(torch.bfloat16).float(), rtol=2 ** -7, atol=1e-6)   # <= 1 bf16 ulp
    got.float().sum().backward()
    assert W.grad.dtype == torch.float32 and bias.grad.dtype == torch.float32
    assert torch.all(bias.grad == 1)   # d(sum)/d bias: each bias element enters one entry once
