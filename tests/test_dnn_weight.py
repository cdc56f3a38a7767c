"""functional.dnn_weight (round 4): the composed itemdnn weight of the projection
restatement as one autograd node, against the eager composition it replaces
(model._dnn_weight's torch form) -- values and every input's gradient, on CPU."""
import torch

from tencent_recommendation_2025_amd import functional as G


def _eager(blocks, bias, mms, width):
    cols, b = list(blocks), bias[:, None]
    for Wk, Wt, bt in mms:
        Mk = Wk @ torch.cat([Wt, bt[:, None]], 1)
        cols.append(Mk[:, :-1])
        b = b + Mk[:, -1:]
    cols.append(b)
    Wc = torch.cat(cols, 1)
    return torch.nn.functional.pad(Wc, (0, width - Wc.shape[1]))


def _inputs(d=64, nb=3, mm=(32, 16)):
    g = torch.Generator().manual_seed(0)
    W = torch.randn(d, nb * d + len(mm) * d, generator=g).requires_grad_(True)
    blocks = [W[:, j * d:(j + 1) * d] for j in range(nb)]
    mms = []
    for i, k in enumerate(mm):
        Wk = W[:, (nb + i) * d:(nb + i + 1) * d]
        mms.append((Wk, torch.randn(d, k, generator=g).requires_grad_(True),
                    torch.randn(d, generator=g).requires_grad_(True)))
    bias = torch.randn(d, generator=g).requires_grad_(True)
    width = nb * d + sum(mm) + 1 + 7
    return W, blocks, bias, mms, width


def test_dnn_weight_matches_eager_composition():
    W, blocks, bias, mms, width = _inputs()
    got = G.dnn_weight(blocks, bias, mms, width, torch.float32)
    want = _eager(blocks, bias, mms, width)
    assert got.shape == want.shape
    assert torch.allclose(got, want, rtol=1e-6, atol=1e-5)
    gy = torch.randn(got.shape, generator=torch.Generator().manual_seed(1))
    leaves = [W, bias] + [t for m in mms for t in m[1:]]
    ga = torch.autograd.grad(got, leaves, gy)
    gb = torch.autograd.grad(want, leaves, gy)
    for a, b in zip(ga, gb):
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-4)


def test_dnn_weight_casts_once_and_returns_fp32_gradients():
    W, blocks, bias, mms, width = _inputs(mm=(8,))
    got = G.dnn_weight(blocks, bias, mms, width, torch.bfloat16)
    assert got.dtype == torch.bfloat16
    assert torch.equal(got, _eager(blocks, bias, mms, width).detach().to(torch.bfloat16))
    got.float().sum().backward()
    assert W.grad.dtype == torch.float32 and bias.grad.dtype == torch.float32
    assert torch.all(bias.grad == 1)   # d(sum)/d bias: each bias element enters one entry once
