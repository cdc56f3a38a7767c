"""CPU: the grk:: custom ops (tencent_recommendation_2025_amd/ops.py) trace
without a GPU -- their fake implementations give the output shapes / dtypes
torch.compile needs, and their registered autograd formulas trace a backward
(make_fx over forward + torch.autograd.grad, fake tensors)."""
import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode
from torch.fx.experimental.proxy_tensor import make_fx

import tencent_recommendation_2025_amd.ops  # noqa: F401  (registers the ops)
from tencent_recommendation_2025_amd import _lib as L

B, T, H, hd = 2, 7, 2, 16
D = H * hd


def _grk_nodes(gm):
    return sorted({str(n.target) for n in gm.graph.nodes if n.op == 'call_function' and 'grk' in str(n.target)})


@pytest.mark.parametrize('dt', [torch.float32, torch.float16, torch.bfloat16])
def test_softmax_attention_traces_forward_and_backward(dt):
    def f(qkv, kv):
        out, _ = torch.ops.grk.softmax_attention(qkv, kv, H, hd, 0.0, 0, None, 1, None)
        return torch.autograd.grad(out.float().sum(), qkv)[0]

    qkv = torch.randn(B * T, 3 * D, dtype=dt, requires_grad=True)
    kv = torch.ones(B, T, dtype=torch.uint8)
    gm = make_fx(f, tracing_mode='fake')(qkv, kv)
    assert _grk_nodes(gm) == ['grk.softmax_attention.default', 'grk.softmax_attention_backward.default']
    with FakeTensorMode():
        q = torch.empty(B * T, 3 * D, dtype=dt, device='cuda')
        out, lse = torch.ops.grk.softmax_attention(q, torch.empty(B, T, dtype=torch.uint8, device='cuda'), H, hd,
                                                   0.0, 0, None, 1, None)
        # fp32 / fp16 inputs: fp32-fidelity kernels with fp32 output; bf16: bf16 output
        assert out.shape == (B * T, D) and lse.shape == (B, H, T) and lse.dtype == torch.float32
        assert out.dtype == (torch.bfloat16 if dt == torch.bfloat16 else torch.float32)


def test_hstu_core_traces_forward_and_backward():
    def f(pre, rab, w, b, kv):
        y, _, _ = torch.ops.grk.hstu_core(pre, rab, w, b, kv, H, hd, 1.0 / T, 1e-8, 1, 0.0, 0, None, None)
        return torch.autograd.grad(y.float().sum(), (pre, rab, w, b))

    pre = torch.randn(B * T, 4 * D, dtype=torch.bfloat16, requires_grad=True)
    rab = torch.zeros(H, T, requires_grad=True)
    w, b = torch.ones(D, requires_grad=True), torch.zeros(D, requires_grad=True)
    gm = make_fx(f, tracing_mode='fake')(pre, rab, w, b, torch.ones(B, T, dtype=torch.uint8))
    assert _grk_nodes(gm) == ['grk.hstu_core.default', 'grk.hstu_core_backward.default']


def test_pair_logits_and_lookup_trace():
    def f(h, ep, en, ntt, t1, t2, idx1, idx2):
        pos, neg = torch.ops.grk.pair_logits(h, ep, en, ntt)
        out = torch.ops.grk.feature_lookup([t1, t2], [idx1, idx2], [0, 1], [0, 8], [L.IDX_PLAIN, L.IDX_PLAIN], [1, 3],
                                           None, 0, B * T, 16)
        loss = pos.sum() - neg.sum() + out.sum()
        return torch.autograd.grad(loss, (h, ep, en, t1, t2))

    N = B * T
    h, ep, en = (torch.randn(N, 8, requires_grad=True) for _ in range(3))
    t1, t2 = torch.randn(11, 8, requires_grad=True), torch.randn(5, 8, requires_grad=True)
    gm = make_fx(f, tracing_mode='fake')(h, ep, en, torch.ones(N, dtype=torch.int32), t1, t2,
                                         torch.randint(0, 11, (N,)), torch.randint(0, 5, (N, 3)))
    assert _grk_nodes(gm) == ['grk.feature_lookup.default', 'grk.feature_lookup_backward.default',
                              'grk.pair_logits.default', 'grk.pair_logits_backward.default']


def test_hstu_core_time_bias_traces_forward_and_backward():
    def f(pre, rab, w, b, kv, ts, rab_t):
        y, _, _ = torch.ops.grk.hstu_core(pre, rab, w, b, kv, H, hd, 1.0 / T, 1e-8, 1, 0.0, 0, None, None, ts, rab_t)
        return torch.autograd.grad(y.float().sum(), (pre, rab, w, b, rab_t))

    pre = torch.randn(B * T, 4 * D, dtype=torch.bfloat16, requires_grad=True)
    rab, rab_t = torch.zeros(H, T, requires_grad=True), torch.zeros(H, 16, requires_grad=True)
    w, b = torch.ones(D, requires_grad=True), torch.zeros(D, requires_grad=True)
    ts = torch.arange(B * T, dtype=torch.int64).view(B, T)
    gm = make_fx(f, tracing_mode='fake')(pre, rab, w, b, torch.ones(B, T, dtype=torch.uint8), ts, rab_t)
    assert _grk_nodes(gm) == ['grk.hstu_core.default', 'grk.hstu_core_backward.default']
    outs = [n for n in gm.graph.nodes if n.op == 'output'][0].args[0]
    assert outs[4].meta['val'].shape == (H, 16)   # drab_t
