"""functional.weight_blocks (the itemdnn / userdnn column blocks of the projection
restatement, model._weight_pieces) against the autograd chain it replaced in
model._projection / model._dnn_weight: column slices of the fp32 weight, the
whole weight cast once to the tables' dtype and indexed per equal-row-count
group.  Forward outputs and the weight gradient must be the same bits (CPU; the
GPU model tests run the integrated path against the reference goldens), and
the backward must issue a handful of block copies instead of a full-size zero
fill per slice / group plus the adds and the cast."""
import collections

import pytest
import torch
from torch.utils._python_dispatch import TorchDispatchMode

from tencent_recommendation_2025_amd import functional as G


class OpCount(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.ops = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        self.ops[str(func.overloadpacket)] += 1
        return func(*args, **(kwargs or {}))


VIEWS = {'aten.view', 'aten.permute', 'aten.select', 'aten.slice', 'aten.detach', 'aten.t', 'aten.transpose',
         'aten.expand', 'aten.as_strided', 'aten.empty', 'aten.unsqueeze', 'aten.alias'}


def kernels(ops):
    """Device kernels an op census stands for: views / allocations none, slice_backward
    two (a full-size zero fill and the copy), everything else one."""
    return sum(n * (2 if k == 'aten.slice_backward' else 1) for k, n in ops.items() if k not in VIEWS)


def old_chain(W, d, singles, stacks):
    """model._projection / _dnn_weight before weight_blocks (round 3)."""
    outs = [W[:, j * d:(j + 1) * d] for j in singles]
    Wv = W.view(W.shape[0], -1, d)
    for js, dt in stacks:
        if Wv.dtype != dt:
            Wv = Wv.to(dt)
        if len(js) > 1:
            outs.append(Wv[:, torch.tensor(js), :].permute(1, 0, 2))
        else:
            outs.append(Wv[:, js[0], :][None])
    return outs


CASES = {
    # C2 itemdnn: W_0 + mm block single, four equal-row-count groups projected (bf16 tables)
    'item_bf16': (16, [0, 15], [((1, 2, 3, 4), torch.bfloat16), ((5, 6, 7, 8), torch.bfloat16),
                                ((9, 10, 11), torch.bfloat16), ((12, 13, 14), torch.bfloat16)]),
    # userdnn: one group
    'user_bf16': (9, [0], [((1, 2, 3, 4, 5, 6, 7, 8), torch.bfloat16)]),
    # drop-in (fp32 tables), a direct-feature block, a one-table group, an unreached block (13)
    'mixed_f32': (14, [0, 3, 12], [((1, 2), torch.float32), ((4,), torch.float32),
                                   ((5, 6, 7, 8, 9, 10, 11), torch.float32)]),
}


@pytest.mark.parametrize('case', sorted(CASES))
def test_weight_blocks_bitwise_equal_to_the_slice_chain(case):
    nb, singles, stacks = CASES[case]
    d, dout = 32, 24
    g = torch.Generator().manual_seed(7)
    W0 = torch.randn(dout, nb * d, generator=g)
    outs_g = []
    for o in old_chain(W0, d, singles, stacks):
        outs_g.append(torch.randn(o.shape, generator=g).to(o.dtype))
    grads = {}
    for name, fn in (('old', old_chain), ('new', lambda *a: G.weight_blocks(*a)),
                     ('sliced', lambda *a: G.weight_blocks_sliced(*a))):
        W = W0.clone().requires_grad_(True)
        outs = fn(W, d, singles, stacks)
        ref = old_chain(W0, d, singles, stacks)
        assert len(outs) == len(ref)
        for o, r in zip(outs, ref):
            assert o.dtype == r.dtype and o.shape == r.shape and o.stride() == r.stride()
            assert torch.equal(o, r)
        used = [(o, gr) for o, gr in zip(outs, outs_g)]
        counter = OpCount()
        with counter:
            torch.autograd.backward([o for o, _ in used], [gr for _, gr in used])
        grads[name] = (W.grad.clone(), counter.ops)
    assert torch.equal(grads['old'][0], grads['new'][0])
    assert torch.equal(grads['old'][0], grads['sliced'][0])       # the form torch.compile traces
    old_k, new_k = kernels(grads['old'][1]), kernels(grads['new'][1])
    # the replaced chain zero-fills one full-size tensor per slice / group and adds them
    assert new_k < old_k, (grads['old'][1], grads['new'][1])
    assert not any(k in grads['new'][1] for k in ('aten.zeros', 'aten.new_zeros', 'aten.slice_backward', 'aten.add'))


def test_weight_blocks_unused_outputs_and_refusals():
    """An output nobody reads leaves its blocks zero in the gradient (set_materialize_grads
    False: no zero tensors materialised for it); overlapping or out-of-range blocks refused."""
    d, dout, nb = 8, 4, 6
    W = torch.randn(dout, nb * d, requires_grad=True)
    a, b, st = G.weight_blocks(W, d, [0, 5], [((1, 3), torch.float32)])
    (a.sum() + st.sum()).backward()
    gv = W.grad.view(dout, nb, d)
    assert torch.equal(gv[:, 0], torch.ones(dout, d)) and torch.equal(gv[:, 1], torch.ones(dout, d))
    assert torch.equal(gv[:, 3], torch.ones(dout, d))
    assert not gv[:, [2, 4, 5]].any()          # 2, 4: in no output; 5: its output unused
    with pytest.raises(ValueError):
        G.weight_blocks(W, d, [0, 1], [((1, 2), torch.float32)])
    with pytest.raises(ValueError):
        G.weight_blocks(W, d, [6], [])
