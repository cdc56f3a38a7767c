"""functional.DenseMerge (CPU): the projected tables' row gradients of several
fused lookups of one forward reduced by ONE embedding-backward call, issued
by whichever lookup's backward runs last.  The device kernels are replaced by
torch stand-ins (gather / scatter-add); what is under test is the host logic:
every merged weight an input of every consumer, None from the earlier
consumers, the sum over all consumers' sources from the last one, in either
backward order, and the same gradients as one call per lookup."""
import pytest
import torch

from tencent_recommendation_2025_amd import functional as G
from tencent_recommendation_2025_amd import kernels as K


class _Res:
    def __init__(self, dense):
        self.dense = dense


def fake_gather(lookups, out, num_tokens, token_type=None, seq_len=0, err_flag=None):
    for lk in lookups:
        idx = lk.idx.reshape(num_tokens, lk.bag).long()
        out[:, lk.out_col:lk.out_col + lk.table.shape[1]] = lk.table[idx].sum(1).to(out.dtype)
    return out


CALLS = []


def fake_backward(sources, num_rows, dim, padding_idx=0, token_type=None, seq_len=0, dense=True, sparse=False,
                  row_slot=None, err_flag=None, chunked=False, dense_dtype=torch.float32):
    CALLS.append(len(sources))
    out = torch.zeros(num_rows, dim, dtype=torch.float64)
    for s in sources:
        n = s.grad.shape[0]
        idx = s.idx.reshape(n, s.bag).long()
        g = s.grad[:, s.grad_col:s.grad_col + dim].double()
        for a in range(s.bag):
            rows = idx[:, a]
            keep = rows != padding_idx
            out.index_add_(0, (rows + s.row_offset)[keep], g[keep])
    return _Res(out.to(dense_dtype))


@pytest.fixture
def fakes(monkeypatch):
    monkeypatch.setattr(K, 'embedding_gather', fake_gather)
    monkeypatch.setattr(K, 'embedding_backward', fake_backward)
    CALLS.clear()


def _step(merge, order):
    torch.manual_seed(0)
    P1 = torch.randn(7, 4, requires_grad=True)
    P2 = torch.randn(5, 4, requires_grad=True)
    m = G.DenseMerge() if merge else None
    if m is not None:
        m.add(P1)
        m.add(P2)
    i_seq1 = torch.randint(0, 7, (6, 3))
    i_seq2 = torch.randint(0, 5, (6, 2))
    i_pair = torch.randint(0, 7, (10, 3))
    seq = G._lookup_groups([G.LookupSpec(G.TableRef(P1, chunked=True, merge=m), i_seq1, 0, bag=3),
                            G.LookupSpec(G.TableRef(P2, chunked=True, merge=m), i_seq2, 4, bag=2)],
                           None, 0, 6, 8, (), ((0, 4), (4, 8)))
    pair = G._lookup_groups([G.LookupSpec(G.TableRef(P1, chunked=True, merge=m), i_pair, 0, bag=3)],
                            None, 0, 10, 4, (), ((0, 4),))
    w = torch.linspace(-1, 1, 4)
    l_seq = (seq[0] * w).sum() + (seq[1] * w).pow(2).sum()
    l_pair = (pair[0] * w).pow(2).sum()
    # the two consumers' backward in either order (autograd runs them as the graph dictates)
    if order == 'pair_first':
        l_pair.backward(retain_graph=True)
        l_seq.backward()
    else:
        l_seq.backward(retain_graph=True)
        l_pair.backward()
    return P1.grad.clone(), P2.grad.clone(), list(CALLS)


@pytest.mark.parametrize('order', ['pair_first', 'seq_first'])
def test_merged_backward_equals_one_call_per_lookup(fakes, order):
    g1, g2, calls = _step(False, order)
    assert calls == [2, 1] or calls == [1, 2]          # one call per lookup
    CALLS.clear()
    m1, m2, mcalls = _step(True, order)
    assert mcalls == [3]                                 # one call over all three sources
    torch.testing.assert_close(m1, g1, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(m2, g2, rtol=1e-6, atol=1e-6)


def test_merge_state_after_resolve(fakes):
    P = torch.randn(4, 2, requires_grad=True)
    m = G.DenseMerge()
    m.add(P)
    m.add(P)
    assert len(m.weights) == 1
    m.pending = 2
    assert m.resolve() == {id(P): None} and m.pending == 1
    out = m.resolve()                                    # last consumer, nothing deposited: no gradient
    assert out == {id(P): None} and m.pending == 0 and m.sources == []
