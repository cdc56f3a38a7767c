"""The fused step's index kernels (csrc/grk_index.hip) against the torch forms they
replace, bit for bit: grk_proj_index (model._proj_index: the projected tables' bag
index) and grk_batch_row_ids (FusedAdamW.begin_step's catch-up ids)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


@pytest.mark.parametrize('dtype', [torch.int64, torch.int32])
def test_proj_index_matches_torch(dtype):
    from tencent_recommendation_2025_amd import kernels as K
    g = torch.Generator(device=DEV).manual_seed(0)
    N = 3001
    widths, offs = [1, 1, 4, 1, 3], [1, 12, 113, 1114, 11115]
    feats = [torch.randint(0, 11, (N, w), device=DEV, generator=g).to(dtype) for w in widths]
    feats[2] = feats[2][:, :4]                        # a sliced view (row stride 4)
    wide = torch.randint(0, 9, (N, 6), device=DEV, generator=g).to(dtype)
    feats[4] = wide[:, 1:4]                           # row stride 6 > width 3
    got = K.proj_index(list(zip(feats, offs)), N)
    x = torch.cat([f.long() for f in feats], 1)
    off = torch.tensor([o for o, w in zip(offs, widths) for _ in range(w)], device=DEV)
    want = torch.where(x > 0, x + off, 0)
    assert got.dtype == torch.int64 and torch.equal(got, want)


@pytest.mark.parametrize('dtype', [torch.int64, torch.int32])
def test_batch_row_ids_match_torch(dtype):
    from tencent_recommendation_2025_amd import kernels as K
    g = torch.Generator(device=DEV).manual_seed(1)
    B, T = 33, 57
    tt = torch.randint(0, 3, (B, T), device=DEV, generator=g)
    seq = torch.randint(0, 1000, (B, T), device=DEV, generator=g) * (tt != 0)
    pos = torch.randint(0, 1000, (B, T), device=DEV, generator=g)
    neg = torch.randint(0, 1000, (B, T), device=DEV, generator=g)
    item, user = K.batch_row_ids(seq.to(dtype), pos.to(dtype), neg.to(dtype), tt.to(dtype))
    skip = torch.full((), -1, dtype=torch.long, device=DEV)
    want_i = torch.cat([torch.where(tt == 1, seq, 0).reshape(-1), pos.reshape(-1), neg.reshape(-1)])
    want_i = torch.where(want_i > 0, want_i, skip)
    want_u = torch.where((tt == 2) & (seq > 0), seq, skip).reshape(-1)
    assert torch.equal(item, want_i) and torch.equal(user, want_u)
    item2, none = K.batch_row_ids(seq, pos, neg, tt, with_user=False)
    assert none is None and torch.equal(item2, want_i)
