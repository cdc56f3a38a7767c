"""Negative sampling (grk_sample_negatives) on the CPU side: the oracle's
contract against the reference's own draws (tests/golden/dataset.npz, written
by the reference MyDataset) and the C ABI's host-side argument checks.

The reference draws with np.random (model/BaseLine/dataset.py:79-95), which no
device generator reproduces: the *values* are parity-unpinned, the properties
the reference guarantees are pinned -- negatives exactly at the positions with
an item next token and a positive (dataset.py:156-161), in [1, itemnum], never
one of the user's items (ts, dataset.py:136-139)."""
import numpy as np
import pytest

from conftest import GOLDEN
from oracle import sampler as osamp


def check_contract(neg, seq, pos, tt, ntt, num_items):
    want_pos = (ntt == 1) & (pos != 0)
    assert np.array_equal(neg != 0, want_pos)
    assert neg[want_pos].min(initial=1) >= 1 and neg[want_pos].max(initial=1) <= num_items
    for b in range(neg.shape[0]):
        window = set(seq[b][tt[b] == 1].tolist()) | set(pos[b].tolist())
        window.discard(0)
        assert not (set(neg[b][neg[b] != 0].tolist()) & window)


@pytest.fixture(scope='module')
def ds():
    return np.load(GOLDEN / 'dataset.npz')


def test_reference_draws_satisfy_the_contract(ds):
    check_contract(ds['neg'], ds['seq'], ds['pos'], ds['token_type'], ds['next_token_type'], int(ds['itemnum']))


def test_oracle_satisfies_the_contract_on_reference_batches(ds):
    seq, pos, tt, ntt = ds['seq'], ds['pos'], ds['token_type'], ds['next_token_type']
    excl = np.concatenate([np.where(tt == 1, seq, 0), pos], 1)
    n = int(ds['itemnum'])
    for seed in (0, 1, 2 ** 63 + 5):
        neg, _, flag = osamp.sample_negatives(pos, ntt, excl, n, seed)
        assert not flag
        check_contract(neg, seq, pos, tt, ntt, n)
    a = osamp.sample_negatives(pos, ntt, excl, n, 7)[0]
    assert np.array_equal(a, osamp.sample_negatives(pos, ntt, excl, n, 7)[0])
    assert not np.array_equal(a, osamp.sample_negatives(pos, ntt, excl, n, 8)[0])


def test_oracle_draws_are_uniform():
    """Chi-square over 20 ids with nothing excluded: the range map has no bias."""
    n, B, T = 20, 40, 50
    pos = np.ones((B, T), np.int32)
    ntt = np.ones((B, T), np.int32)
    neg = osamp.sample_negatives(pos, ntt, np.zeros((B, 1), np.int32), n, 3)[0]
    counts = np.bincount(neg.ravel(), minlength=n + 1)[1:]
    exp = B * T / n
    chi2 = ((counts - exp) ** 2 / exp).sum()
    assert chi2 < 43.8  # p = 0.001 at 19 degrees of freedom


def test_oracle_redraws_ids_without_feature_rows():
    """_random_neq also redraws ids missing from item_feat_dict (dataset.py:92):
    with every odd id featureless, no negative is odd; the ids with features
    keep the draws they had without the mask."""
    rng = np.random.default_rng(1)
    n, B, T = 200, 6, 40
    pos = rng.integers(1, n + 1, (B, T)).astype(np.int32)
    ntt = rng.integers(0, 3, (B, T)).astype(np.int32)
    excl = rng.integers(0, n + 1, (B, 30)).astype(np.int32)
    ok = np.arange(n + 1) % 2 == 0
    neg, _, flag = osamp.sample_negatives(pos, ntt, excl, n, 11, item_ok=ok)
    free, _, _ = osamp.sample_negatives(pos, ntt, excl, n, 11)
    assert not flag
    assert np.all(neg[neg != 0] % 2 == 0)
    same = (free != 0) & (free % 2 == 0)
    assert np.array_equal(neg[same], free[same])       # a first draw with features is kept
    assert np.array_equal(neg != 0, free != 0)


def test_oracle_exhaustion_keeps_last_draw_and_flags():
    pos = np.array([[5, 6]], np.int32)
    ntt = np.array([[1, 1]], np.int32)
    neg, _, flag = osamp.sample_negatives(pos, ntt, np.array([[1, 2, 3]], np.int32), 3, 0, max_tries=8)
    assert flag and set(neg.ravel().tolist()) <= {1, 2, 3}


def test_capi_rejects_bad_arguments():
    from tencent_recommendation_2025_amd import _lib as L
    h = L.lib()
    rc = h.grk_sample_negatives(None, None, 4, 10, None, -1, 100, 0, 10, None, 0, None, None, None, None, None)
    assert rc == L.GRK_EINVAL and b'excl_len' in h.grk_last_error()
    rc = h.grk_sample_negatives(None, None, 4, 10, None, 5000, 100, 0, 10, None, 0, None, None, None, None, None)
    assert rc == L.GRK_EINVAL and b'excl is NULL' in h.grk_last_error()   # any length, but a list is required
    rc = h.grk_sample_negatives(None, None, 4, 10, None, 0, 0, 0, 10, None, 0, None, None, None, None, None)
    assert rc == L.GRK_EINVAL and b'num_items' in h.grk_last_error()
    rc = h.grk_sample_negatives(None, None, 4, 10, None, 0, 100, 0, 0, None, 0, None, None, None, None, None)
    assert rc == L.GRK_EINVAL and b'max_tries' in h.grk_last_error()
    assert h.grk_sample_negatives(None, None, 0, 10, None, 0, 100, 0, 10, None, 0, None, None, None, None, None) == 0
