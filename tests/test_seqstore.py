"""Tensorised data path (SeqStore) on the CPU: the batch it
assembles from its columnar cache equals the reference's own MyDataset +
collate output (tests/golden/dataset.npz, written by the imported reference)
and this package's MyDataset.collate_tensor_fn on a larger synthetic
directory -- every field but the negatives, which the device draws
(tests/test_gpu_seqstore.py)."""
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from conftest import GOLDEN_DATA_KW


@pytest.fixture(scope='module')
def golden_dir(tmp_path_factory):
    from tencent_recommendation_2025_amd.dataset import write_synthetic_tencentgr
    d = tmp_path_factory.mktemp('tgr')
    write_synthetic_tencentgr(d, **GOLDEN_DATA_KW)
    return d


def test_store_batch_matches_reference_golden(golden, golden_dir):
    from tencent_recommendation_2025_amd.seqstore import SeqStore
    d = golden('dataset.npz')
    st = SeqStore(golden_dir, maxlen=20)
    assert st.itemnum == int(d['itemnum']) and st.usernum == int(d['usernum'])
    b = st.batch(d['uids'])
    for i, k in enumerate(('seq', 'pos', 'neg', 'token_type', 'next_token_type', 'next_action_type')):
        if k == 'neg':
            assert torch.all(b[i] == 0)
            continue
        assert b[i].dtype == torch.int32 and np.array_equal(b[i].numpy(), d[k]), k
    for j, side in ((6, 'seq_feat'), (7, 'pos_feat')):
        keys = sorted(k.split('.', 1)[1] for k in d.files if k.startswith(side + '.'))
        assert sorted(b[j]) == keys
        for k in keys:
            want = d[f'{side}.{k}']
            assert b[j][k].dtype == torch.from_numpy(want).dtype and np.array_equal(b[j][k].numpy(), want), (side, k)


@pytest.mark.parametrize('maxlen', [20, 7, 60])
def test_store_batch_matches_collate_tensor_fn(tmp_path, maxlen):
    """Every user of a 200-user directory (histories 3..90 events: shorter and
    longer than the window), in shuffled batches."""
    from tencent_recommendation_2025_amd.dataset import MyDataset, write_synthetic_tencentgr
    from tencent_recommendation_2025_amd.seqstore import SeqStore
    write_synthetic_tencentgr(tmp_path, num_users=200, num_items=800, max_events=90, seed=3)
    ds = MyDataset(tmp_path, SimpleNamespace(maxlen=maxlen, mm_emb_id=['81']))
    st = SeqStore(tmp_path, maxlen=maxlen)
    order = np.random.default_rng(0).permutation(len(ds))
    for s in range(0, len(order), 64):
        uids = order[s:s + 64]
        np.random.seed(1)
        want = ds.collate_tensor_fn([ds[int(u)] for u in uids])
        got = st.batch(uids)
        for i in (0, 1, 3, 4, 5):
            assert torch.equal(got[i], want[i]), i
        for j in (6, 7):
            assert list(got[j]) == list(want[j])
            for k in want[j]:
                assert got[j][k].dtype == want[j][k].dtype and torch.equal(got[j][k], want[j][k]), (j, k)


def test_store_cache_reused_and_history(tmp_path):
    from tencent_recommendation_2025_amd.dataset import MyDataset, write_synthetic_tencentgr
    from tencent_recommendation_2025_amd.seqstore import SeqStore
    write_synthetic_tencentgr(tmp_path, num_users=30, num_items=100, max_events=50, seed=5)
    st = SeqStore(tmp_path, maxlen=10)
    stamp = (tmp_path / 'grk_seqstore' / 'tid.npy').stat().st_mtime_ns
    st2 = SeqStore(tmp_path, maxlen=25)                 # another window over the same cache
    assert (tmp_path / 'grk_seqstore' / 'tid.npy').stat().st_mtime_ns == stamp and len(st2) == 30
    ds = MyDataset(tmp_path, SimpleNamespace(maxlen=10, mm_emb_id=['81']))
    uids = np.r_[np.arange(30), [7, 7, 0]]               # repeated users are fine
    hist = st.history_items(uids).numpy()
    width = 0
    for r, u in enumerate(uids):
        recs = ds._load_user_data(int(u))
        items = sorted({i for _, i, _, f, _, _ in recs if i and f})
        width = max(width, len(items))
        # ascending distinct ids, then zero padding
        assert hist[r][:len(items)].tolist() == items and not hist[r][len(items):].any()
    assert hist.shape == (len(uids), max(1, width)) and hist.dtype == np.int32
    # negatives' feature table = fill_missing_feat(item_feat_dict[str(i)])
    for i in (1, 17, 99):
        d = ds.item_feat_dict[str(i)]
        from tencent_recommendation_2025_amd.dataset import ITEM_SPARSE
        assert [int(st.item_sparse[i, c]) for c in range(len(ITEM_SPARSE))] == [d.get(k, 0) for k in ITEM_SPARSE]
    assert st.item_ok[0] == 0 and st.item_ok[1:].all()


def test_store_batches_dataloader(tmp_path):
    """StoreBatches through a 2-worker DataLoader: every user once per epoch, each
    batch equal to SeqStore.batch of its uids; set_epoch reshuffles."""
    from tencent_recommendation_2025_amd.dataset import write_synthetic_tencentgr
    from tencent_recommendation_2025_amd.seqstore import SeqStore, StoreBatches
    write_synthetic_tencentgr(tmp_path, num_users=70, num_items=200, max_events=40, seed=6)
    st = SeqStore(tmp_path, maxlen=15)
    sb = StoreBatches(st, 16, seed=1, drop_last=False)
    dl = torch.utils.data.DataLoader(sb, batch_size=None, num_workers=2)
    seen = []
    for uids, b in dl:
        ref = st.batch(uids.numpy())
        assert all(torch.equal(x, y) for x, y in zip(b[:6], ref[:6]))
        assert all(torch.equal(b[6][k], ref[6][k]) for k in ref[6])
        seen += uids.tolist()
    assert sorted(seen) == list(range(70))
    first = sb.perm.copy()
    sb.set_epoch(1)
    assert not np.array_equal(first, sb.perm)


def test_store_pickles_as_its_path(tmp_path):
    """A SeqStore crosses into spawned DataLoader workers as its cache path (the
    memory-mapped blocks are mapped again there, not copied into the pickle), and
    the unpickled store assembles the same batches; a spawn-context loader too."""
    import pickle
    from tencent_recommendation_2025_amd.dataset import write_synthetic_tencentgr
    from tencent_recommendation_2025_amd.seqstore import SeqStore, StoreBatches
    write_synthetic_tencentgr(tmp_path, num_users=60, num_items=200, max_events=40, seed=8)
    st = SeqStore(tmp_path, maxlen=15)
    blob = pickle.dumps(st)
    assert len(blob) < 4096 < st.sparse.nbytes + st.arr.nbytes
    st2 = pickle.loads(blob)
    uids = np.arange(0, 60, 3)
    a, b = st.batch(uids), st2.batch(uids)
    assert all(torch.equal(x, y) for x, y in zip(a[:6], b[:6]))
    assert all(torch.equal(a[j][k], b[j][k]) for j in (6, 7) for k in a[j])
    dl = torch.utils.data.DataLoader(StoreBatches(st, 20, seed=2), batch_size=None, num_workers=1,
                                     multiprocessing_context='spawn')
    for u, bb in dl:
        ref = st.batch(u.numpy())
        assert all(torch.equal(x, y) for x, y in zip(bb[:6], ref[:6]))


@pytest.mark.parametrize('maxlen', [20, 60])
def test_store_timestamps_match_dataset(tmp_path, maxlen):
    """Event times (the HSTU time-bias input; the reference loader reads and drops
    them, model/BaseLine/dataset.py:117): SeqStore.batch(timestamps=True)'s tenth
    field == MyDataset(args.timestamps)'s, and each position carries its own
    record's time (user token: the user record's; padding: 0)."""
    import json
    from tencent_recommendation_2025_amd.dataset import MyDataset, write_synthetic_tencentgr
    from tencent_recommendation_2025_amd.seqstore import SeqStore
    write_synthetic_tencentgr(tmp_path, num_users=80, num_items=300, max_events=90, seed=4)
    ds = MyDataset(tmp_path, SimpleNamespace(maxlen=maxlen, mm_emb_id=['81'], timestamps=True))
    st = SeqStore(tmp_path, maxlen=maxlen)
    uids = np.arange(80)
    np.random.seed(1)
    want = ds.collate_tensor_fn([ds[int(u)] for u in uids])
    got = st.batch(uids, timestamps=True)
    assert len(got) == len(want) == 10
    assert got[9].dtype == want[9].dtype == torch.int64 and torch.equal(got[9], want[9])
    for i in (0, 1, 3, 4, 5):
        assert torch.equal(got[i], want[i]), i
    # direct: rebuild each user's token order from seq.jsonl
    T = maxlen + 1
    with open(tmp_path / 'seq.jsonl') as f:
        lines = [json.loads(x) for x in f]
    for u in uids:
        toks = []
        for uu, i, uf, itf, _a, when in lines[u]:
            if uu and uf:
                toks.insert(0, (uu, when))
            if i and itf:
                toks.append((i, when))
        body = toks[:-1][-T:]
        exp = np.zeros(T, np.int64)
        exp[T - len(body):] = [w for _, w in body]
        assert np.array_equal(got[9][u].numpy(), exp), u
        assert np.array_equal(got[0][u].numpy()[T - len(body):], [t for t, _ in body])
    # the default batch keeps the reference's nine fields
    assert len(st.batch(uids[:4])) == 9 and len(MyDataset(tmp_path, SimpleNamespace(maxlen=maxlen))[0]) == 9


def _store_view(sparse, arr, arr_len, mm):
    from tencent_recommendation_2025_amd import _lib as L
    return L.GrkStoreView(sparse.ctypes.data, arr.ctypes.data, arr_len.ctypes.data, mm.ctypes.data, len(sparse),
                          sparse.shape[1], arr.shape[1], arr.shape[2], mm.shape[1])


def test_store_features_entry_points_restated():
    """grk_store_features / grk_store_array_widths (host code, include/grk.h) on a random
    store against a numpy restatement: unselected positions take the defaults (id 0,
    array [0] padded with 0, mm row 0), arrays are cut at each length and padded to the
    requested width, widths are the selected tokens' longest arrays (>= 1); a selected
    token or a stored mm row out of range is refused before anything is written."""
    import ctypes as C
    from tencent_recommendation_2025_amd import _lib as L
    rng = np.random.default_rng(3)
    n_tok, Fs, Fa, cap, Fm, mm_rows, W = 500, 5, 3, 6, 2, 40, 8
    sparse = rng.integers(0, 1000, (n_tok, Fs)).astype(np.int32)
    arr_len = rng.integers(1, cap + 1, (n_tok, Fa)).astype(np.int32)
    arr = rng.integers(1, 99, (n_tok, Fa, cap)).astype(np.int32)     # values past each length must not leak
    mm = rng.integers(0, mm_rows, (n_tok, Fm)).astype(np.int32)
    tab = rng.standard_normal((mm_rows, W)).astype(np.float32)
    tab[0] = 0
    view = _store_view(sparse, arr, arr_len, mm)
    n = 300
    tok = rng.integers(0, n_tok, n).astype(np.int64)
    sel = (rng.random(n) < 0.7).astype(np.uint8)
    tok[sel == 0] = -5                                               # ignored where unselected
    widths = np.zeros(Fa, np.int32)
    lib = L.lib()
    L.check(lib.grk_store_array_widths(C.byref(view), tok.ctypes.data, sel.ctypes.data, n, widths.ctypes.data), 'w')
    on = sel.astype(bool)
    assert widths.tolist() == [max(1, int(arr_len[tok[on], c].max())) for c in range(Fa)]
    outs = [np.full(n, -1, np.int64), np.full((n, 4), -1, np.int64), np.full((n, W), -1, np.float32)]
    cols = (L.GrkStoreCol * 3)(L.GrkStoreCol(L.STORE_SPARSE, 3, 1, 0, 0, None, outs[0].ctypes.data),
                               L.GrkStoreCol(L.STORE_ARRAY, 1, 4, 0, 0, None, outs[1].ctypes.data),
                               L.GrkStoreCol(L.STORE_MM, 1, W, 0, mm_rows, tab.ctypes.data, outs[2].ctypes.data))
    L.check(lib.grk_store_features(C.byref(view), tok.ctypes.data, sel.ctypes.data, n, cols, 3), 'f')
    t = np.where(on, tok, 0)
    assert np.array_equal(outs[0], np.where(on, sparse[t, 3], 0))
    keep = on[:, None] & (np.arange(4)[None, :] < arr_len[t, 1][:, None])
    assert np.array_equal(outs[1], np.where(keep, arr[t, 1, :4], 0))
    assert np.array_equal(outs[2], tab[np.where(on, mm[t, 1], 0)])
    # refused inputs leave the outputs untouched
    before = [o.copy() for o in outs]
    bad = tok.copy()
    bad[np.flatnonzero(on)[0]] = n_tok
    assert lib.grk_store_features(C.byref(view), bad.ctypes.data, sel.ctypes.data, n, cols, 3) == L.GRK_EINVAL
    assert b'outside the store' in lib.grk_last_error()
    mm_bad = mm.copy()
    mm_bad[tok[on][0], 1] = mm_rows
    view_bad = _store_view(sparse, arr, arr_len, mm_bad)
    assert lib.grk_store_features(C.byref(view_bad), tok.ctypes.data, sel.ctypes.data, n, cols, 3) == L.GRK_EINVAL
    cols[1].width = cap + 1
    assert lib.grk_store_features(C.byref(view), tok.ctypes.data, sel.ctypes.data, n, cols, 3) == L.GRK_EINVAL
    assert all(np.array_equal(a, b) for a, b in zip(outs, before))
