"""CPU checks of the RQ-VAE oracle (oracle/rqvae.py): the code search's
definition (fixed-order fp32 distances, lowest index on ties, residual chain),
the loss restatement and the k-means initialiser.  The reference has no
tokenizer, so these pin the oracle by construction (parity unpinned as a
model); the HIP kernel is then held bit-exact to it (tests/test_gpu_rqvae.py)."""
import numpy as np

from oracle import rqvae as orq


def _brute(z, cb):
    """Scalar restatement of one level-by-level search, pure Python loops."""
    n, d = z.shape
    L, K, _ = cb.shape
    codes = np.zeros((n, L), np.int32)
    for i in range(n):
        r = z[i].astype(np.float32).copy()
        for lvl in range(L):
            best, bk = np.float32(np.inf), 0
            for k in range(K):
                acc = np.float32(0)
                for j in range(d):
                    t = np.float32(r[j] - cb[lvl, k, j])
                    acc = np.float32(acc + np.float32(t * t))
                if acc < best:
                    best, bk = acc, k
            codes[i, lvl] = bk
            r = (r - cb[lvl, bk]).astype(np.float32)
    return codes


def test_assign_matches_scalar_restatement():
    rng = np.random.default_rng(0)
    z = rng.standard_normal((9, 16)).astype(np.float32)
    cb = rng.standard_normal((3, 11, 16)).astype(np.float32)
    codes, quant, dist, resid = orq.rq_assign(z, cb)
    assert np.array_equal(codes, _brute(z, cb))
    want_q = cb[0][codes[:, 0]] + cb[1][codes[:, 1]] + cb[2][codes[:, 2]]
    assert np.array_equal(quant, want_q)
    r = z.copy()
    for lvl in range(3):
        r = r - cb[lvl][codes[:, lvl]]
    assert np.array_equal(resid, r)
    assert (dist >= 0).all()


def test_ties_take_lowest_code():
    rng = np.random.default_rng(1)
    cb = rng.standard_normal((2, 8, 16)).astype(np.float32)
    cb[0, 5] = cb[0, 2]          # duplicated codewords: code 2 must win
    cb[1, 7] = cb[1, 0]
    z = np.concatenate([cb[0, 2:3] + 1e-3, cb[0, 5:6]]).astype(np.float32)
    codes = orq.rq_assign(z, cb)[0]
    assert (codes[:, 0] == 2).all()
    assert not (codes[:, 1] == 7).any()


def test_codeword_rows_quantise_exactly():
    rng = np.random.default_rng(2)
    cb = rng.standard_normal((1, 32, 32)).astype(np.float32)
    idx = rng.integers(0, 32, 50)
    codes, _, dist, resid = orq.rq_assign(cb[0][idx], cb)
    assert np.array_equal(codes[:, 0], idx)
    assert (dist == 0).all() and (resid == 0).all()


def test_loss_and_forward_consistent():
    rng = np.random.default_rng(3)
    x = rng.standard_normal((20, 24))
    enc = [(rng.standard_normal((32, 24)) * 0.2, rng.standard_normal(32) * 0.1),
           (rng.standard_normal((16, 32)) * 0.2, np.zeros(16))]
    dec = [(rng.standard_normal((32, 16)) * 0.2, np.zeros(32)), (rng.standard_normal((24, 32)) * 0.2, np.zeros(24))]
    cb = rng.standard_normal((2, 8, 16)).astype(np.float32) * 0.5
    loss, recon, rql, codes, x_hat = orq.rqvae_forward(x, enc, cb, dec, beta=0.25)
    assert np.isclose(loss, recon + rql)
    z = orq.mlp(x, enc)
    r = z.copy()
    want = 0.0
    for lvl in range(2):
        c = cb[lvl][codes[:, lvl]].astype(np.float64)
        want += 1.25 * np.mean((r - c) ** 2)
        r = r - c
    assert np.isclose(rql, want)
    assert x_hat.shape == x.shape


def test_kmeans_init_recovers_clusters():
    rng = np.random.default_rng(4)
    centres = rng.standard_normal((8, 16)).astype(np.float32) * 10
    z = (centres[rng.integers(0, 8, 800)] + rng.standard_normal((800, 16)) * 0.01).astype(np.float32)
    cent = orq.kmeans_init(z, 8, iters=10, seed=0)
    d = ((cent[:, None] - centres[None]) ** 2).sum(-1)
    assert d.min(1).max() < 0.1 or len(set(d.argmin(1))) < 8   # converged or a seeded local optimum
    assert orq.semantic_feature_ids(np.array([[0, 255]]), 256).tolist() == [[1, 256]]


def test_semantic_id_features_in_synthetic_batches():
    """Host logic of config 4's data path (CPU tensors): 1-based id table, the
    schema entries and the per-token sid features of seq / pos / neg."""
    import torch
    from tencent_recommendation_2025_amd import synthetic as S
    from tencent_recommendation_2025_amd.rqvae import semantic_id_schema, semantic_id_table
    codes = torch.randint(0, 16, (50, 2), dtype=torch.int32, generator=torch.Generator().manual_seed(0))
    sid = semantic_id_table(codes, 50)
    assert sid.shape == (51, 2) and int(sid[0].abs().sum()) == 0 and torch.equal(sid[1:], codes.long() + 1)
    names, stats = semantic_id_schema(2, 16)
    assert names == ['sid0', 'sid1'] and stats == {'sid0': 16, 'sid1': 16}
    cfg = S.SyntheticConfig(batch_size=3, maxlen=10, num_items=50, num_users=7, min_len=3, sid_table=sid, sid_codes=16)
    st, types = S.feature_schema(cfg)
    assert types['item_sparse'][-2:] == names and st['sid1'] == 16
    seq, pos, neg, tt, _, _, sf, pf, nf = S.make_batch(cfg, torch.Generator().manual_seed(1), 'cpu')
    item = torch.where(tt == 1, seq, 0)
    for lvl in range(2):
        assert torch.equal(sf[f'sid{lvl}'], torch.where(item > 0, sid[item, lvl], 0))
        assert torch.equal(pf[f'sid{lvl}'], torch.where(pos > 0, sid[pos, lvl], 0))
        assert torch.equal(nf[f'sid{lvl}'], torch.where(neg > 0, sid[neg, lvl], 0))


def test_dedup_level_matches_oracle():
    """The collision level (rqvae.dedup_level, torch ops -- here on CPU tensors)
    equals the oracle's item-order walk; every extended tuple is unique."""
    import torch
    from tencent_recommendation_2025_amd.rqvae import dedup_level
    rng = np.random.default_rng(5)
    for n, lv, k in ((1, 3, 4), (200, 2, 3), (1000, 3, 4), (500, 1, 2)):
        codes = rng.integers(0, k, (n, lv)).astype(np.int32)
        got = dedup_level(torch.from_numpy(codes)).numpy()
        want = orq.dedup_level(codes)
        assert np.array_equal(got, want)
        assert len({tuple(r) for r in got}) == n
    assert dedup_level(torch.zeros(0, 3, dtype=torch.int32)).shape == (0, 4)


def test_semantic_id_schema_covers_collision_level():
    """dedup_level's extra level can exceed the codebook size (a collision group
    larger than K): the schema built from the codes sizes every level's table so
    each 1-based id of semantic_id_table has a row."""
    import torch
    from tencent_recommendation_2025_amd.rqvae import dedup_level, semantic_id_schema, semantic_id_table
    codes = torch.zeros(40, 2, dtype=torch.int32)      # every item shares one tuple: collision group of 40
    codes[::2, 1] = 1
    ext = dedup_level(codes)
    names, stats = semantic_id_schema(ext.shape[1], 4, codes=ext)
    assert names == ['sid0', 'sid1', 'sid2']
    assert stats['sid0'] == 4 and stats['sid1'] == 4 and stats['sid2'] == int(ext[:, 2].max()) + 1 == 20
    tab = semantic_id_table(ext, 40)
    for lvl, k in enumerate(names):
        emb = torch.nn.Embedding(stats[k] + 1, 8, padding_idx=0)   # the O1 table of that feature
        assert int(tab[:, lvl].max()) < emb.num_embeddings
        emb(tab[:, lvl])                                           # every id has a row
