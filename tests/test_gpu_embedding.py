"""GPU parity of the embedding kernels (grk_embedding_gather / _backward,
grk_table_adamw) against the oracle, which is itself pinned to the reference's
golden vectors (tests/test_oracle_golden.py).  Integer/byte work is checked
bit-exact; the fp32 order-defined sums too."""

import numpy as np
import pytest
import torch

from oracle import adamw as oadam
from oracle import embedding as oemb

pytestmark = pytest.mark.gpu
DEV = 'cuda'


@pytest.fixture(scope='module')
def K():
    from tencent_recommendation_2025_amd import _lib, kernels
    _lib.lib()
    return kernels


def T(x, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(x)).to(DEV)
    return t if dtype is None else t.to(dtype)


def gather1(K, table, idx, bag=1, mode=0, token_type=None, seq_len=0, dtype=torch.float32):
    D = table.shape[1]
    n = idx.numel() // bag
    out = torch.full((n, D), float('nan'), dtype=dtype, device=DEV)
    K.embedding_gather([K.Lookup(table, idx, 0, mode, bag)], out, n, token_type, seq_len)
    torch.cuda.synchronize()
    return out


def test_gather_golden_bitexact(K, golden):
    g = golden('emb_ops.npz')
    table = T(g['table'])
    out = gather1(K, table, T(g['idx']))
    assert np.array_equal(out.cpu().numpy().reshape(g['out'].shape), g['out'])
    out32 = gather1(K, table, T(g['idx']).int())
    assert torch.equal(out32, out)


def test_bag_sum_golden_bitexact(K, golden):
    g = golden('emb_ops.npz')
    out = gather1(K, T(g['table']), T(g['idx_arr']), bag=4)
    assert np.array_equal(out.cpu().numpy().reshape(g['bag'].shape), g['bag'])


def test_backward_golden_bitexact(K, golden):
    g = golden('emb_ops.npz')
    D = g['table'].shape[1]
    res = K.embedding_backward([K.GradSource(T(g['idx']), T(g['gout']).reshape(-1, D), 0)], 1001, D)
    assert np.array_equal(res.dense.cpu().numpy(), g['dgrad'])
    res = K.embedding_backward([K.GradSource(T(g['idx_arr']), T(g['gbag']).reshape(-1, D), 0, bag=4)], 1001, D)
    assert np.array_equal(res.dense.cpu().numpy(), g['dgrad_bag'])


def test_backward_multi_source(K, golden):
    g = golden('emb_ops.npz')
    D = 64
    src = [K.GradSource(T(g['item_idx'][i]), T(g['item_gout'][i]).reshape(-1, D), 0) for i in range(3)]
    res = K.embedding_backward(src, 1001, D)
    want = oemb.multi_source_backward([(g['item_gout'][i], g['item_idx'][i]) for i in range(3)], 1001)
    assert np.array_equal(res.dense.cpu().numpy(), want)
    # vs the reference's autograd (sums three dense grads): equal to rounding
    np.testing.assert_allclose(res.dense.cpu().numpy(), g['item_dgrad'], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize('D', [128, 512])   # 512: the wave-per-row gather (64 x 16-byte chunks)
def test_bf16_gather_bagsum_backward(K, D):
    rng = np.random.default_rng(0)
    R, N, A = 5000, 777, 3
    tab = oemb.to_bf16_f32(rng.standard_normal((R, D)).astype(np.float32))
    idx = rng.integers(0, R, (N,))
    idx[:50] = 0
    arr = rng.integers(0, R, (N, A))
    tb = T(tab).to(torch.bfloat16)
    out = gather1(K, tb, T(idx), dtype=torch.bfloat16)
    assert np.array_equal(out.float().cpu().numpy(), oemb.gather(tab, idx))
    out = gather1(K, tb, T(arr), bag=A, dtype=torch.bfloat16)
    assert np.array_equal(out.float().cpu().numpy(), oemb.bag_sum(tab, arr, out_bf16=True))
    gr = oemb.to_bf16_f32(rng.standard_normal((N, D)).astype(np.float32))
    res = K.embedding_backward([K.GradSource(T(arr), T(gr).to(torch.bfloat16), 0, bag=A)], R, D)
    want = oemb.dense_backward(np.repeat(gr[:, None, :], A, axis=1), arr, R)
    assert np.array_equal(res.dense.cpu().numpy(), want)


@pytest.mark.parametrize('D', [64, 256])    # fp32 256: the wave-per-row gather
def test_index_modes_and_fused_features(K, D):
    rng = np.random.default_rng(1)
    B, Tn = 6, 17
    item = rng.standard_normal((300, D)).astype(np.float32)
    user = rng.standard_normal((50, D)).astype(np.float32)
    pos = rng.standard_normal((2 * 16 + 1, D)).astype(np.float32)
    sp = rng.standard_normal((20, D)).astype(np.float32)
    seq = np.zeros((B, Tn), np.int64)
    tt = np.zeros((B, Tn), np.int32)
    for b in range(B):
        n = int(rng.integers(1, Tn + 1))
        seq[b, Tn - n] = rng.integers(1, 50)
        tt[b, Tn - n] = 2
        seq[b, Tn - n + 1:] = rng.integers(1, 300, n - 1)
        tt[b, Tn - n + 1:] = 1
    f = rng.integers(0, 20, (B, Tn))
    arr = rng.integers(0, 20, (B, Tn, 3))
    out = torch.full((B * Tn, 5 * D + 8), -7.0, device=DEV)
    ttd = T(tt)
    lk = [K.Lookup(T(item), T(seq), 0, 1), K.Lookup(T(user), T(seq), D, 2), K.Lookup(T(pos), T(seq), 2 * D, 3),
          K.Lookup(T(sp), T(f), 3 * D), K.Lookup(T(sp), T(arr), 4 * D, bag=3)]
    K.embedding_gather(lk, out, B * Tn, ttd, Tn)
    o = out.cpu().numpy().reshape(B, Tn, -1)
    posidx = np.arange(1, Tn + 1)[None, :] * (seq != 0)
    assert np.array_equal(o[..., :D], item[(tt == 1) * seq])
    assert np.array_equal(o[..., D:2 * D], user[(tt == 2) * seq])
    assert np.array_equal(o[..., 2 * D:3 * D], pos[posidx])
    assert np.array_equal(o[..., 3 * D:4 * D], sp[f])
    assert np.array_equal(o[..., 4 * D:5 * D], oemb.bag_sum(sp, arr))
    assert np.all(o[..., 5 * D:] == -7.0)  # columns outside every feature untouched
    # backward through the masked / positional modes
    gout = rng.standard_normal((B * Tn, 5 * D)).astype(np.float32)
    gd = T(gout)
    res = K.embedding_backward([K.GradSource(T(seq), gd, 0, 1)], 300, D, token_type=ttd, seq_len=Tn)
    assert np.array_equal(res.dense.cpu().numpy(), oemb.dense_backward(gout[:, :D], ((tt == 1) * seq), 300))
    res = K.embedding_backward([K.GradSource(T(seq), gd, 2 * D, 3)], 33, D, token_type=ttd, seq_len=Tn)
    assert np.array_equal(res.dense.cpu().numpy(), oemb.dense_backward(gout[:, 2 * D:3 * D], posidx, 33))


def test_sparse_output_row_slot_and_adamw(K):
    rng = np.random.default_rng(2)
    R, D, N = 2000, 64, 3000
    idx = rng.integers(0, R, (N,))
    idx[rng.random(N) < 0.3] = 7  # hot row
    gr = rng.standard_normal((N, D)).astype(np.float32)
    slot = torch.full((R,), -1, dtype=torch.int32, device=DEV)
    res = K.embedding_backward([K.GradSource(T(idx), T(gr), 0)], R, D, dense=True, sparse=True, row_slot=slot)
    cnt = int(res.count.item())
    uniq = oemb.unique_rows(idx)
    assert cnt == len(uniq)
    assert np.array_equal(res.ids[:cnt].cpu().numpy(), uniq)
    dense = oemb.dense_backward(gr, idx, R)
    got_rows = res.rows[:cnt].cpu().numpy()
    cold = uniq != 7
    # every row, the ~900-occurrence hot row included (k_seg_hot: one sequential fp32
    # chain per column in occurrence order), equals the reference's CPU order bit for bit
    assert np.array_equal(got_rows, dense[uniq])
    s = slot.cpu().numpy()
    assert np.array_equal(s[uniq], np.arange(cnt)) and np.all(np.delete(s, uniq) == -1)
    p0 = rng.standard_normal((R, D)).astype(np.float32)
    m0 = rng.standard_normal((R, D)).astype(np.float32) * 0.01
    v0 = np.abs(rng.standard_normal((R, D)).astype(np.float32)) * 0.01
    for lazy in (False, True):
        p, m, v = T(p0), T(m0), T(v0)
        slot2 = slot.clone()
        hp = K.adamw_hparams(1e-3, 0.9, 0.98, 1e-8, 0.01, 3)
        K.table_adamw(p, m, v, hp, res.ids, res.rows, res.count, res.capacity, None if lazy else slot2, lazy=lazy)
        fn = oadam.lazy_rows if lazy else oadam.dense_rows
        wp, wm, wv = fn(p0, m0, v0, uniq, got_rows, 3, 1e-3, 0.9, 0.98, 1e-8, 0.01)
        np.testing.assert_allclose(p.cpu().numpy(), wp, rtol=2e-6, atol=1e-7)
        np.testing.assert_allclose(m.cpu().numpy(), wm, rtol=2e-6, atol=1e-8)
        np.testing.assert_allclose(v.cpu().numpy(), wv, rtol=2e-6, atol=1e-10)
        if not lazy:
            assert torch.all(slot2 == -1)


def test_adamw_bf16_param(K):
    rng = np.random.default_rng(3)
    R, D = 300, 32
    p0 = oemb.to_bf16_f32(rng.standard_normal((R, D)).astype(np.float32))
    ids = np.arange(0, R, 3)
    g = rng.standard_normal((len(ids), D)).astype(np.float32)
    p = T(p0).to(torch.bfloat16)
    m = torch.zeros(R, D, device=DEV); v = torch.zeros(R, D, device=DEV)
    slot = torch.full((R,), -1, dtype=torch.int32, device=DEV)
    slot[T(ids)] = torch.arange(len(ids), dtype=torch.int32, device=DEV)
    K.table_adamw(p, m, v, K.adamw_hparams(1e-2, 0.9, 0.98, 1e-8, 0.01, 1), T(ids), T(g),
                  torch.tensor([len(ids)], dtype=torch.int32, device=DEV), len(ids), slot)
    wp, _, _ = oadam.dense_rows(p0, np.zeros((R, D), np.float32), np.zeros((R, D), np.float32), ids, g, 1, 1e-2)
    got = p.float().cpu().numpy()
    # fp32 math then one RNE rounding: equal to the rounded oracle up to 1 bf16 ulp (fma contraction)
    np.testing.assert_allclose(got, oemb.to_bf16_f32(wp), rtol=2 ** -7, atol=1e-30)
    assert np.mean(got == oemb.to_bf16_f32(wp)) > 0.99


@pytest.mark.parametrize('D,dt,bulk', [(256, torch.float32, 20000), (512, torch.bfloat16, 20000),
                                       (512, torch.float32, 20000), (64, torch.bfloat16, 20000),
                                       (40, torch.float32, 20000), (520, torch.bfloat16, 20000),
                                       (512, torch.bfloat16, 160000), (256, torch.float32, 160000)])
def test_backward_wave_path(K, D, dt, bulk):
    """Every row bit-exact in occurrence order (the reference's CPU
    embedding_dense_backward): rows inside one chunk, rows crossing chunk
    edges (re-summed up to 2 chunks), and hot rows of 600-3000 occurrences
    (k_seg_hot, one wave per column slice; D = 40 and 520 leave a partial
    column slice) -- on the one-wave-per-row path (D = 64 x 16 bytes; 64-entry
    chunks below 2^17 occurrences, 256 above: `bulk`) and the generic one;
    padding skipped; deterministic."""
    rng = np.random.default_rng(11)
    R = 3000
    idx = np.concatenate([np.full(3000, 5), np.full(600, 7), np.full(1031, 8),
                          np.repeat(np.arange(10, 20), rng.integers(300, 513, 10)),
                          np.repeat(np.arange(20, 30), rng.integers(60, 129, 10)),
                          rng.integers(30, R, bulk), np.zeros(2000, np.int64)])
    rng.shuffle(idx)
    g = rng.standard_normal((len(idx), D)).astype(np.float32)
    if dt == torch.bfloat16:
        g = oemb.to_bf16_f32(g)
    src = [K.GradSource(T(idx), T(g).to(dt), 0)]
    res = K.embedding_backward(src, R, D, dense=True, sparse=True)
    want = oemb.dense_backward(g, idx, R)
    got = res.dense.cpu().numpy()
    counts = np.bincount(idx, minlength=R)
    assert counts[10:20].min() >= 300 and counts[5] == 3000 and counts[8] == 1031
    assert np.array_equal(got, want)
    cnt = int(res.count.item())
    uniq = oemb.unique_rows(idx)
    assert cnt == len(uniq) and np.array_equal(res.ids[:cnt].cpu().numpy(), uniq)
    assert np.array_equal(res.rows[:cnt].cpu().numpy(), got[uniq])
    again = K.embedding_backward(src, R, D, dense=True).dense
    assert torch.equal(again, res.dense)


@pytest.mark.parametrize('D', [16, 256])
def test_out_of_range_flag_and_empty(K, D):
    table = torch.randn(10, D, device=DEV)
    idx = torch.tensor([1, 2, 10, -1], device=DEV)
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    out = torch.full((4, D), 5.0, device=DEV)
    K.embedding_gather([K.Lookup(table, idx, 0)], out, 4, err_flag=err)
    assert err.item() == 1
    assert torch.all(out[2:] == 0) and torch.equal(out[:2], table[1:3])
    empty = torch.empty(0, D, device=DEV)
    K.embedding_gather([K.Lookup(table, idx[:0], 0)], empty, 0)
    res = K.embedding_backward([K.GradSource(idx[:0], empty, 0)], 10, D)
    assert res.count.item() == 0 and torch.all(res.dense == 0)


def test_full_size_c2_properties(K):
    """BASELINE config 2 sizes: 1M x 512 bf16 item table, B=128, T=201, 16 lookups."""
    g = torch.Generator(device=DEV).manual_seed(0)
    R, D, B, Tn = 1_000_001, 512, 128, 201
    N = B * Tn
    table = torch.randn(R, D, device=DEV, generator=g).to(torch.bfloat16)
    idx = torch.randint(0, R, (16, N), device=DEV, generator=g)
    out = torch.empty(N, 16 * D, dtype=torch.bfloat16, device=DEV)
    K.embedding_gather([K.Lookup(table, idx[f], f * D) for f in range(16)], out, N)
    sel = torch.randint(0, N, (2048,), device=DEV, generator=g)
    want = table.float().cpu().numpy()[idx[:, sel].cpu().numpy()]          # [16, S, D]
    got = out[sel].float().cpu().numpy().reshape(len(sel), 16, D).transpose(1, 0, 2)
    assert np.array_equal(got, want)
    # backward: three sources on one table; checksum of the dense grad == sum of all grad rows
    grad = torch.randn(N, 3 * D, device=DEV, generator=g).to(torch.bfloat16)
    src = [K.GradSource(idx[f], grad, f * D) for f in range(3)]
    res = K.embedding_backward(src, R, D, padding_idx=None, dense=True, sparse=True)
    total = res.dense.double().sum(0)
    want_total = grad.double().reshape(N, 3, D).sum((0, 1))
    torch.testing.assert_close(total, want_total, rtol=1e-6, atol=1e-3)
    cnt = int(res.count.item())
    assert cnt == torch.unique(idx[:3]).numel()
    ids = res.ids[:cnt]
    assert torch.all(ids[1:] > ids[:-1])


def test_hot_rows_bit_exact(K):
    """Rows with thousands of occurrences (cardinality-10 feature tables, two
    lookups of one group): bit-exact in occurrence order, as the reference."""
    rng = np.random.default_rng(4)
    R, D, N = 12, 128, 40000
    idx = rng.integers(1, R, (N,))
    idx[:300] = 3                                      # a 300-occurrence row crossing chunk boundaries
    gr = oemb.to_bf16_f32(rng.standard_normal((N, 2 * D)).astype(np.float32))
    g = T(gr).to(torch.bfloat16)
    src = [K.GradSource(T(idx), g, 0), K.GradSource(T(idx[::-1].copy()), g, D)]
    a = K.embedding_backward(src, R, D, dense=True)
    b = K.embedding_backward(src, R, D, dense=True)
    assert torch.equal(a.dense, b.dense)
    want = oemb.dense_backward(np.concatenate([gr[:, :D], gr[:, D:]]), np.concatenate([idx, idx[::-1]]), R)
    assert np.array_equal(a.dense.cpu().numpy(), want)


@pytest.mark.parametrize('D,dt', [(512, torch.bfloat16), (256, torch.float32), (512, torch.float32)])
def test_backward_chunked_mode(K, D, dt):
    """GRK_BWD_CHUNKED (projected feature rows of the fused trainer): rows
    inside one chunk bit-exact in occurrence order as before, rows spanning
    chunks equal to the oracle's chunk-order restatement bit for bit (hot rows
    of 600-30000 occurrences, rows of <= 512 crossing one edge, a row filling
    whole chunks); within fp32 rounding of the occurrence-order sums;
    deterministic; row-sparse outputs and row_slot consistent."""
    rng = np.random.default_rng(5)
    R = 3000
    idx = np.concatenate([np.full(30000, 5), np.full(600, 7), np.full(1031, 8), np.full(256, 9),
                          np.repeat(np.arange(10, 20), rng.integers(300, 513, 10)),
                          rng.integers(20, R, 20000), np.zeros(2000, np.int64)])
    rng.shuffle(idx)
    g = rng.standard_normal((len(idx), 2 * D)).astype(np.float32)
    if dt == torch.bfloat16:
        g = oemb.to_bf16_f32(g)
    gt = T(g).to(dt)
    rev = idx[::-1].copy()
    src = [K.GradSource(T(idx), gt, 0), K.GradSource(T(rev), gt, D)]
    slot = torch.full((R,), -1, dtype=torch.int32, device=DEV)
    res = K.embedding_backward(src, R, D, dense=True, sparse=True, chunked=True, row_slot=slot)
    gg = np.concatenate([g[:, :D], g[:, D:]])
    ii = np.concatenate([idx, rev])
    got = res.dense.cpu().numpy()
    assert np.array_equal(got, oemb.chunked_backward(gg, ii, R, chunk=K.chunked_size()))
    exact = oemb.dense_backward(gg, ii, R)
    np.testing.assert_allclose(got, exact, rtol=1e-4, atol=1e-3)
    counts = np.bincount(ii, minlength=R)
    small = (counts > 0) & (counts <= 20)
    small[0] = False
    assert small.sum() > 1000
    # rows of a handful of occurrences sit in one chunk unless they straddle an edge
    assert np.mean(np.all(got[small] == exact[small], axis=1)) > min(0.9, 1 - 12 / K.chunked_size())
    cnt = int(res.count.item())
    uniq = oemb.unique_rows(ii)
    assert cnt == len(uniq) and np.array_equal(res.ids[:cnt].cpu().numpy(), uniq)
    assert np.array_equal(res.rows[:cnt].cpu().numpy(), got[uniq])
    s = slot.cpu().numpy()
    assert np.array_equal(s[uniq], np.arange(cnt)) and np.all(np.delete(s, uniq) == -1)
    again = K.embedding_backward(src, R, D, dense=True, chunked=True).dense
    assert torch.equal(again, res.dense)


@pytest.mark.parametrize('n,R', [(1, 4), (200, 50), (8192 + 77, 900), (140000, 41952)])
def test_backward_chunked_dense_only_column_sliced(K, n, R):
    """The dense-only chunked call at d = 512 with bf16 gradient rows (the projected
    feature rows' backward) runs k_seg_chunks_cols: per XCD one 64-column slice, 8
    chunks per wave.  Bit-exact against the oracle's chunk-order restatement, in fp32
    and as the bf16 rounding of it; sizes from one occurrence to a partial last group
    of chunks and a C2-like spread (hot rows, rows crossing chunk edges, row 0)."""
    rng = np.random.default_rng(n)
    D = 512
    if n < 1000:
        idx = rng.integers(0, R, n)
    else:
        idx = np.concatenate([np.full(n // 7, 3), np.repeat(np.arange(10, 30), 300),
                              rng.integers(0, R, n - n // 7 - 6000)])
        rng.shuffle(idx)
    g = oemb.to_bf16_f32(rng.standard_normal((len(idx), D)).astype(np.float32))
    src = [K.GradSource(T(idx), T(g).to(torch.bfloat16), 0)]
    want = oemb.chunked_backward(g, idx, R, chunk=K.chunked_size())
    got = K.embedding_backward(src, R, D, dense=True, chunked=True).dense
    assert np.array_equal(got.cpu().numpy(), want)
    got16 = K.embedding_backward(src, R, D, dense=True, chunked=True, dense_dtype=torch.bfloat16).dense
    assert torch.equal(got16, T(want).to(torch.bfloat16))


def test_backward_chunked_bf16_dense_is_the_rounded_fp32_result(K):
    """GRK_BWD_DENSE_BF16: the dense rows are the chunked fp32 result rounded
    to bf16 once (round to nearest even, as torch's cast) -- bit-exact against
    the fp32 call; untouched rows zero; row-sparse outputs stay fp32 and equal."""
    rng = np.random.default_rng(6)
    R, D = 3000, 512
    idx = np.concatenate([np.full(9000, 5), np.repeat(np.arange(10, 20), rng.integers(300, 513, 10)),
                          rng.integers(20, R, 12000), np.zeros(500, np.int64)])
    rng.shuffle(idx)
    gt = T(oemb.to_bf16_f32(rng.standard_normal((len(idx), D)).astype(np.float32))).to(torch.bfloat16)
    src = [K.GradSource(T(idx), gt, 0)]
    ref = K.embedding_backward(src, R, D, dense=True, sparse=True, chunked=True)
    got = K.embedding_backward(src, R, D, dense=True, sparse=True, chunked=True, dense_dtype=torch.bfloat16)
    assert got.dense.dtype == torch.bfloat16 and got.dense.shape == (R, D)
    assert torch.equal(got.dense, ref.dense.to(torch.bfloat16))
    cnt = int(ref.count.item())
    assert int(got.count.item()) == cnt and torch.equal(got.rows[:cnt], ref.rows[:cnt])
    with pytest.raises(RuntimeError):
        K.embedding_backward(src, R, D, dense=True, chunked=False, dense_dtype=torch.bfloat16)


# ------------------------------------------------ occurrence sort (grk_sort) --
@pytest.mark.parametrize('n,end_bit,card', [(1, 1, 2), (4095, 8, 200), (4097, 9, 300), (70001, 16, 40000),
                                            (200000, 21, 1000001), (150000, 21, 10), (33333, 32, 1 << 31),
                                            (5000, 11, 2048), (100000, 20, 1000001), (43008, 20, 30000)])
def test_sort_pairs_is_stable_and_exact(n, end_bit, card):
    """grk_sort_pairs (the embedding backward's occurrence grouping) against
    numpy's stable argsort: keys and values identical, ties in input order --
    hot keys (card 10: every key repeated ~15k times), tile-boundary sizes,
    1- to 32-bit keys: one digit of 1-11 bits, two of 8 / 10 / 11, three of 11."""
    from tencent_recommendation_2025_amd import kernels as K
    rng = np.random.default_rng(n + end_bit)
    keys = rng.integers(0, min(card, 1 << end_bit), n, dtype=np.int64).astype(np.uint32)
    vals = rng.integers(0, 1 << 62, n, dtype=np.int64)
    kd = torch.from_numpy(keys.view(np.int32)).to(DEV)
    vd = torch.from_numpy(vals).to(DEV)
    ko, vo = K.sort_pairs(kd, vd, end_bit)
    order = np.argsort(keys & np.uint32((1 << end_bit) - 1) if end_bit < 32 else keys, kind='stable')
    assert np.array_equal(ko.cpu().numpy().view(np.uint32), keys[order])
    assert np.array_equal(vo.cpu().numpy(), vals[order])
    assert np.array_equal(kd.cpu().numpy().view(np.uint32), keys)  # input untouched


def test_sort_pairs_empty():
    from tencent_recommendation_2025_amd import kernels as K
    k, v = K.sort_pairs(torch.empty(0, dtype=torch.int32, device=DEV), torch.empty(0, dtype=torch.int64, device=DEV))
    assert k.numel() == 0 and v.numel() == 0


@pytest.mark.parametrize('n', [128, 1000, 2048])
@pytest.mark.parametrize('D,dt', [(512, torch.bfloat16), (256, torch.float32), (512, torch.float32)])
def test_small_sparse_call_one_workgroup(K, n, D, dt):
    """Sparse calls of <= 2048 occurrences run in one workgroup (k_bwd_tiny: keys,
    stable ranks, heads and the ordered row sums in one launch -- the user table's
    128-occurrence call at C2): ids, rows, count and row_slot equal the oracle's
    occurrence-order sums bit for bit, over two lookups with a row offset, a hot
    row, padding and an out-of-range id (error flag set, skipped)."""
    rng = np.random.default_rng(n + D)
    R = 5000
    idx = rng.integers(0, 400, n)
    idx[rng.random(n) < 0.2] = 3                     # hot row
    idx[rng.random(n) < 0.1] = 0                     # padding
    g = rng.standard_normal((n, D)).astype(np.float32)
    if dt == torch.bfloat16:
        g = oemb.to_bf16_f32(g)
    h = n // 2
    idx2 = idx.copy()
    idx2[h - 1] = R                                  # out of range in the first lookup
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    slot = torch.full((R + 100,), -1, dtype=torch.int32, device=DEV)
    src = [K.GradSource(T(idx2[:h]), T(g[:h]).to(dt), 0, table_rows=R),
           K.GradSource(T(idx2[h:]), T(g[h:]).to(dt), 0, row_offset=100, table_rows=R)]
    res = K.embedding_backward(src, R + 100, D, dense=False, sparse=True, row_slot=slot, err_flag=err)
    assert int(err.item()) == 1
    rows = np.concatenate([idx2[:h], idx2[h:] + 100])
    keep = np.ones(n, bool)
    keep[h - 1] = False
    keep &= np.concatenate([idx2[:h] != 0, idx2[h:] != 0])
    want_dense = oemb.dense_backward(g[keep], rows[keep], R + 100, padding_idx=None)
    uniq = np.unique(rows[keep])
    cnt = int(res.count.item())
    assert cnt == len(uniq)
    assert np.array_equal(res.ids[:cnt].cpu().numpy(), uniq)
    assert np.array_equal(res.rows[:cnt].cpu().numpy(), want_dense[uniq])
    s = slot.cpu().numpy()
    assert np.array_equal(s[uniq], np.arange(cnt)) and np.all(np.delete(s, uniq) == -1)


@pytest.mark.parametrize('D,dt', [(512, torch.bfloat16), (64, torch.float32)])
def test_skip_row0_bag_slots_change_no_sum(K, D, dt):
    """GRK_FEAT_SKIP_ROW0 (round 4): bag slots on a zero padding row 0 are not read;
    the bag sums equal the flag-less gather and the oracle's slot-0-upward sums
    (values; an all-padding bag is +0 either way)."""
    rng = np.random.default_rng(D)
    R, N, A = 3000, 999, 6
    tab = rng.standard_normal((R, D)).astype(np.float32)
    tab[0] = 0.0
    if dt == torch.bfloat16:
        tab = oemb.to_bf16_f32(tab)
    idx = rng.integers(1, R, (N, A))
    idx[rng.random((N, A)) < 0.6] = 0
    idx[:7] = 0                                    # all-padding bags
    tb = T(tab).to(dt)
    outs = []
    for skip in (False, True):
        out = torch.full((N, D), float('nan'), dtype=dt, device=DEV)
        K.embedding_gather([K.Lookup(tb, T(idx), 0, bag=A, skip_row0=skip)], out, N)
        outs.append(out.float().cpu().numpy())
    assert np.array_equal(outs[0], outs[1])
    assert np.array_equal(outs[1], oemb.bag_sum(tab, idx, out_bf16=dt == torch.bfloat16))
    assert np.all(outs[1][:7] == 0)


@pytest.mark.parametrize('odt', [torch.bfloat16, torch.float32])
def test_write_columns_equals_copies(K, odt):
    """grk_write_columns (round 4): the gather buffer's dense blocks (an fp32 [N, 32]
    mm block, a broadcast [1, 8] constant row, a bf16 block) in one launch == the
    per-block copy_ it replaces, bit for bit; other columns untouched."""
    g = torch.Generator(device=DEV).manual_seed(3)
    N = 3001
    mm = torch.randn(N, 40, generator=g, device=DEV)[:, 3:35]          # strided rows
    unit = torch.zeros(1, 8, device=DEV)
    unit[0, 0] = 1.0
    b16 = torch.randn(N, 16, generator=g, device=DEV).bfloat16()
    blocks = [(64, mm), (96, unit), (112, b16)]
    got = torch.full((N, 136), -3.0, dtype=odt, device=DEV)
    want = got.clone()
    K.write_columns(got, blocks)
    for col, x in blocks:
        want[:, col:col + x.shape[1]].copy_(x)
    assert torch.equal(got, want)
