"""GPU parity of grk_attention_fwd/bwd against the oracle (oracle/attention.py
is pinned to the reference's SDPA in tests/test_oracle_golden.py; oracle/hstu.py
is parity-unpinned, checked by finite differences in test_oracle_selfcheck.py).

Tolerance (BASELINE.json north star): 1e-3 normwise relative error for bf16
attention, against the fp64 oracle fed the SAME bf16-rounded inputs.  fp32
outputs are compared as they are; bf16 outputs against the oracle's outputs
rounded to bf16 (and the softmax backward's delta = rowsum(dO * O) formed from
the bf16-rounded O, as the kernels form it from the O they stored).  The
product path (model, bench) runs the precise (hi/lo P / dS operand) kernels,
the default; the opt-in fast mode (P and dS rounded to bf16) is held to 1e-2.

The C2 tests run the bench's exact attention shape (B=128, T=201, H=8, hd=64,
ragged left padding, SiLU on load for HSTU)."""
import os

import numpy as np
import pytest
import torch

from oracle import attention as oatt
from oracle import hstu as ohstu
from oracle.embedding import to_bf16_f32

pytestmark = pytest.mark.gpu
DEV = 'cuda'
TOL_PRECISE = 1e-3
TOL_FAST = 1e-2


@pytest.fixture(scope='module')
def K():
    from tencent_recommendation_2025_amd import _lib, kernels
    _lib.lib()
    return kernels


def nrel(got, want):
    want = np.asarray(want, np.float64)
    den = np.linalg.norm(want)
    return float(np.linalg.norm(np.asarray(got, np.float64) - want) / (den if den > 0 else 1.0))


def make_inputs(B, T, H, hd, lens, seed, width_mult=3):
    """Packed bf16 qkv [B*T, 3*H*hd] (q|k|v column blocks) + key_valid from left-padded lengths."""
    rng = np.random.default_rng(seed)
    D = H * hd
    x = to_bf16_f32(rng.standard_normal((B * T, width_mult * D)).astype(np.float32))
    valid = np.zeros((B, T), np.uint8)
    for b, n in enumerate(lens):
        valid[b, T - n:] = 1
    return x, valid


def heads(x, B, T, H, hd):
    return x.reshape(B, T, H, hd).transpose(0, 2, 1, 3)


def flat(x):
    B, H, T, hd = x.shape
    return x.transpose(0, 2, 1, 3).reshape(B * T, H * hd)


def drop_mask_np(seed, B, H, T, p):
    """numpy replica of drop_keep() in grk_attention.hip (test infrastructure)."""
    with np.errstate(over='ignore'):
        bh = np.arange(B * H, dtype=np.uint64)[:, None, None]
        q = np.arange(T, dtype=np.uint64)[None, :, None]
        k = np.arange(T, dtype=np.uint64)[None, None, :]
        T64 = np.uint64(T)
        x = np.uint64(seed) ^ (((bh * T64 + q) * T64 + k) * np.uint64(0x9E3779B97F4A7C15))
        x ^= x >> np.uint64(30); x *= np.uint64(0xBF58476D1CE4E5B9)
        x ^= x >> np.uint64(27); x *= np.uint64(0x94D049BB133111EB)
        x ^= x >> np.uint64(31)
    u = (x >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    return (u >= np.float32(p)).reshape(B, H, T, T)


def run(K, kind, B, T, H, hd, lens, precise, seed=0, dropout=0.0, nb=None, out_dtype=torch.float32, act=None,
        holes=False, use_ranges=False, oracle=True, nbt=0):
    """act='silu': x holds pre-activations; the oracle sees SiLU(x) rounded to bf16
    and its q/k/v gradients are chained through dSiLU(x)."""
    from tencent_recommendation_2025_amd import _lib as L
    D = H * hd
    x, valid = make_inputs(B, T, H, hd, lens, seed)
    if holes:  # non-contiguous key validity (not the dataset's left padding): the masked path
        valid[:, ::7] = 0
    pre = x
    xd = torch.from_numpy(x).to(DEV).to(torch.bfloat16)
    q, k, v = xd[:, :D], xd[:, D:2 * D], xd[:, 2 * D:]
    kv = torch.from_numpy(valid).to(DEV)
    rng = np.random.default_rng(seed + 1)
    rab = None
    extra = {}
    ts_np = rabt_np = None
    if kind == L.ATTN_HSTU:
        nb = nb or T
        rab_np = (rng.standard_normal((H, nb)) * 0.5).astype(np.float32)
        rab = torch.from_numpy(rab_np).to(DEV)
        extra = dict(rab=rab, inv_n=1.0 / T, scale=hd ** -0.5)
        if nbt:  # time bias: unix-like seconds, heavy-tailed gaps (seconds .. months)
            trng = np.random.default_rng(seed + 7)
            ts_np = (1_700_000_000 + np.cumsum(np.exp(trng.uniform(0, 16, (B, T))), 1)).astype(np.int64)
            rabt_np = (trng.standard_normal((H, nbt)) * 0.5).astype(np.float32)
            extra.update(timestamps=torch.from_numpy(ts_np).to(DEV), rab_t=torch.from_numpy(rabt_np).to(DEV))
    args = K.attn_args(kind, q, k, v, B, T, H, hd, key_valid=kv, precise=precise, dropout_p=dropout, seed=1234,
                       out_dtype=out_dtype, act=act, seq_range=K.seq_ranges(kv) if use_ranges else None, **extra)
    if act == 'silu':
        x = to_bf16_f32((pre / (1.0 + np.exp(-pre.astype(np.float64)))).astype(np.float32))
    out = torch.empty(B * T, D, dtype=out_dtype, device=DEV)
    lse = torch.empty(B, H, T, dtype=torch.float32, device=DEV)
    K.attention_fwd(args, out, lse)
    dout_np = to_bf16_f32(rng.standard_normal((B * T, D)).astype(np.float32))
    dout = torch.from_numpy(dout_np).to(DEV).to(out_dtype)
    dq, dk, dv = (torch.empty(B * T, D, dtype=out_dtype, device=DEV) for _ in range(3))
    delta = torch.empty(B, H, T, device=DEV)
    drab = torch.zeros(H, nb, device=DEV) if kind == L.ATTN_HSTU else None
    drab_t = torch.zeros(H, nbt, device=DEV) if nbt else None
    K.attention_bwd(args, out, dout, lse, delta, dq, dk, dv, drab, drab_t=drab_t)
    torch.cuda.synchronize()
    qh, kh, vh = (heads(x[:, i * D:(i + 1) * D], B, T, H, hd) for i in range(3))
    doh = heads(dout_np, B, T, H, hd)
    res = dict(out=out.float().cpu().numpy(), dq=dq.float().cpu().numpy(), dk=dk.float().cpu().numpy(),
               dv=dv.float().cpu().numpy(), lse=lse.cpu().numpy())
    if kind == L.ATTN_HSTU:
        res['drab'] = drab.cpu().numpy()
    if nbt:
        res['drab_t'] = drab_t.cpu().numpy()
    if not oracle:
        return res, None, valid
    if kind == L.ATTN_SOFTMAX:
        keep = drop_mask_np(1234, B, H, T, dropout) if dropout > 0 else None
        o, lse_ref, _ = oatt.forward(qh, kh, vh, valid.astype(bool), keep=keep, dropout_p=dropout)
        stored = None if out_dtype == torch.float32 else to_bf16_f32(o.astype(np.float32))
        gq, gk, gv = oatt.backward(qh, kh, vh, valid.astype(bool), doh, keep=keep, dropout_p=dropout,
                                   out_stored=stored)
        want = dict(out=flat(o), dq=flat(gq), dk=flat(gk), dv=flat(gv), lse=lse_ref)
    else:
        o, _, _ = ohstu.forward(qh, kh, vh, valid.astype(bool), rab_np, hd ** -0.5, 1.0 / T, ts_np, rabt_np)
        g = ohstu.backward(qh, kh, vh, valid.astype(bool), rab_np, hd ** -0.5, 1.0 / T, doh, ts_np, rabt_np)
        want = dict(out=flat(o), dq=flat(g[0]), dk=flat(g[1]), dv=flat(g[2]), drab=g[3])
        if nbt:
            want['drab_t'] = g[4]
    if act == 'silu':
        for i, key in enumerate(('dq', 'dk', 'dv')):
            want[key] = want[key] * ohstu.dsilu(pre[:, i * D:(i + 1) * D].astype(np.float64))
    return res, want, valid


@pytest.mark.parametrize('hd', [16, 32, 64, 128])
@pytest.mark.parametrize('kind', [0, 1], ids=['softmax', 'hstu'])
def test_attention_parity_precise(K, kind, hd):
    H = 2 if hd >= 64 else 4
    res, want, valid = run(K, kind, B=3, T=201, H=H, hd=hd, lens=[201, 120, 7], precise=True)
    for key in ('out', 'dq', 'dk', 'dv') + (('drab',) if kind == 1 else ()):
        err = nrel(res[key], want[key])
        assert err < TOL_PRECISE, f'{key}: normwise rel err {err:.2e}'
    if kind == 0:
        live = np.isfinite(want['lse'])
        np.testing.assert_allclose(res['lse'][live], want['lse'][live], rtol=1e-5, atol=1e-4)
        assert np.all(np.isneginf(res['lse'][~live]))


@pytest.mark.parametrize('kind', [0, 1], ids=['softmax', 'hstu'])
def test_attention_parity_fast_bf16(K, kind):
    """Opt-in fast mode (precise=False; not used by the model or the bench)."""
    res, want, _ = run(K, kind, B=4, T=201, H=8, hd=64, lens=[201, 150, 64, 33], precise=False,
                       out_dtype=torch.bfloat16)
    for key in ('out', 'dq', 'dk', 'dv'):
        err = nrel(res[key], want[key])
        assert err < TOL_FAST, f'{key}: normwise rel err {err:.2e}'


C2_LENS = np.random.default_rng(3).integers(32, 202, 128).tolist()   # U{32..201}, as synthetic.make_batch


@pytest.mark.parametrize('out_dtype', [torch.float32, torch.bfloat16], ids=['f32out', 'bf16out'])
@pytest.mark.parametrize('kind', [0, 1], ids=['softmax', 'hstu'])
def test_attention_parity_c2_shape(K, kind, out_dtype):
    """The product kernels at the bench's shape: < 1e-3 normwise for out, dq, dk,
    dv (and drab) against the fp64 oracle on identically rounded inputs."""
    res, want, _ = run(K, kind, B=128, T=201, H=8, hd=64, lens=C2_LENS, precise=True, seed=11,
                       out_dtype=out_dtype, act='silu' if kind == 1 else None)
    for key in ('out', 'dq', 'dk', 'dv') + (('drab',) if kind == 1 else ()):
        w = want[key]
        if out_dtype == torch.bfloat16 and key != 'drab':
            w = to_bf16_f32(np.asarray(w, np.float32))
        err = nrel(res[key], w)
        assert err < TOL_PRECISE, f'{key}: normwise rel err {err:.2e}'


@pytest.mark.parametrize('kind', [0, 1], ids=['softmax', 'hstu'])
def test_c2_shape_repeatable(K, kind):
    """Forward + backward at the C2 shape (1024 workgroups: two share a CU)
    repeated: bitwise equal outputs.  Round 1 built these kernels with
    -amdgpu-mfma-vgpr-form, which gave timing-dependent wrong rows in the HSTU
    forward exactly when workgroups shared a CU."""
    runs = [run(K, kind, B=128, T=201, H=8, hd=64, lens=C2_LENS, precise=True, seed=4,
                act='silu' if kind == 1 else None, out_dtype=torch.bfloat16, oracle=False)[0] for _ in range(3)]
    for r in runs[1:]:
        for key in runs[0]:
            if key == 'lse' and kind == 1:
                continue  # HSTU writes no lse
            assert np.array_equal(runs[0][key], r[key]), key


def test_fully_masked_rows_are_zero(K):
    res, want, valid = run(K, 0, B=2, T=70, H=2, hd=64, lens=[70, 5], precise=True)
    pad_rows = np.where(valid.reshape(-1) == 0)[0]
    for key in ('out', 'dq'):
        assert np.all(res[key][pad_rows] == 0)
        assert np.all(np.isfinite(res[key]))
    assert np.all(np.isfinite(res['dk'])) and np.all(np.isfinite(res['dv']))


def test_softmax_dropout_matches_masked_oracle(K):
    res, want, _ = run(K, 0, B=2, T=97, H=2, hd=32, lens=[97, 40], precise=True, dropout=0.2)
    for key in ('out', 'dq', 'dk', 'dv'):
        err = nrel(res[key], want[key])
        assert err < TOL_PRECISE, f'{key}: normwise rel err {err:.2e}'


def test_long_sequence_multi_chunk(K):
    """T=1025 (config 5 length): many K/V chunks and q-blocks."""
    res, want, _ = run(K, 1, B=1, T=1025, H=1, hd=128, lens=[900], precise=True, nb=1025)
    for key in ('out', 'dq', 'dk', 'dv', 'drab'):
        err = nrel(res[key], want[key])
        assert err < TOL_PRECISE, f'{key}: normwise rel err {err:.2e}'


def test_hstu_bucket_clipping(K):
    res, want, _ = run(K, 1, B=2, T=150, H=2, hd=64, lens=[150, 90], precise=True, nb=33)
    for key in ('out', 'dq', 'dk', 'dv', 'drab'):
        assert nrel(res[key], want[key]) < TOL_PRECISE, key


@pytest.mark.parametrize('kind', [0, 1], ids=['softmax', 'hstu'])
@pytest.mark.parametrize('T', [130, 600])  # whole-sequence and chunked kernels
def test_determinism(K, kind, T):
    a, _, _ = run(K, kind, B=3, T=T, H=2, hd=64, lens=[T, 77, 9], precise=False, seed=5)
    b, _, _ = run(K, kind, B=3, T=T, H=2, hd=64, lens=[T, 77, 9], precise=False, seed=5)
    for key in ('out', 'dq', 'dk', 'dv') + (('drab',) if kind == 1 else ()):
        assert np.array_equal(a[key], b[key]), key


@pytest.mark.parametrize('kind', [0, 1], ids=['softmax', 'hstu'])
def test_silu_on_load_matches_oracle(K, kind):
    """GRK_ACT_SILU: q/k/v are pre-activations; dq/dk/dv are w.r.t. them."""
    res, want, _ = run(K, kind, B=3, T=201, H=2, hd=64, lens=[201, 120, 7], precise=True, act='silu')
    for key in ('out', 'dq', 'dk', 'dv') + (('drab',) if kind == 1 else ()):
        err = nrel(res[key], want[key])
        assert err < TOL_PRECISE, f'{key}: normwise rel err {err:.2e}'


def test_seq_ranges(K):
    valid = np.zeros((5, 40), np.uint8)
    valid[0, 10:] = 1          # left padding
    valid[1, :] = 1            # full
    valid[2, 5:20] = 1         # hole at the end: not contiguous to T
    valid[3, [3, 9]] = 1       # scattered
    got = K.seq_ranges(torch.from_numpy(valid).to(DEV)).cpu().numpy()  # row 4: no valid key
    np.testing.assert_array_equal(got[:, :2], [[10, 1], [0, 1], [5, 0], [3, 0], [40, 1]])
    np.testing.assert_array_equal(got[:, 2], [1, 3, 2, 0, 4])   # T - first: 30, 40, 35, 37, 0


@pytest.mark.parametrize('B', [1, 128, 240, 1024, 1025, 9000])   # one launch (B T <= 48 KiB), LDS rank, memory rank
def test_seq_ranges_random(K, B):
    T = 201
    rng = np.random.default_rng(B)
    first = rng.integers(0, T + 1, B)
    first[rng.random(B) < 0.3] = rng.integers(0, 4)          # many ties in the length order
    valid = (np.arange(T)[None, :] >= first[:, None]).astype(np.uint8)
    holes = rng.random(B) < 0.2
    valid[holes, -1] = 0                                     # not contiguous to T
    got = K.seq_ranges(torch.from_numpy(valid).to(DEV)).cpu().numpy()
    f = np.where(valid.any(1), valid.argmax(1), T)
    contig = valid.sum(1) == T - f
    np.testing.assert_array_equal(got[:, 0], f)
    np.testing.assert_array_equal(got[:, 1], contig.astype(np.int32))
    np.testing.assert_array_equal(got[:, 2], np.argsort(-(T - f), kind='stable'))


@pytest.mark.parametrize('kind', [0, 1], ids=['softmax', 'hstu'])
def test_precomputed_ranges_bitwise_equal(K, kind):
    a, _, _ = run(K, kind, B=3, T=201, H=2, hd=64, lens=[201, 120, 7], precise=False, act='silu' if kind else None)
    b, _, _ = run(K, kind, B=3, T=201, H=2, hd=64, lens=[201, 120, 7], precise=False, act='silu' if kind else None,
                  use_ranges=True)
    for key in a:
        if key == 'lse' and kind == 1:
            continue  # HSTU writes no lse
        assert np.array_equal(a[key], b[key]), key


@pytest.mark.parametrize('kind', [0, 1], ids=['softmax', 'hstu'])
@pytest.mark.parametrize('use_ranges', [False, True])
def test_non_contiguous_key_valid(K, kind, use_ranges):
    res, want, _ = run(K, kind, B=3, T=150, H=2, hd=64, lens=[150, 90, 40], precise=True, holes=True,
                       use_ranges=use_ranges)
    for key in ('out', 'dq', 'dk', 'dv') + (('drab',) if kind == 1 else ()):
        err = nrel(res[key], want[key])
        assert err < TOL_PRECISE, f'{key}: normwise rel err {err:.2e}'


@pytest.mark.parametrize('T,nbt', [(130, 0), (201, 16), (600, 0)])  # whole-sequence (+ time bias), chunked
def test_bwd_drab_set_clean_scratch_equals_accumulate(K, T, nbt):
    """GRK_ATTN_BWD_WS_CLEAN | GRK_ATTN_BWD_DRAB_SET (the model's path): drab / drab_t
    written through the stream's clean fixed-point scratch -- finalized by the last dq
    workgroup (whole-sequence kernel) or by the fallback launch (chunked) -- equal the
    accumulate path into zeroed buffers bit for bit, call after call (the scratch and
    its counter are left zero); dq / dk / dv unchanged."""
    from tencent_recommendation_2025_amd import _lib as L
    B, H, hd = 3, 2, 64
    D = H * hd
    x, valid = make_inputs(B, T, H, hd, [T, T // 2, 7], 9)
    xd = torch.from_numpy(x).to(DEV).to(torch.bfloat16)
    kv = torch.from_numpy(valid).to(DEV)
    extra = dict(rab=0.3 * torch.randn(H, T, device=DEV), inv_n=1.0 / T, scale=hd ** -0.5)
    if nbt:
        ts = 1_700_000_000 + torch.cumsum(torch.randint(1, 100000, (B, T)), 1)
        extra.update(timestamps=ts.to(DEV), rab_t=0.3 * torch.randn(H, nbt, device=DEV))
    args = K.attn_args(L.ATTN_HSTU, xd[:, :D], xd[:, D:2 * D], xd[:, 2 * D:], B, T, H, hd, key_valid=kv,
                       out_dtype=torch.bfloat16, act='silu', precise=1, **extra)
    out = torch.empty(B * T, D, dtype=torch.bfloat16, device=DEV)
    K.attention_fwd(args, out, torch.empty(B, H, T, device=DEV))
    dout = torch.randn(B * T, D, device=DEV).bfloat16()

    def bwd(drab_set, fill):
        g = [torch.empty(B * T, D, dtype=torch.bfloat16, device=DEV) for _ in range(3)]
        drab = torch.full((H, T), fill, device=DEV)
        drab_t = torch.full((H, nbt), fill, device=DEV) if nbt else None
        K.attention_bwd(args, None, dout, None, None, *g, drab, drab_t=drab_t, drab_set=drab_set)
        return g, drab, drab_t

    ref = bwd(False, 0.0)
    for _ in range(3):
        got = bwd(True, float('nan'))   # written, not accumulated: the fill never shows
        for a, b in zip(ref[0], got[0]):
            assert torch.equal(a, b)
        assert torch.equal(ref[1], got[1])
        if nbt:
            assert torch.equal(ref[2], got[2])
    acc = bwd(False, 1.0)   # the default still accumulates
    assert torch.equal(acc[1], ref[1] + 1.0)


@pytest.mark.parametrize('kind', [0, 1], ids=['softmax', 'hstu'])
@pytest.mark.parametrize('T', [130, 600])  # whole-sequence and chunked kernels
def test_bwd_parts_equal_full_backward(K, kind, T):
    """grk_attention_bwd_parts: the dq half then the dk/dv half (each may run on
    its own stream) give bitwise the outputs of the one-call backward."""
    from tencent_recommendation_2025_amd import _lib as L
    B, H, hd = 3, 2, 64
    D = H * hd
    x, valid = make_inputs(B, T, H, hd, [T, T // 2, 7], 5)
    xd = torch.from_numpy(x).to(DEV).to(torch.bfloat16)
    kv = torch.from_numpy(valid).to(DEV)
    extra = dict(rab=0.3 * torch.randn(H, T, device=DEV), inv_n=1.0 / T) if kind == L.ATTN_HSTU else {}
    args = K.attn_args(kind, xd[:, :D], xd[:, D:2 * D], xd[:, 2 * D:], B, T, H, hd, key_valid=kv,
                       out_dtype=torch.bfloat16, act='silu' if kind == L.ATTN_HSTU else None, **extra)
    out = torch.empty(B * T, D, dtype=torch.bfloat16, device=DEV)
    lse = torch.empty(B, H, T, device=DEV)
    K.attention_fwd(args, out, lse)
    dout = torch.randn(B * T, D, device=DEV).bfloat16()

    def bwd(split):
        g = [torch.full((B * T, D), 7.0, dtype=torch.bfloat16, device=DEV) for _ in range(3)]
        delta = torch.empty(B, H, T, device=DEV)
        drab = torch.zeros(H, T, device=DEV) if kind == L.ATTN_HSTU else None
        if split:
            K.attention_bwd(args, out, dout, lse, delta, g[0], None, None, drab, parts=L.ATTN_BWD_DQ)
            assert torch.all(g[1] == 7.0) and torch.all(g[2] == 7.0)
            K.attention_bwd(args, out, dout, lse, delta, None, g[1], g[2], None, parts=L.ATTN_BWD_DKDV)
        else:
            K.attention_bwd(args, out, dout, lse, delta, *g, drab)
        return g, drab

    (a, ra), (b, rb) = bwd(False), bwd(True)
    for x1, x2 in zip(a, b):
        assert torch.equal(x1, x2)
    if ra is not None:
        assert torch.equal(ra, rb)


def run_fidelity(K, kind, B, T, H, hd, lens, in_dtype, seed=0, act=None):
    """precise=2: q/k/v given in fp32 / fp16 (not rounded to bf16), fp32 outputs."""
    from tencent_recommendation_2025_amd import _lib as L
    D = H * hd
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((B * T, 3 * D)).astype(np.float32)
    if in_dtype == torch.float16:
        x = x.astype(np.float16).astype(np.float32)
    valid = np.zeros((B, T), np.uint8)
    for b, n in enumerate(lens):
        valid[b, T - n:] = 1
    xd = torch.from_numpy(x).to(DEV).to(in_dtype)
    kv = torch.from_numpy(valid).to(DEV)
    extra, rab_np = {}, None
    if kind == L.ATTN_HSTU:
        rab_np = (np.random.default_rng(seed + 1).standard_normal((H, T)) * 0.5).astype(np.float32)
        extra = dict(rab=torch.from_numpy(rab_np).to(DEV), inv_n=1.0 / T, scale=hd ** -0.5)
    args = K.attn_args(kind, xd[:, :D], xd[:, D:2 * D], xd[:, 2 * D:], B, T, H, hd, key_valid=kv, precise=2,
                       out_dtype=torch.float32, act=act, **extra)
    out = torch.empty(B * T, D, device=DEV)
    lse = torch.empty(B, H, T, device=DEV)
    K.attention_fwd(args, out, lse)
    dout_np = np.random.default_rng(seed + 2).standard_normal((B * T, D)).astype(np.float32)
    dout = torch.from_numpy(dout_np).to(DEV)
    dq, dk, dv = (torch.empty(B * T, D, device=DEV) for _ in range(3))
    drab = torch.zeros(H, T, device=DEV) if kind == L.ATTN_HSTU else None
    K.attention_bwd(args, out, dout, lse, torch.empty(B, H, T, device=DEV), dq, dk, dv, drab)
    torch.cuda.synchronize()
    xa = x.astype(np.float64)
    if act == 'silu':
        xa = xa / (1.0 + np.exp(-xa))
    qh, kh, vh = (heads(xa[:, i * D:(i + 1) * D], B, T, H, hd) for i in range(3))
    doh = heads(dout_np, B, T, H, hd)
    if kind == L.ATTN_SOFTMAX:
        o, _, _ = oatt.forward(qh, kh, vh, valid.astype(bool))
        gq, gk, gv = oatt.backward(qh, kh, vh, valid.astype(bool), doh)
        want = dict(out=flat(o), dq=flat(gq), dk=flat(gk), dv=flat(gv))
    else:
        o, _, _ = ohstu.forward(qh, kh, vh, valid.astype(bool), rab_np, hd ** -0.5, 1.0 / T)
        gq, gk, gv, gr = ohstu.backward(qh, kh, vh, valid.astype(bool), rab_np, hd ** -0.5, 1.0 / T, doh)
        want = dict(out=flat(o), dq=flat(gq), dk=flat(gk), dv=flat(gv), drab=gr)
    if act == 'silu':
        for i, key in enumerate(('dq', 'dk', 'dv')):
            want[key] = want[key] * ohstu.dsilu(x[:, i * D:(i + 1) * D].astype(np.float64))
    res = dict(out=out.cpu().numpy(), dq=dq.cpu().numpy(), dk=dk.cpu().numpy(), dv=dv.cpu().numpy())
    if drab is not None:
        res['drab'] = drab.cpu().numpy()
    return res, want


FIDELITY_TOL = 2e-5   # normwise vs the fp64 oracle on the unrounded inputs (measured: see DESIGN.md §4)


@pytest.mark.parametrize('in_dtype', [torch.float32, torch.float16], ids=['f32', 'f16'])
@pytest.mark.parametrize('hd,T,lens', [(16, 102, [102, 60, 7, 1]), (64, 102, [102, 60, 7, 33]),
                                       (64, 201, [201, 120, 7]), (128, 102, [102, 50])])
@pytest.mark.parametrize('kind', [0, 1], ids=['softmax', 'hstu'])
def test_fidelity_mode_matches_fp64_oracle(K, kind, hd, T, lens, in_dtype):
    """precise=2 (fp32 fidelity, the drop-in fp32 / fp16-autocast path): Q/K/V and
    dO enter every MFMA as bf16 hi + lo (hi*hi + hi*lo + lo*hi), P / dS likewise,
    so out / dq / dk / dv / drab match the fp64 oracle on the unrounded inputs to
    fp32-level error (reference BaseLine/main.py:163-190 runs fp32)."""
    H = 2 if hd >= 64 else 4
    res, want = run_fidelity(K, kind, len(lens), T, H, hd, lens, in_dtype, seed=hd + T,
                             act='silu' if kind == 1 else None)
    for key in res:
        err = nrel(res[key], want[key])
        print(f'fidelity {key}: {err:.2e}')
        assert err < FIDELITY_TOL, f'{key}: normwise rel err {err:.2e}'


def test_fidelity_supported_shapes(K):
    assert K.fidelity_supported(201, 64) and K.fidelity_supported(102, 128)
    assert not K.fidelity_supported(201, 128) and not K.fidelity_supported(1025, 64)


# ---------------------------------------------------------------- wide heads --
# head_dim 256 / 512 (grk_attention_wide.hip): one head over the whole hidden
# width, as the O1 baseline's num_heads=1 (model/BaseLineO1/main.py:45).
WIDE = [(256, 2), (512, 1)]


@pytest.mark.parametrize('hd,H', WIDE)
@pytest.mark.parametrize('kind', [0, 1], ids=['softmax', 'hstu'])
def test_wide_head_parity(K, kind, hd, H):
    res, want, _ = run(K, kind, B=3, T=201, H=H, hd=hd, lens=[201, 120, 7], precise=True, seed=hd,
                       act='silu' if kind == 1 else None)
    for key in ('out', 'dq', 'dk', 'dv') + (('drab',) if kind == 1 else ()):
        err = nrel(res[key], want[key])
        assert err < TOL_PRECISE, f'{key}: normwise rel err {err:.2e}'
    if kind == 0:
        live = np.isfinite(want['lse'])
        np.testing.assert_allclose(res['lse'][live], want['lse'][live], rtol=1e-5, atol=1e-4)
        assert np.all(np.isneginf(res['lse'][~live]))


@pytest.mark.parametrize('hd,H', WIDE)
def test_wide_head_dropout_holes_bf16(K, hd, H):
    """Dropout (the drop_keep stream of the narrow kernels), non-contiguous key
    validity and bf16 outputs (compared with the oracle rounded to bf16)."""
    res, want, _ = run(K, 0, B=2, T=97, H=H, hd=hd, lens=[97, 40], precise=True, dropout=0.2, holes=True,
                       out_dtype=torch.bfloat16)
    for key in ('out', 'dq', 'dk', 'dv'):
        err = nrel(res[key], to_bf16_f32(np.asarray(want[key], np.float32)))
        assert err < TOL_PRECISE, f'{key}: normwise rel err {err:.2e}'


def test_wide_head_long_sequence_and_repeatable(K):
    """T=600: many 32-row tiles per workgroup; clipped rab buckets; bitwise repeatable."""
    a, want, _ = run(K, 1, B=2, T=600, H=1, hd=256, lens=[600, 333], precise=True, nb=257)
    for key in ('out', 'dq', 'dk', 'dv', 'drab'):
        err = nrel(a[key], want[key])
        assert err < TOL_PRECISE, f'{key}: normwise rel err {err:.2e}'
    b, _, _ = run(K, 1, B=2, T=600, H=1, hd=256, lens=[600, 333], precise=True, nb=257, oracle=False)
    for key in ('out', 'dq', 'dk', 'dv', 'drab'):
        assert np.array_equal(a[key], b[key]), key


def test_wide_head_masked_rows_and_fast_mode(K):
    res, want, valid = run(K, 0, B=2, T=70, H=1, hd=512, lens=[70, 5], precise=False)
    pad_rows = np.where(valid.reshape(-1) == 0)[0]
    for key in ('out', 'dq'):
        assert np.all(res[key][pad_rows] == 0)
    for key in ('out', 'dq', 'dk', 'dv'):
        assert np.all(np.isfinite(res[key]))
        assert nrel(res[key], want[key]) < TOL_FAST, key


def test_wide_head_fidelity_mode_supported():
    """fp32 fidelity at head_dim 256 / 512 (the wide kernels' FID instantiations,
    hardware-verified in round 4): supported at any length; other widths beyond the
    whole-sequence LDS are refused."""
    from tencent_recommendation_2025_amd import kernels as K
    assert K.fidelity_supported(101, 512) and K.fidelity_supported(3000, 256)
    assert not K.fidelity_supported(3000, 64)


# fp32 fidelity at head_dim 256 / 512 (grk_attention_wide_fid.hip): written in round 3
# without hardware, verified on MI355X in round 4 (this test, then default).
@pytest.mark.parametrize('in_dtype', [torch.float32, torch.float16], ids=['f32', 'f16'])
@pytest.mark.parametrize('H,T,lens', [(1, 102, [102, 60, 7]), (2, 201, [201, 33])])
@pytest.mark.parametrize('kind', [0, 1], ids=['softmax', 'hstu'])
@pytest.mark.parametrize('hd', [256, 512])
def test_wide_fidelity_matches_fp64_oracle(K, hd, kind, H, T, lens, in_dtype):
    """precise=2 at head_dim 256 / 512 (O1's num_heads=1 at hidden 256 / 512): Q/K/V /
    dO read exactly and split into bf16 hi + lo, every product hi*hi + hi*lo + lo*hi,
    against the fp64 oracle on the unrounded inputs (the narrow kernels' bound).  At
    512 the waves' partial products meet in four rounds (WideF)."""
    assert K.fidelity_supported(T, hd)
    res, want = run_fidelity(K, kind, len(lens), T, H, hd, lens, in_dtype, seed=T + H,
                             act='silu' if kind == 1 else None)
    for key in res:
        err = nrel(res[key], want[key])
        print(f'wide fidelity {key}: {err:.2e}')
        assert err < FIDELITY_TOL, f'{key}: normwise rel err {err:.2e}'


# ------------------------------------------------------------- time bias --
# HSTU rab_time: rab_t[h, half-octave bucket of t_q - t_k]
@pytest.mark.parametrize('hd,H,T,lens,act', [(64, 2, 201, [201, 120, 7], 'silu'), (32, 4, 97, [97, 40], None),
                                             (64, 2, 150, [150, 90, 40], 'silu')])
def test_time_bias_matches_oracle(K, hd, H, T, lens, act):
    res, want, _ = run(K, 1, B=len(lens), T=T, H=H, hd=hd, lens=lens, precise=True, nbt=48, act=act, seed=T)
    for key in ('out', 'dq', 'dk', 'dv', 'drab', 'drab_t'):
        err = nrel(res[key], want[key])
        assert err < TOL_PRECISE, f'{key}: normwise rel err {err:.2e}'
    assert np.count_nonzero(want['drab_t']) > 10


def test_time_bias_c2_shape_and_repeatable(K):
    a, want, _ = run(K, 1, B=128, T=201, H=8, hd=64, lens=C2_LENS, precise=True, seed=13, act='silu', nbt=64,
                     out_dtype=torch.bfloat16)
    for key in ('out', 'dq', 'dk', 'dv'):
        assert nrel(a[key], to_bf16_f32(np.asarray(want[key], np.float32))) < TOL_PRECISE, key
    for key in ('drab', 'drab_t'):
        assert nrel(a[key], want[key]) < TOL_PRECISE, key
    b, _, _ = run(K, 1, B=128, T=201, H=8, hd=64, lens=C2_LENS, precise=True, seed=13, act='silu', nbt=64,
                  out_dtype=torch.bfloat16, oracle=False)
    for key in a:
        if key != 'lse':
            assert np.array_equal(a[key], b[key]), key


def test_time_bias_is_hstu_only(K):
    """The time bias is an HSTU score term: a softmax attention call with time stamps
    is refused (the chunked / wide kernels take it since round 4, below)."""
    from tencent_recommendation_2025_amd import _lib as L
    x = torch.zeros(64, 3 * 64, dtype=torch.bfloat16, device=DEV)
    with pytest.raises(RuntimeError, match='HSTU'):
        K.attn_args(L.ATTN_SOFTMAX, x[:, :64], x[:, 64:128], x[:, 128:], 2, 32, 1, 64,
                    timestamps=torch.zeros(2, 32, dtype=torch.int64, device=DEV),
                    rab_t=torch.zeros(1, 8, device=DEV))


# The chunked kernels (T beyond the whole-sequence kernels' LDS) and the wide-head
# kernels (head_dim 256 / 512) carry the time bias in their TB instantiations
# (written in round 3 without hardware, verified on MI355X in round 4).
@pytest.mark.parametrize('hd,H,T,lens,act,nbt', [(64, 2, 300, [300, 170, 20], 'silu', 48),
                                                 (128, 1, 1025, [1025, 600], None, 64),
                                                 (32, 4, 260, [260, 3], None, 16),
                                                 (256, 1, 150, [150, 90, 7], 'silu', 32),
                                                 (512, 2, 70, [70, 33], None, 16)])
def test_time_bias_chunked_and_wide_kernels_match_oracle(K, hd, H, T, lens, act, nbt):
    res, want, _ = run(K, 1, B=len(lens), T=T, H=H, hd=hd, lens=lens, precise=True, nbt=nbt, act=act, seed=T)
    for key in ('out', 'dq', 'dk', 'dv', 'drab', 'drab_t'):
        err = nrel(res[key], want[key])
        assert err < TOL_PRECISE, f'{key}: normwise rel err {err:.2e}'
    assert np.count_nonzero(want['drab_t']) > 10
    again, _, _ = run(K, 1, B=len(lens), T=T, H=H, hd=hd, lens=lens, precise=True, nbt=nbt, act=act, seed=T,
                      oracle=False)
    for key in res:
        if key != 'lse':
            assert np.array_equal(res[key], again[key]), key


# ----------------------------------------------------------- fp8 (C5) ----
# Config C5 (BASELINE.json configs[4]): d=1024, T=1025, fp8 attention.  q/k/v
# are OCP e4m3 activations; the oracle sees exactly those values (widened to
# fp64), so the 1e-3 bar applies unchanged: QK^T products of fp8 values are
# exact in the MFMA's fp32 accumulation and P / dS enter as bf16 hi + lo.
def run_fp8(K, kind, B, T, H, hd, lens, seed=0, out_dtype=torch.float32):
    from tencent_recommendation_2025_amd import _lib as L
    D = H * hd
    rng = np.random.default_rng(seed)
    x8 = torch.from_numpy(rng.standard_normal((B * T, 3 * D)).astype(np.float32)).to(torch.float8_e4m3fn)
    x = x8.float().numpy()
    valid = np.zeros((B, T), np.uint8)
    for b, n in enumerate(lens):
        valid[b, T - n:] = 1
    xd = x8.to(DEV)
    kv = torch.from_numpy(valid).to(DEV)
    extra, rab_np = {}, None
    if kind == L.ATTN_HSTU:
        rab_np = (np.random.default_rng(seed + 1).standard_normal((H, T)) * 0.5).astype(np.float32)
        extra = dict(rab=torch.from_numpy(rab_np).to(DEV), inv_n=1.0 / T, scale=hd ** -0.5)
    args = K.attn_args(kind, xd[:, :D], xd[:, D:2 * D], xd[:, 2 * D:], B, T, H, hd, key_valid=kv, precise=1,
                       out_dtype=out_dtype, **extra)
    out = torch.empty(B * T, D, device=DEV, dtype=out_dtype)
    lse = torch.empty(B, H, T, device=DEV)
    K.attention_fwd(args, out, lse)
    dout_np = to_bf16_f32(np.random.default_rng(seed + 2).standard_normal((B * T, D)).astype(np.float32))
    dout = torch.from_numpy(dout_np).to(DEV).to(out_dtype)
    dq, dk, dv = (torch.empty(B * T, D, device=DEV, dtype=out_dtype) for _ in range(3))
    drab = torch.zeros(H, T, device=DEV) if kind == L.ATTN_HSTU else None
    K.attention_bwd(args, out, dout, lse, torch.empty(B, H, T, device=DEV), dq, dk, dv, drab)
    torch.cuda.synchronize()
    qh, kh, vh = (heads(x[:, i * D:(i + 1) * D].astype(np.float64), B, T, H, hd) for i in range(3))
    doh = heads(dout_np, B, T, H, hd)
    if kind == L.ATTN_SOFTMAX:
        o, _, _ = oatt.forward(qh, kh, vh, valid.astype(bool))
        gq, gk, gv = oatt.backward(qh, kh, vh, valid.astype(bool), doh)
        want = dict(out=flat(o), dq=flat(gq), dk=flat(gk), dv=flat(gv))
    else:
        o, _, _ = ohstu.forward(qh, kh, vh, valid.astype(bool), rab_np, hd ** -0.5, 1.0 / T)
        gq, gk, gv, gr = ohstu.backward(qh, kh, vh, valid.astype(bool), rab_np, hd ** -0.5, 1.0 / T, doh)
        want = dict(out=flat(o), dq=flat(gq), dk=flat(gk), dv=flat(gv), drab=gr)
    res = {k_: t.float().cpu().numpy() for k_, t in (('out', out), ('dq', dq), ('dk', dk), ('dv', dv))}
    if drab is not None:
        res['drab'] = drab.cpu().numpy()
    return res, want


@pytest.mark.parametrize('kind', [0, 1], ids=['softmax', 'hstu'])
@pytest.mark.parametrize('hd,H,T,lens', [(128, 2, 1025, [1025, 700]), (64, 2, 300, [300, 129, 1]),
                                         (128, 1, 77, [77, 40])])
def test_fp8_attention_matches_oracle(K, kind, hd, H, T, lens):
    res, want = run_fp8(K, kind, B=len(lens), T=T, H=H, hd=hd, lens=lens, seed=T + hd)
    for key in want:
        err = nrel(res[key], want[key])
        assert err < TOL_PRECISE, f'{key}: normwise rel err {err:.2e}'


def test_fp8_attention_bf16_out_repeatable(K):
    a, want = run_fp8(K, 1, B=2, T=1025, H=2, hd=128, lens=[1025, 513], seed=5, out_dtype=torch.bfloat16)
    for key in ('out', 'dq', 'dk', 'dv'):
        assert nrel(a[key], to_bf16_f32(np.asarray(want[key], np.float32))) < TOL_PRECISE, key
    assert nrel(a['drab'], want['drab']) < TOL_PRECISE
    b, _ = run_fp8(K, 1, B=2, T=1025, H=2, hd=128, lens=[1025, 513], seed=5, out_dtype=torch.bfloat16)
    for key in a:
        assert np.array_equal(a[key], b[key]), key


def test_fp8_attention_refusals(K):
    from tencent_recommendation_2025_amd import _lib as L
    x = torch.zeros(64, 3 * 32, device=DEV).to(torch.float8_e4m3fn)
    a = K.attn_args(L.ATTN_SOFTMAX, x[:, :32], x[:, 32:64], x[:, 64:], 2, 32, 1, 32, precise=1)
    with pytest.raises(RuntimeError, match='head_dim 64 / 128'):
        K.attention_fwd(a, torch.empty(64, 32, device=DEV), torch.empty(2, 1, 32, device=DEV))
    with pytest.raises(RuntimeError, match='act'):
        K.attn_args(L.ATTN_SOFTMAX, x[:, :32], x[:, 32:64], x[:, 64:], 2, 32, 1, 32, act='silu')
