"""The jagged (valid-token) layout of the fused trainer (jagged.py, grk_jagged.hip).

* layout / row gather bit-exact vs the numpy oracle (oracle/jagged.py), incl.
  holes, empty sequences, dead capacity rows and the error flags;
* the attention kernels on jagged rows == the padded kernels, bit for bit, on
  every span row (HSTU with rab and time bias, softmax with dropout: forward,
  dQ + drab (+ drab_t), dK/dV; delta) -- and the dead capacity rows of every
  output zeroed;
* the jagged training step against the padded one: log_feats / item
  embeddings equal on the span rows, loss and every gradient equal up to the
  summation order of the GEMMs over fewer rows (fp32: 1e-5; bf16: the bench
  tolerances), graph replay == eager bitwise across two capacities.
The padded step is pinned to the reference (test_gpu_model.py), so the jagged
one is pinned through it."""

import numpy as np
import pytest
import torch

from oracle import jagged as ojag
from oracle.embedding import to_bf16_f32

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def nrel(a, b):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    d = np.linalg.norm(b)
    return float(np.linalg.norm(a - b) / (d if d > 0 else 1.0))


def test_layout_and_gather_match_oracle():
    from tencent_recommendation_2025_amd import jagged as J
    from tencent_recommendation_2025_amd import kernels as K
    rng = np.random.default_rng(0)
    B, T = 37, 51
    tt = np.zeros((B, T), np.int64)
    for b in range(B):
        n = rng.integers(0, T + 1)
        tt[b, T - n:] = rng.integers(1, 3, n)
    tt[3, 40:45] = 0            # a hole inside a span
    tt[5] = 0                   # an empty sequence
    n_rows = int(ojag.layout(tt, B * T)[3])
    assert J.span_rows(torch.from_numpy(tt)) == n_rows == J.span_rows(torch.from_numpy(tt).to(DEV))
    for cap in (n_rows, J.capacity_for(n_rows, 256)):
        jag = J.layout(torch.from_numpy(tt).to(DEV), cap)
        rng_w, base_w, map_w, n_w = ojag.layout(tt, cap)
        assert int(jag.n.item()) == n_w and int(jag.err.item()) == 0
        assert np.array_equal(jag.seq_range.cpu().numpy()[:, :2], rng_w)
        assert np.array_equal(jag.row_base.cpu().numpy()[:B], base_w) and int(jag.row_base[B]) == n_w
        assert np.array_equal(jag.row_map.cpu().numpy(), map_w)
        feats = {'a': rng.integers(0, 100, (B, T)), 'arr': rng.integers(0, 9, (B, T, 3)),
                 'mm': rng.standard_normal((B, T, 32)).astype(np.float32)}
        srcs = {k: torch.from_numpy(v).to(DEV) for k, v in feats.items()}
        dsts = {k: torch.full((cap,) + v.shape[2:], 7, dtype=v.dtype, device=DEV) for k, v in srcs.items()}
        K.gather_rows([(srcs[k].reshape(B * T, *srcs[k].shape[2:]), dsts[k]) for k in srcs], jag.row_map)
        for k in feats:
            assert np.array_equal(dsts[k].cpu().numpy(), ojag.gather_rows(feats[k], map_w)), k
    # error flags: a next-item label before the span (bit 1)
    ntt = (tt != 0).astype(np.int64)
    b0 = int(np.flatnonzero(tt[:, 0] == 0)[0])
    ntt[b0, 0] = 1
    jag = J.layout(torch.from_numpy(tt).to(DEV), n_rows, torch.from_numpy(ntt).to(DEV))
    assert int(jag.err.item()) == 1
    # more span rows than capacity (bit 2): the trailing spans are dropped, exactly as
    # the oracle restates, and nothing is mapped past the capacity
    for cap in (n_rows - 1, n_rows // 2, 1):
        ntt = (tt != 0).astype(np.int64)
        jag = J.layout(torch.from_numpy(tt).to(DEV), cap, torch.from_numpy(ntt).to(DEV))
        rng_w, base_w, map_w, n_w = ojag.layout(tt, cap)
        assert int(jag.err.item()) & 2
        assert int(jag.n.item()) == n_w <= cap
        assert np.array_equal(jag.seq_range.cpu().numpy()[:, :2], rng_w)
        assert np.array_equal(jag.row_base.cpu().numpy()[:B], base_w)
        assert np.array_equal(jag.row_map.cpu().numpy(), map_w)
        with pytest.raises(ValueError, match='more span rows'):
            J.check_error(jag.err)


@pytest.mark.parametrize('B', [200, 300])   # one-launch ranges + row bases (B T <= 48 KiB) and the two-launch form
def test_layout_at_bench_lengths_matches_oracle(B):
    from tencent_recommendation_2025_amd import jagged as J
    rng = np.random.default_rng(B)
    T = 201
    tt = np.zeros((B, T), np.int64)
    for b in range(B):
        n = rng.integers(0, T + 1)
        tt[b, T - n:] = rng.integers(1, 3, n)
    tt[7, 100:110] = 0          # a hole inside a span
    n_rows = int(ojag.layout(tt, B * T)[3])
    for cap in (n_rows, J.capacity_for(n_rows, 1024), n_rows // 2):
        jag = J.layout(torch.from_numpy(tt).to(DEV), cap)
        rng_w, base_w, map_w, n_w = ojag.layout(tt, cap)
        assert int(jag.n.item()) == n_w
        assert bool(int(jag.err.item()) & 2) == (cap < n_rows)
        assert np.array_equal(jag.seq_range.cpu().numpy()[:, :2], rng_w)
        assert np.array_equal(jag.row_base.cpu().numpy()[:B], base_w)
        assert np.array_equal(jag.row_map.cpu().numpy(), map_w)


def test_gather_rows_many_copies_every_unit_width():
    """70 copies (two launches of <= 64) with rows of 4 .. 132 bytes: 16-, 8- and
    4-byte units, and sources offset by 4 / 8 bytes from 16-byte alignment."""
    from tencent_recommendation_2025_amd import kernels as K
    rng = np.random.default_rng(5)
    N, rows = 3001, 2113
    row_map = rng.integers(-1, N, rows).astype(np.int32)
    rmap = torch.from_numpy(row_map).to(DEV)
    pairs, want = [], []
    for i in range(70):
        width = [1, 2, 3, 4, 8, 33, 6][i % 7]                       # int32 words per row
        lead = [0, 1, 2][i % 3]                                     # misalign the source start
        base = torch.from_numpy(rng.integers(-2**31, 2**31 - 1, N * width + lead).astype(np.int32)).to(DEV)
        src = base[lead:].view(N, width)
        dst = torch.full((rows, width), 9, dtype=torch.int32, device=DEV)
        pairs.append((src, dst))
        s = src.cpu().numpy()
        want.append(np.where(row_map[:, None] >= 0, s[np.maximum(row_map, 0)], 0))
    K.gather_rows(pairs, rmap)
    for i, ((_, dst), w) in enumerate(zip(pairs, want)):
        assert np.array_equal(dst.cpu().numpy(), w), i


def _hstu_case(B, T, H, hd, seed, holes=False):
    rng = np.random.default_rng(seed)
    D = H * hd
    pre = to_bf16_f32(rng.standard_normal((B * T, 4 * D)).astype(np.float32))
    kv = np.zeros((B, T), np.uint8)
    lens = rng.integers(1, T + 1, B)
    lens[0] = T
    for b in range(B):
        kv[b, T - lens[b]:] = 1
    if holes:
        kv[1, T - 3] = 0
    return pre, kv


@pytest.mark.parametrize('kind,T,hd,nbt,holes', [('hstu', 201, 64, 0, False), ('hstu', 77, 64, 24, True),
                                                  ('hstu', 100, 128, 0, False), ('softmax', 201, 64, 0, False),
                                                  ('softmax', 60, 32, 0, True)])
def test_attention_jagged_equals_padded_bitwise(kind, T, hd, nbt, holes):
    from tencent_recommendation_2025_amd import _lib as L
    from tencent_recommendation_2025_amd import jagged as J
    from tencent_recommendation_2025_amd import kernels as K
    B, H = 24, 4 if hd <= 64 else 2
    D = H * hd
    pre_np, kv_np = _hstu_case(B, T, H, hd, seed=T + hd, holes=holes)
    pre = torch.from_numpy(pre_np).to(DEV).to(torch.bfloat16)
    kv = torch.from_numpy(kv_np).to(DEV)
    n = J.span_rows(kv)
    cap = J.capacity_for(n, 128)
    jag = J.layout(kv.to(torch.int64), cap)
    jpre = torch.empty(cap, 4 * D, dtype=torch.bfloat16, device=DEV)
    K.gather_rows([(pre, jpre)], jag.row_map)
    g = torch.Generator(device=DEV).manual_seed(1)
    hstu = kind == 'hstu'
    extra = {}
    if hstu:
        extra = dict(rab=0.2 * torch.randn(H, T, device=DEV, generator=g), inv_n=1.0 / T, act='silu')
        if nbt:
            ts = torch.cumsum(torch.randint(1, 10 ** 5, (B, T), device=DEV, generator=g), 1)
            extra.update(timestamps=ts, rab_t=0.3 * torch.randn(H, nbt, device=DEV, generator=g))
    else:
        extra = dict(dropout_p=0.1, seed=1234)
    ktype = L.ATTN_HSTU if hstu else L.ATTN_SOFTMAX
    do = torch.randn(B * T, D, device=DEV, generator=g).bfloat16()
    jdo = torch.empty(cap, D, dtype=torch.bfloat16, device=DEV)
    K.gather_rows([(do, jdo)], jag.row_map)
    outs = []
    for jagged in (False, True):
        x = jpre if jagged else pre
        N = x.shape[0]
        a = K.attn_args(ktype, x[:, 2 * D:3 * D], x[:, 3 * D:], x[:, D:2 * D], B, T, H, hd, key_valid=kv,
                        scale=hd ** -0.5, out_dtype=torch.bfloat16, seq_range=jag.seq_range,
                        row_base=jag.row_base if jagged else None, **extra)
        sentinel = -7.0
        o = torch.full((N, D), sentinel, dtype=torch.bfloat16, device=DEV)
        lse = torch.empty(B, H, T, device=DEV) if not hstu else None
        K.attention_fwd(a, o, lse)
        dx = torch.full((N, 4 * D), sentinel, dtype=torch.bfloat16, device=DEV)
        delta = torch.empty(B, H, T, device=DEV) if not hstu else None
        drab = torch.zeros(H, T, device=DEV) if hstu else None
        drab_t = torch.zeros(H, nbt, device=DEV) if nbt else None
        K.attention_bwd(a, o if not hstu else None, jdo if jagged else do, lse, delta, dx[:, 2 * D:3 * D],
                        dx[:, 3 * D:], dx[:, D:2 * D], drab, drab_t=drab_t)
        outs.append((o, dx, drab, drab_t, lse, delta))
    rm = jag.row_map.cpu().numpy()
    live = rm >= 0
    (o0, dx0, dr0, dt0, l0, d0), (o1, dx1, dr1, dt1, l1, d1) = outs
    assert torch.equal(o1[torch.from_numpy(np.flatnonzero(live)).to(DEV)], o0[torch.from_numpy(rm[live]).to(DEV).long()])
    sel = torch.from_numpy(rm[live]).to(DEV).long()
    rows = torch.from_numpy(np.flatnonzero(live)).to(DEV)
    assert torch.equal(dx1[rows][:, D:], dx0[sel][:, D:])             # dv | dq | dk of every span row
    dead = ~torch.from_numpy(live).to(DEV)
    assert bool((o1[dead] == 0).all())                                # dead capacity rows: zeroed outputs
    assert bool((dx1[dead][:, D:] == 0).all()) and bool((dx1[dead][:, :D] == -7.0).all())   # u block untouched
    if hstu:
        assert torch.equal(dr0, dr1)
        if nbt:
            assert torch.equal(dt0, dt1)
    else:
        assert torch.equal(l0, l1)
        assert torch.equal(d0[kv.bool().unsqueeze(1).expand_as(d0)], d1[kv.bool().unsqueeze(1).expand_as(d1)])


def _model(cfg_kw, args_kw, seed=0):
    from tencent_recommendation_2025_amd import synthetic as S
    from tencent_recommendation_2025_amd.model import BaselineModel, init_reference_
    cfg = S.SyntheticConfig(**cfg_kw)
    stats, types = S.feature_schema(cfg)
    torch.manual_seed(seed)
    m = BaselineModel(cfg.num_users, cfg.num_items, stats, types, S.make_args(**args_kw)).to(DEV)
    init_reference_(m, seed=seed, live_norms=True)
    return m, cfg


@pytest.mark.parametrize('block', ['hstu', 'softmax'])
def test_jagged_encode_equals_padded_fp32(block):
    """fp32 (no autocast): the jagged encode's log_feats / pos / neg embeddings equal
    the padded ones on every span row (1e-6), the BCE loss to 1e-6, and the table and
    dense gradients to 1e-5 normwise (GEMM summation order over fewer rows)."""
    from tencent_recommendation_2025_amd import functional as G
    from tencent_recommendation_2025_amd import jagged as J
    from tencent_recommendation_2025_amd import synthetic as S
    from tencent_recommendation_2025_amd.optim import FusedAdamW
    res = []
    for jagged in (False, True):
        m, cfg = _model(dict(batch_size=12, maxlen=40, num_items=3000, num_users=300, min_len=3),
                        dict(hidden_units=64, maxlen=40, num_blocks=2, num_heads=2, block=block))
        opt = FusedAdamW(m, lr=1e-3, table_dtype=torch.float32)
        batch = S.make_batch(cfg, torch.Generator(device=DEV).manual_seed(5), DEV)
        seq, pos, neg, tt, ntt, _nat, sf, pf, nf = batch
        opt.zero_grad()
        opt.begin_step(batch)
        if jagged:
            jag = J.layout(tt, J.capacity_for(J.span_rows(tt), 64), ntt)
            jb = J.compact(batch, jag)
            h, pe, ne = m.encode(jb[0], jb[1], jb[2], jb[3], jb[6], jb[7], jb[8], jagged=jag, pos_idx=jb[10])
            loss = G.bce_loss(h, pe, ne, jb[4])
            rows = jag.row_map
        else:
            h, pe, ne = m.encode(seq, pos, neg, tt, sf, pf, nf)
            loss = G.bce_loss(h, pe, ne, ntt)
            rows = None
        loss.backward()
        grads = {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}
        for grp in opt.groups:
            grads['group.' + grp.name] = grp.dense_gradient().clone()
        res.append((h.detach(), pe.detach(), ne.detach(), loss.detach(), grads, rows))
    (h0, p0, n0, l0, g0, _), (h1, p1, n1, l1, g1, rm) = res
    live = rm >= 0
    sel = rm[live].long()
    D = h0.shape[-1]
    for a, b in ((h0, h1), (p0, p1), (n0, n1)):
        assert nrel(b.reshape(-1, D)[live].cpu(), a.reshape(-1, D)[sel].cpu()) < 1e-6
    assert abs(l0.item() - l1.item()) < 1e-6 * abs(l0.item())
    assert set(g0) == set(g1)
    # k_linear.bias: analytically zero gradient (softmax is shift-invariant), rounding noise only
    bad = {k: nrel(g1[k].cpu(), g0[k].cpu()) for k in g0
           if not k.endswith('k_linear.bias') and nrel(g1[k].cpu(), g0[k].cpu()) > 1e-5}
    assert not bad, bad


_TRAINER_CFG = (dict(batch_size=16, maxlen=60, num_items=4000, num_users=500, min_len=4),
                dict(hidden_units=128, maxlen=60, num_blocks=2, num_heads=2))


def _trainer_batches(cfg):
    """Three batches of the config plus one of short sequences (a second capacity bucket)."""
    from tencent_recommendation_2025_amd import synthetic as S
    g = torch.Generator(device=DEV).manual_seed(3)
    batches = [S.make_batch(cfg, g, DEV) for _ in range(3)]
    batches.append(S.make_batch(S.SyntheticConfig(**{**cfg.__dict__, 'min_len': 2}), g, DEV))
    return batches


def _one_step_grads(state, jagged, batch, quantum=128):
    """Loss and every gradient (dense parameters; each table group's dense row
    gradient) of ONE bf16-autocast trainer step from the parameters ``state``."""
    from tencent_recommendation_2025_amd.optim import FusedAdamW
    from tencent_recommendation_2025_amd.train import Trainer
    m, _ = _model(*_TRAINER_CFG)
    m.load_state_dict(state)
    opt = FusedAdamW(m, lr=1e-3, defer_period=4)
    tr = Trainer(m, opt, loss='bce', jagged=jagged, jagged_quantum=quantum)
    opt.zero_grad()
    opt.begin_step(batch)
    loss = tr.compute_loss(batch)
    loss.backward()
    if jagged:
        tr.check_jagged()
    grads = {n: p.grad.detach().float().clone() for n, p in m.named_parameters() if p.grad is not None}
    for grp in opt.groups:
        grads['group.' + grp.name] = grp.dense_gradient().float().clone()
    return float(loss), grads


# Per-step bounds of the bf16 jagged step against the padded one from identical
# parameters.  The dead rows contribute exact zeros and every span row sees the
# same inputs, so what can differ is (a) the order of the sums over rows (dW = dY^T X,
# LayerNorm gamma / beta, the row reductions of the tables) and (b), when the
# jagged capacity differs from B*T, which hipBLASLt kernel grk_gemm picks for the
# other row count -- each GEMM output is rounded to bf16, so another kernel's fp32
# summation order can move an output by one bf16 ulp.  Measured on MI355X
# (round 4; scripts/diag/jagged_vs_padded.py): with the capacity rounded to 128
# rows, loss bitwise, every gradient of every span row bitwise, parameters 1e-7
# .. 4e-4 -- in another process (other GEMM kernels picked) up to 2.7e-3.  The
# largest are the dnn weights whose sums over tokens mix pos-item and neg-item
# terms of opposite sign (BCE at logits near 0): the sum is far smaller than its
# terms, so any reordering is amplified.  fp32 (no bf16 rounding at all) pins
# every gradient at 1e-5: test_jagged_encode_equals_padded_fp32.
#   capacity == B*T (same GEMM shapes, so the same kernels): every parameter 1e-5
#     normwise except the cancellation-dominated dnn / feature-table sums (1e-3);
#   the bench's capacity rounding (128 rows here): every parameter 5e-3, and the loss
#   5e-5: the forward GEMMs of another row count may run other hipBLASLt kernels (the
#   timed plan choice also varies by process), each output one bf16 ulp
#   apart -- bitwise in most runs, 1.46e-5 once in round 6 (gpurun_out/r6x, after 5
#   steps, capacity 512) with every gradient inside its 5e-3.
JAGGED_STEP_TOL = dict(loss=1e-5, loss_capacity=5e-5, grad_same=1e-5, grad_sums=1e-3, grad_capacity=5e-3)
DNN_SUMS = ('itemdnn.', 'userdnn.', 'emb_transform.', 'group.small', 'group.item', 'group.user')


def test_jagged_step_matches_padded_from_identical_parameters():
    """bf16 autocast HSTU (the bench's regime), dropout 0: from the SAME parameters,
    one jagged step's loss and every gradient against the padded step's, at the
    initial parameters and after 2 and 5 padded training steps, on batches of two
    capacity buckets (reference loop: model/BaseLine/main.py:177-185); once with
    capacity B*T (same GEMM shapes) and once with the bench's capacity rounding."""
    from tencent_recommendation_2025_amd import jagged as J
    from tencent_recommendation_2025_amd.optim import FusedAdamW
    from tencent_recommendation_2025_amd.train import Trainer
    m, cfg = _model(*_TRAINER_CFG)
    batches = _trainer_batches(cfg)
    tr = Trainer(m, FusedAdamW(m, lr=1e-3, defer_period=4), loss='bce')
    done = 0
    bad = {}
    for trained, probe in ((0, 0), (2, 3), (5, 1)):
        while done < trained:
            tr.step(batches[done % 4])
            done += 1
        state = {k: v.detach().clone() for k, v in m.state_dict().items()}   # flushes deferred rows
        batch = batches[probe]
        B, T = batch[0].shape
        lp, gp = _one_step_grads(state, False, batch)
        for name, quantum in (('same', B * T), ('capacity', 128)):
            lj, gj = _one_step_grads(state, True, batch, quantum=quantum)
            assert set(gp) == set(gj)
            errs = {k: nrel(gj[k].cpu(), gp[k].cpu()) for k in gp}
            loss_err = abs(lj - lp) / abs(lp)
            top = sorted(errs, key=lambda k: -errs[k])[:5]
            print(f'after {trained} steps, batch {probe}, {name} (capacity '
                  f'{J.capacity_for(J.span_rows(batch[3]), quantum)}): loss {loss_err:.2e}',
                  [(k, f'{errs[k]:.2e}') for k in top])
            if loss_err > JAGGED_STEP_TOL['loss_capacity' if name == 'capacity' else 'loss']:
                bad[(trained, name, 'loss')] = loss_err
            for k, v in errs.items():
                tol = (JAGGED_STEP_TOL['grad_capacity'] if name == 'capacity' else
                       JAGGED_STEP_TOL['grad_sums'] if k.startswith(DNN_SUMS) else JAGGED_STEP_TOL['grad_same'])
                if v > tol:
                    bad[(trained, name, k)] = v
    assert not bad, bad


def test_jagged_trainer_graph_replay_is_bitwise_and_tracks_padded():
    """The jagged step replayed from HIP graphs of two capacities == the eager jagged
    step, bitwise (losses and every parameter over 8 steps).  The padded trainer's
    8-step loss trajectory is reported beside it, held only to 5e-3: AdamW's first
    steps move every parameter by ~lr * sign(g), so a gradient element that is
    rounding noise in either run (e.g. an analytically zero one) moves by +-lr and
    the trajectories separate by design; per-step parity is the test above."""
    from tencent_recommendation_2025_amd import jagged as J
    from tencent_recommendation_2025_amd.optim import FusedAdamW
    from tencent_recommendation_2025_amd.train import Trainer
    runs = {}
    for name, jagged, graph in (('padded', False, False), ('jagged', True, False), ('jagged_graph', True, True)):
        m, cfg = _model(*_TRAINER_CFG)
        tr = Trainer(m, FusedAdamW(m, lr=1e-3, defer_period=4), loss='bce', graph=graph, graph_warmup=1,
                     jagged=jagged, jagged_quantum=128)
        batches = _trainer_batches(cfg)
        rows = [J.span_rows(b[3]) for b in batches]
        losses = [tr.step(batches[i % 4], rows=rows[i % 4] if jagged else None).clone() for i in range(8)]
        if graph:
            assert len(tr._graphs) >= 2, tr._graphs.keys()
        if jagged:
            tr.check_jagged()
        runs[name] = (torch.stack(losses), m.state_dict())
    lp, lj, lg = runs['padded'][0], runs['jagged'][0], runs['jagged_graph'][0]
    assert torch.equal(lj, lg), (lj, lg)
    for k in runs['jagged'][1]:
        assert torch.equal(runs['jagged'][1][k], runs['jagged_graph'][1][k]), k
    rel = ((lj - lp).abs() / lp.abs())
    print('8-step loss trajectory, jagged vs padded (rel):', [f'{x:.1e}' for x in rel.tolist()])
    assert rel.max().item() < 5e-3, (lp, lj)


def test_understated_rows_raise_instead_of_addressing_past_capacity():
    """a caller that under-states the batch's span rows gets a ValueError
    (err bit 2 checked after the eager step), and no kernel touches a row past the
    capacity (the layout drops the trailing spans)."""
    from tencent_recommendation_2025_amd import jagged as J
    from tencent_recommendation_2025_amd.optim import FusedAdamW
    from tencent_recommendation_2025_amd.train import Trainer
    m, cfg = _model(*_TRAINER_CFG)
    batch = _trainer_batches(cfg)[0]
    n = J.span_rows(batch[3])
    assert n > 256
    tr = Trainer(m, FusedAdamW(m, lr=1e-3), loss='bce', jagged=True, jagged_quantum=128)
    with pytest.raises(ValueError, match='more span rows'):
        tr.step(batch, rows=n // 2)
    assert tr._cap is None
    torch.cuda.synchronize()
    # a direct compute_loss call after a step recomputes the capacity (no stale _cap)
    tr2 = Trainer(m, FusedAdamW(m, lr=1e-3), loss='bce', jagged=True, jagged_quantum=128)
    tr2.step(batch, rows=n)
    small = _trainer_batches(cfg)[3]
    loss = tr2.compute_loss(small)
    assert torch.isfinite(loss).all()
    tr2.check_jagged()


def test_merged_projection_backward_matches_and_replays_bitwise():
    """args.merge_proj_backward (functional.DenseMerge): the projected tables' row
    gradients of the seq-side and pair lookups in ONE chunked call -- bf16 trainer
    losses within the bench tolerance (1e-3) of the per-lookup calls over 6 steps
    (the chunk order differs, so not bitwise), and the merged step replayed from
    HIP graphs == its eager step, bitwise."""
    from tencent_recommendation_2025_amd import jagged as J
    from tencent_recommendation_2025_amd import kernels as K
    from tencent_recommendation_2025_amd import synthetic as S
    from tencent_recommendation_2025_amd.optim import FusedAdamW
    from tencent_recommendation_2025_amd.train import Trainer
    runs = {}
    for name, merge, graph in (('split', False, False), ('merged', True, False), ('merged_graph', True, True)):
        m, cfg = _model(dict(batch_size=16, maxlen=60, num_items=4000, num_users=500, min_len=4),
                        dict(hidden_units=128, maxlen=60, num_blocks=2, num_heads=2, merge_proj_backward=merge))
        tr = Trainer(m, FusedAdamW(m, lr=1e-3, defer_period=4), loss='bce', graph=graph, graph_warmup=1,
                     jagged=True, jagged_quantum=128)
        g = torch.Generator(device=DEV).manual_seed(3)
        batches = [S.make_batch(cfg, g, DEV) for _ in range(3)]
        rows = [J.span_rows(b[3]) for b in batches]
        K.BACKWARD_TRACE = [] if name == 'merged' else None
        losses = [tr.step(batches[i % 3], rows=rows[i % 3]).clone() for i in range(6)]
        if name == 'merged':
            chunked = [c for c in K.BACKWARD_TRACE if c.get('chunked')]
            K.BACKWARD_TRACE = None
            assert len(chunked) == 6, len(chunked)        # one chunked call per step
        runs[name] = (torch.stack(losses), m.state_dict())
    ls, lm, lg = runs['split'][0], runs['merged'][0], runs['merged_graph'][0]
    assert ((lm - ls).abs() / ls.abs()).max().item() < 1e-3, (ls, lm)
    assert torch.equal(lm, lg), (lm, lg)
    for k in runs['merged'][1]:
        assert torch.equal(runs['merged'][1][k], runs['merged_graph'][1][k]), k


def test_packed_batches_replay_equals_unpacked():
    """Graph replays fed arena-packed batches (train.pack_batch: the input copy is one
    launch) give the same losses and parameters, bit for bit, as replays fed the
    plain batches (a multi-tensor copy per dtype) -- jagged rows, two capacities."""
    from tencent_recommendation_2025_amd import jagged as J
    from tencent_recommendation_2025_amd import synthetic as S
    from tencent_recommendation_2025_amd.model import BaselineModel
    from tencent_recommendation_2025_amd.optim import FusedAdamW
    from tencent_recommendation_2025_amd.train import Trainer, pack_batch
    cfg = S.SyntheticConfig(batch_size=8, maxlen=40, num_items=2000, num_users=300, min_len=4)
    short = S.SyntheticConfig(**{**cfg.__dict__, 'min_len': 2})
    stats, types = S.feature_schema(cfg)
    args = S.make_args(hidden_units=64, maxlen=40, num_blocks=1, num_heads=2)
    runs = []
    for packed in (False, True):
        torch.manual_seed(0)
        m = BaselineModel(cfg.num_users, cfg.num_items, stats, types, args).to(DEV)
        tr = Trainer(m, FusedAdamW(m, lr=1e-3), loss='bce', graph=True, graph_warmup=1, jagged=True,
                     jagged_quantum=64)
        g = torch.Generator(device=DEV).manual_seed(5)
        pool = [S.make_batch(cfg, g, DEV), S.make_batch(short, g, DEV), S.make_batch(cfg, g, DEV)]
        if packed:
            pool = [pack_batch(b) for b in pool]
        rows = [J.span_rows(b[3]) for b in pool]
        losses = torch.stack([tr.step(pool[i % 3], rows=rows[i % 3]).clone() for i in range(9)])
        torch.cuda.synchronize()
        runs.append((losses, {k: v.clone() for k, v in m.state_dict().items()}))
    assert torch.equal(runs[0][0], runs[1][0])
    for k in runs[0][1]:
        assert torch.equal(runs[0][1][k], runs[1][1][k]), k


def test_compact_lays_pos_neg_pairs_out_adjacent():
    """jagged.compact puts pos / neg ids and each pos / neg feature of one shape into
    the halves of one buffer (round 4), so feat2emb_pair stacks them as a view: the
    stacked tensors share the buffer and equal the copying stack."""
    from tencent_recommendation_2025_amd import jagged as J
    from tencent_recommendation_2025_amd import model as Mm
    from tencent_recommendation_2025_amd import synthetic as S
    cfg = S.SyntheticConfig(batch_size=8, maxlen=40, num_items=500, num_users=50, min_len=4)
    gen = torch.Generator(device=DEV).manual_seed(5)
    batch = S.make_batch(cfg, gen, DEV)
    tt = batch[3]
    jag = J.layout(tt, J.capacity_for(J.span_rows(tt), 64), batch[4])
    jb = J.compact(batch, jag)
    pos, neg = jb[1], jb[2]
    v = Mm._adjacent(pos.reshape(1, -1), neg.reshape(1, -1))
    assert v is not None and torch.equal(Mm._cat0(pos, neg), torch.cat([pos, neg], 0))
    pf, nf = jb[7], jb[8]
    fids = sorted(set(pf) & set(nf))
    assert fids
    st = Mm._stack_pairs(pf, nf, fids)
    for k in fids:
        assert torch.equal(st[k], torch.cat([pf[k], nf[k]], 0)), k
        if pf[k].shape[1:] == nf[k].shape[1:] and pf[k].dtype == nf[k].dtype:
            assert st[k].data_ptr() == pf[k].data_ptr(), k     # a view, no copy
