"""Host-side helpers of the fused step (CPU, no kernel launched).

* kernels.adamw_hparams -- the per-step constants every table AdamW kernel
  consumes (grk_optim.hip adam1: p *= 1 - lr wd; m += (1 - b1)(g - m);
  v = b2 v + (1 - b2) g^2; p -= step_size m / (sqrt(v) / bias_corr2_sqrt + eps)):
  restated here in fp32 numpy with those constants over several steps, it
  tracks torch.optim.AdamW (model/BaseLine/main.py:131,189, betas (0.9, 0.98)).
* jagged.span_rows / capacity_for -- the host metadata that picks the jagged
  step's capacity (and with it the GEMM plans and the captured graph)."""
import numpy as np
import pytest
import torch

from tencent_recommendation_2025_amd import jagged as J
from tencent_recommendation_2025_amd import kernels as K


def adam1(p, m, v, g, hp):
    """grk_optim.hip adam1 in fp32 (IEEE sqrt / division where the kernel uses the
    1-ulp hardware forms)."""
    f = np.float32
    pe = p * f(1.0 - f(hp.lr) * f(hp.weight_decay))
    me = m + f(1.0 - f(hp.beta1)) * (g - m)
    ve = v * f(hp.beta2) + f(1.0 - f(hp.beta2)) * g * g
    denom = np.sqrt(ve) * f(1.0 / f(hp.bias_corr2_sqrt)) + f(hp.eps)
    return pe - f(hp.step_size) * (me / denom), me, ve


@pytest.mark.parametrize('wd', [0.0, 0.01])
def test_adamw_hparams_track_torch_adamw(wd):
    rng = np.random.default_rng(0)
    p0 = rng.standard_normal(4096).astype(np.float32)
    grads = [rng.standard_normal(4096).astype(np.float32) * s for s in (1.0, 1e-3, 0.0, 3.0, 1e-6)]
    lr, b1, b2, eps = 1e-3, 0.9, 0.98, 1e-8
    tp = torch.nn.Parameter(torch.from_numpy(p0.copy()))
    opt = torch.optim.AdamW([tp], lr=lr, betas=(b1, b2), eps=eps, weight_decay=wd)
    p, m, v = p0.copy(), np.zeros_like(p0), np.zeros_like(p0)
    for t, g in enumerate(grads, start=1):
        hp = K.adamw_hparams(lr, b1, b2, eps, wd, t)
        assert hp.step_size == pytest.approx(lr / (1 - b1 ** t), rel=1e-6)
        assert hp.bias_corr2_sqrt == pytest.approx((1 - b2 ** t) ** 0.5, rel=1e-6)
        p, m, v = adam1(p, m, v, g, hp)
        tp.grad = torch.from_numpy(g.copy())
        opt.step()
        st = opt.state[tp]
        # torch forms m with lerp (its own rounding of m + w (g - m)): ulps of max |m|
        np.testing.assert_allclose(m, st['exp_avg'].numpy(), rtol=1e-6, atol=1e-6 * np.abs(m).max())
        np.testing.assert_allclose(v, st['exp_avg_sq'].numpy(), rtol=1e-5, atol=1e-6 * np.abs(v).max())
        # the update term is ~lr: a few fp32 ulp of it on top of p's own rounding
        np.testing.assert_allclose(p, tp.detach().numpy(), rtol=0, atol=4e-8 + 2e-7 * np.abs(p).max())


def test_span_rows_and_capacity():
    T = 9
    tt = torch.zeros(4, T, dtype=torch.int64)
    starts = [0, 4, 9, 8]                        # full, partial, empty, one token
    for b, s0 in enumerate(starts):
        tt[b, s0:] = 1
    assert J.span_rows(tt) == sum(T - s0 for s0 in starts)
    tt[1, 6] = 0                                 # a hole inside a span still counts (span = [first, T))
    assert J.span_rows(tt) == sum(T - s0 for s0 in starts)
    assert J.capacity_for(0) == 1024 and J.capacity_for(1) == 1024 and J.capacity_for(1024) == 1024
    assert J.capacity_for(1025) == 2048 and J.capacity_for(13670) == 14336
    assert J.capacity_for(5000, 1024, limit=4096) == 4096
    assert J.capacity_for(100, 128) == 128


def test_device_clock_advances_on_its_device():
    clk = K.DeviceClock(16, torch.device('cpu'))
    assert clk.ring.shape[0] == 16 and int(clk.t.item()) == 0
    clk.advance()
    clk.advance()
    assert int(clk.t.item()) == 2


def test_dense_flat_layout_and_grad_runs():
    """optim.DenseFlat's host logic: parameters packed back to back as [rows, 8]
    (sizes multiples of 8, refused otherwise), and the multi-range update launched
    per maximal run of consecutive parameters that all have a gradient (torch's
    AdamW skips a parameter without one; k_adamw_ranges moves every row it covers)."""
    from tencent_recommendation_2025_amd.optim import flat_layout, grad_runs
    starts, rows = flat_layout([16, 8, 64, 24])
    assert starts == [0, 2, 3, 11] and rows == 14
    with pytest.raises(ValueError):
        flat_layout([16, 12])
    ends = [2, 3, 11, 14]
    assert grad_runs(starts, ends, [True] * 4) == [(0, 14, [0, 1, 2, 3])]
    assert grad_runs(starts, ends, [True, False, True, True]) == [(0, 2, [0]), (3, 14, [2, 3])]
    assert grad_runs(starts, ends, [False, False, False, False]) == []
    assert grad_runs(starts, ends, [False, True, True, False]) == [(2, 11, [1, 2])]


@pytest.mark.parametrize('dt', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('m', [0, 32, 7])
def test_operand_extras_equal_the_cat_pad_form(dt, m):
    """The dnn operand's dense columns (model._embed.operand): the mm features copied as
    they are plus one broadcast [1, 0, ...] row (functional.write_extras) write the same
    bytes as the round-3 form -- cat(mm, ones), zero-padded to a multiple of 8, cast,
    copied -- for fp32 and bf16 gather buffers."""
    import torch.nn.functional as F
    from tencent_recommendation_2025_amd import functional as G
    from tencent_recommendation_2025_amd.model import _unit_row
    N, col = 37, 16
    g = torch.Generator().manual_seed(m)
    dense = [torch.randn(N, m, generator=g) * 3] if m else []
    old = torch.full((N, 64), 7.0, dtype=dt)
    x = torch.cat(dense + [torch.ones(N, 1)], 1)
    pad = (-x.shape[1]) % 8
    x = F.pad(x, (0, pad)) if pad else x
    old[:, col:col + x.shape[1]] = x.to(dt)
    new = torch.full((N, 64), 7.0, dtype=dt)
    extras, c = [], col
    for t in dense:
        extras.append((c, t))
        c += t.shape[1]
    w = 1 + (-(sum(t.shape[1] for t in dense) + 1)) % 8
    extras.append((c, _unit_row(w, 'cpu')))
    c += w
    G.write_extras(new, extras)
    assert c - col == x.shape[1]
    assert torch.equal(old.view(torch.int16 if dt == torch.bfloat16 else torch.int32),
                       new.view(torch.int16 if dt == torch.bfloat16 else torch.int32))


def test_key_valid_bytes_and_jagged_positions():
    """bool -> uint8 by view (no cast kernel) and the cached position index equal the
    casting forms: key_valid bytes 0 / 1, pidx = (t + 1) where the token is valid."""
    from tencent_recommendation_2025_amd.jagged import _positions
    g = torch.Generator().manual_seed(1)
    tt = torch.randint(0, 3, (5, 11), generator=g, dtype=torch.int32)
    assert torch.equal((tt != 0).contiguous().view(torch.uint8), (tt != 0).to(torch.uint8))
    seq = torch.randint(0, 4, (5, 11), generator=g)
    want = (torch.arange(1, 12).unsqueeze(0) * (seq != 0)).to(torch.int64)
    got = torch.where(seq != 0, _positions(11, 'cpu'), 0)
    assert got.dtype == torch.int64 and torch.equal(got, want)


def test_pair_split_backward_equals_slices():
    """feat2emb_pair returns x.split(B) (backward: one cat of the two gradients) where it
    returned x[:B], x[B:] (backward: a zero-filled full-size gradient per slice, added):
    same views forward, same gradient bits, fewer kernels."""
    import collections
    from torch.utils._python_dispatch import TorchDispatchMode

    class Ops(TorchDispatchMode):
        def __init__(self):
            super().__init__()
            self.n = collections.Counter()

        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            self.n[str(func.overloadpacket)] += 1
            return func(*args, **(kwargs or {}))

    g = torch.Generator().manual_seed(2)
    x0 = torch.randn(2, 7, 16, generator=g).bfloat16()
    ga, gb = torch.randn(1, 7, 16, generator=g).bfloat16(), torch.randn(1, 7, 16, generator=g).bfloat16()
    res = []
    for form in ('slices', 'split'):
        x = x0.clone().requires_grad_(True)
        y = x * 1                                     # a non-leaf, as the dnn output is
        a, b = (y[:1], y[1:]) if form == 'slices' else y.split(1, 0)
        ops = Ops()
        with ops:
            torch.autograd.backward([a, b], [ga, gb])
        res.append((x.grad.clone(), ops.n))
    assert torch.equal(res[0][0], res[1][0])
    assert 'aten.slice_backward' in res[0][1] and 'aten.slice_backward' not in res[1][1]


def _stub_adamw_ranges(monkeypatch, O, fn):
    """DenseFlat plans its launches (K.prepare_table_adamw_ranges) and runs them
    (K.launch_prepared): both stubbed so that each launch calls fn with the plan's
    arguments at launch time, as the device would read them."""
    monkeypatch.setattr(O.K, 'prepare_table_adamw_ranges',
                        lambda param, m, v, clock, ranges, shadow=None: (param, m, v, clock, ranges, shadow))
    monkeypatch.setattr(O.K, 'launch_prepared', lambda call: fn(*call))


def test_dense_flat_step_plumbing_tracks_torch_adamw(monkeypatch):
    """optim.DenseFlat on the CPU with grk_table_adamw_ranges_dev emulated by the element
    update restated above (adam1): parameters become views of the flat buffer (the
    Parameter objects stay), each gradient lands on its own rows, a parameter without a
    gradient is skipped for that step (torch's rule; the kernel would move every row it
    covers), and several steps track torch.optim.AdamW parameter by parameter."""
    from tencent_recommendation_2025_amd import optim as O
    lr, b1, b2, eps, wd = 1e-3, 0.9, 0.98, 1e-8, 0.01
    calls = []

    class Clock:
        t = 0

    def emulated(param, exp_avg, exp_avg_sq, clock, ranges, shadow=None):
        hp = K.adamw_hparams(lr, b1, b2, eps, wd, clock.t)
        assert len(ranges) <= K.MAX_GRAD_RANGES          # the kernel refuses more (kMaxGradRanges)
        calls.append(param.shape[0])
        g = np.zeros(param.shape, np.float32)
        for off, gr in ranges:
            g[off:off + gr.shape[0]] = gr.float().numpy()
        p, m, v = adam1(param.numpy(), exp_avg.numpy(), exp_avg_sq.numpy(), g, hp)
        param.copy_(torch.from_numpy(p))
        exp_avg.copy_(torch.from_numpy(m))
        exp_avg_sq.copy_(torch.from_numpy(v))

    _stub_adamw_ranges(monkeypatch, O, emulated)
    gen = torch.Generator().manual_seed(5)
    shapes = [(16, 8), (24,), (4, 6, 2), (8,), (40, 16)]
    ps = [torch.nn.Parameter(torch.randn(s, generator=gen)) for s in shapes]
    twins = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    flat = O.DenseFlat(ps, 'cpu')
    assert all(flat.buf.data_ptr() <= p.data_ptr() < flat.buf.data_ptr() + flat.buf.numel() * 4 for p in ps)
    assert all(torch.equal(p.detach(), q.detach()) for p, q in zip(ps, twins))
    ref = torch.optim.AdamW(twins, lr=lr, betas=(b1, b2), eps=eps, weight_decay=wd)
    clock = Clock()
    skip = {2: {2}, 4: {0, 4}}                      # step -> parameters without a gradient
    skipped = set()
    for step in range(1, 8):
        clock.t = step
        before = [p.detach().clone() for p in ps]
        for i, (p, q) in enumerate(zip(ps, twins)):
            if i in skip.get(step, ()):
                p.grad = q.grad = None
            else:
                g = torch.randn(p.shape, generator=gen) * (1e-3 if i == 1 else 1.0)
                if step >= 6:   # gradients written in place: step 5's launch plan is reused
                    p.grad.copy_(g)
                    q.grad.copy_(g)
                else:
                    p.grad, q.grad = g.clone(), g.clone()
        calls.clear()
        flat.step(clock)
        ref.step()
        assert len(calls) == len(O.split_runs(O.grad_runs(flat.starts, flat.ends, [p.grad is not None for p in ps]),
                                              flat.starts, flat.ends, K.MAX_GRAD_RANGES))
        for i, (p, q) in enumerate(zip(ps, twins)):
            if i in skip.get(step, ()):
                assert torch.equal(p.detach(), before[i])   # no gradient: not moved this step
                skipped.add(i)
            elif i not in skipped:
                # (after a skipped step torch counts that parameter's steps apart -- its own bias
                # correction -- where the clock's step is global: DESIGN.md §3c, dense_flat)
                np.testing.assert_allclose(p.detach().numpy(), q.detach().numpy(), rtol=0,
                                           atol=4e-8 + 2e-7 * float(q.detach().abs().max()))
    assert skipped == {0, 2, 4}
    assert flat._prep_key is not None and len(flat._prepared) == 1   # the plan kept since step 5
    st = flat.state(ps[1])
    np.testing.assert_allclose(st['exp_avg'].numpy(), ref.state[twins[1]]['exp_avg'].numpy(), rtol=1e-5, atol=1e-9)


def test_dense_flat_splits_runs_beyond_the_kernel_range_cap(monkeypatch):
    """a run of more than kMaxGradRanges (64) parameters with gradients -- the
    softmax-block model's ~70 dense parameters -- is cut into launches of at most 64
    ranges, each over contiguous rows, and every parameter still takes exactly its
    torch AdamW update."""
    from tencent_recommendation_2025_amd import optim as O
    lr, b1, b2, eps, wd = 1e-3, 0.9, 0.98, 1e-8, 0.01
    calls = []

    class Clock:
        t = 1

    def emulated(param, exp_avg, exp_avg_sq, clock, ranges, shadow=None):
        assert len(ranges) <= K.MAX_GRAD_RANGES
        calls.append(len(ranges))
        hp = K.adamw_hparams(lr, b1, b2, eps, wd, clock.t)
        g = np.zeros(param.shape, np.float32)
        for off, gr in ranges:
            assert 0 <= off and off + gr.shape[0] <= param.shape[0]
            g[off:off + gr.shape[0]] = gr.float().numpy()
        p, m, v = adam1(param.numpy(), exp_avg.numpy(), exp_avg_sq.numpy(), g, hp)
        param.copy_(torch.from_numpy(p))
        exp_avg.copy_(torch.from_numpy(m))
        exp_avg_sq.copy_(torch.from_numpy(v))

    _stub_adamw_ranges(monkeypatch, O, emulated)
    gen = torch.Generator().manual_seed(9)
    ps = [torch.nn.Parameter(torch.randn((8 * (1 + i % 3),), generator=gen)) for i in range(150)]
    twins = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    flat = O.DenseFlat(ps, 'cpu')
    ref = torch.optim.AdamW(twins, lr=lr, betas=(b1, b2), eps=eps, weight_decay=wd)
    for p, q in zip(ps, twins):
        g = torch.randn(p.shape, generator=gen)
        p.grad, q.grad = g.clone(), g.clone()
    flat.step(Clock())
    ref.step()
    assert calls == [64, 64, 22]
    for p, q in zip(ps, twins):
        np.testing.assert_allclose(p.detach().numpy(), q.detach().numpy(), rtol=0,
                                   atol=4e-8 + 2e-7 * float(q.detach().abs().max()))


def test_valid_bytes_eager_and_compiled():
    """model._valid_bytes: the key-valid bytes of a token_type batch -- a bool -> uint8
    view in eager mode, a cast when traced (round 4: inductor cannot lower the dtype view
    of a bool tensor, which broke the reference's --use_torch_compile path)."""
    from tencent_recommendation_2025_amd import model as M
    tt = torch.tensor([[0, 0, 2, 1, 1], [0, 1, 1, 0, 1]], dtype=torch.int64)
    want = (tt != 0).to(torch.uint8)
    assert torch.equal(M._valid_bytes(tt), want)
    got = torch.compile(lambda t: M._valid_bytes(t) + 0, backend='inductor', fullgraph=True)(tt)
    assert got.dtype == torch.uint8 and torch.equal(got, want)


def test_pack_batch_one_arena_same_values():
    """train.pack_batch: every tensor of a collate-shaped batch (tuple fields, feature
    dicts, mixed dtypes) becomes a view of one byte arena with the same values,
    dtypes and shapes; a clone has the same layout, and copying one arena into the
    other's is the whole batch copy a graph replay does (one launch)."""
    from tencent_recommendation_2025_amd import synthetic as S
    from tencent_recommendation_2025_amd import train as T
    cfg = S.SyntheticConfig(batch_size=4, maxlen=12, num_items=300, num_users=40, min_len=3)
    b1 = S.make_batch(cfg, torch.Generator().manual_seed(1), 'cpu')
    b2 = S.make_batch(cfg, torch.Generator().manual_seed(2), 'cpu')
    p1, p2 = T.pack_batch(b1), T.pack_batch(b2)
    assert isinstance(p1, T.PackedBatch) and p1.layout == p2.layout
    for a, b in zip(T._tensors(p1), T._tensors(b1)):
        assert a.dtype == b.dtype and a.shape == b.shape and torch.equal(a, b)
        assert a.untyped_storage().data_ptr() == p1.arena.untyped_storage().data_ptr()
    st = T._clone_batch(p1)
    assert isinstance(st, T.PackedBatch) and st.layout == p1.layout and st.arena.data_ptr() != p1.arena.data_ptr()
    st.arena.copy_(p2.arena)
    for a, b in zip(T._tensors(st), T._tensors(b2)):
        assert torch.equal(a, b)
    assert isinstance(st[6], dict) and set(st[6]) == set(b2[6])


def test_stack_pairs_is_a_view_for_adjacent_halves():
    """model._stack_pairs / _cat0 (round 4): pos / neg tensors that are the two
    halves of one buffer stack as a view of it; anything else is copied as before."""
    from tencent_recommendation_2025_amd import model as Mm
    buf = torch.arange(2 * 3 * 5 * 4).reshape(6, 5, 4)
    a, b = buf[:3], buf[3:]
    other = buf[3:].clone()
    st = Mm._stack_pairs({'x': a, 'y': a}, {'x': b, 'y': other}, ['x', 'y'])
    assert st['x'].data_ptr() == buf.data_ptr() and torch.equal(st['x'], buf)
    assert st['y'].data_ptr() != buf.data_ptr() and torch.equal(st['y'], buf)
    assert Mm._adjacent(b, a) is None                       # wrong order
    assert Mm._adjacent(buf[:2], buf[3:]) is None           # a gap
    assert torch.equal(Mm._cat0(buf[:2], buf[3:]), torch.cat([buf[:2], buf[3:]]))


def test_split_pair_joins_adjacent_gradients_without_a_copy():
    """functional.split_pair (round 4): forward = x[:n], x[n:]; backward returns the two
    gradient halves as one view when they are adjacent, a cat otherwise -- same values
    as torch's split either way."""
    from tencent_recommendation_2025_amd import functional as G
    x = torch.randn(6, 3, requires_grad=True)
    a, b = G.split_pair(x, 2)
    assert torch.equal(a, x[:2]) and torch.equal(b, x[2:])
    buf = torch.randn(6, 3)
    (a * buf[:2]).sum().backward(retain_graph=True)   # gb None: zeros for the second half
    assert torch.equal(x.grad, torch.cat([buf[:2], torch.zeros(4, 3)]))
    x.grad = None
    ga, gb = buf[:2], buf[2:]
    gx, = torch.autograd.grad((a, b), (x,), (ga, gb))
    assert torch.equal(gx, buf) and gx.data_ptr() == buf.data_ptr()     # a view of the joint buffer
    gx, = torch.autograd.grad((a, b), (x,), (ga.clone(), gb.clone()))
    assert torch.equal(gx, buf)


def test_dense_flat_shadow_registry_does_not_keep_parameters_alive():
    """the bf16-shadow registry held each DenseFlat (and through it
    the Parameters, the flat buffer, both moments and the shadow) for the life of the
    process.  Dropping the parameters and the DenseFlat must free them and clear
    their registry entries."""
    import gc
    import weakref
    from tencent_recommendation_2025_amd import functional as G
    from tencent_recommendation_2025_amd import optim as O
    ps = [torch.nn.Parameter(torch.randn(4, 8)), torch.nn.Parameter(torch.randn(16))]
    keys = [id(p) for p in ps]
    flat = O.DenseFlat(ps, 'cpu', shadow=True)
    assert all(k in G._SHADOWS for k in keys)
    assert torch.equal(G.bf16_shadow(ps[0]), ps[0].detach().bfloat16())
    wp, wf = weakref.ref(ps[0]), weakref.ref(flat)
    del ps, flat
    gc.collect()
    assert wp() is None and wf() is None
    assert not any(k in G._SHADOWS for k in keys)


def test_dense_flat_shadow_follows_writes_outside_the_optimizer():
    """the bf16 shadow tracks in-place writes to a parameter (its own version
    counter) and writes through the flat buffer or any view of it (the counter the
    views share); writes through ``p.data`` need sync_shadow(force=True).  A refresh
    never bumps the counter the shadow views share, so a shadow view saved for
    backward before the refresh stays usable."""
    from tencent_recommendation_2025_amd import functional as G
    from tencent_recommendation_2025_amd import optim as O
    ps = [torch.nn.Parameter(torch.randn(4, 8)), torch.nn.Parameter(torch.randn(2, 8))]
    flat = O.DenseFlat(ps, 'cpu', shadow=True)
    s1 = G.bf16_shadow(ps[1])
    saved_version = s1._version
    with torch.no_grad():
        ps[0].mul_(3.0)                                    # in place on the parameter
    assert torch.equal(G.bf16_shadow(ps[0]), ps[0].detach().bfloat16())
    flat.buf[4:6].add_(1.0)                                # through the flat buffer (= ps[1]'s rows)
    assert torch.equal(G.bf16_shadow(ps[1]), ps[1].detach().bfloat16())
    ps[1].data.copy_(torch.full((2, 8), 0.25))             # invisible to version counters ...
    flat.sync_shadow(force=True)                           # ... hence the explicit refresh
    assert torch.equal(G.bf16_shadow(ps[1]), torch.full((2, 8), 0.25, dtype=torch.bfloat16))
    assert s1._version == saved_version                    # refreshes did not bump the shared counter
