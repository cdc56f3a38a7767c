"""GPU check of the row-sharded optimizer path in one process (world size 1,
RCCL): ShardedFusedAdamW must train exactly like FusedAdamW (same model,
same batches), i.e. the fetch/push/owner-reduction plumbing is an identity
at G = 1.  Multi-rank equivalence is covered by tests/test_sharding_gloo.py
(CPU) and the gloo rehearsal in scripts/rehearse_multirank.sh."""
import os
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu
DEV = 'cuda'


@pytest.fixture(scope='module')
def pg():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('nccl', rank=0, world_size=1, device_id=torch.device(DEV, 0))
    yield None
    dist.destroy_process_group()


def build(seed=0):
    from tencent_recommendation_2025_amd import synthetic as S
    from tencent_recommendation_2025_amd.model import BaselineModel, init_reference_
    cfg = S.SyntheticConfig(batch_size=8, maxlen=40, num_items=3000, num_users=400, min_len=8)
    stats, types = S.feature_schema(cfg)
    torch.manual_seed(seed)
    m = BaselineModel(cfg.num_users, cfg.num_items, stats, types,
                      S.make_args(hidden_units=64, maxlen=40, num_blocks=2, num_heads=2)).to(DEV)
    init_reference_(m, seed=seed, live_norms=True)
    return m, cfg


def test_sharded_optimizer_world1_equals_fused(pg):
    from tencent_recommendation_2025_amd import synthetic as S
    from tencent_recommendation_2025_amd.optim import FusedAdamW
    from tencent_recommendation_2025_amd.sharding import ShardedFusedAdamW
    from tencent_recommendation_2025_amd.train import Trainer
    m1, cfg = build()
    m2, _ = build()
    # both on the flat multi-range AdamW for the dense parameters (the sharded one after its
    # bucketed all-reduce)
    t1 = Trainer(m1, FusedAdamW(m1, lr=2e-3, table_dtype=torch.float32, defer_period=2), loss='bce',
                 amp_dtype=None)
    t2 = Trainer(m2, ShardedFusedAdamW(m2, lr=2e-3, table_dtype=torch.float32, defer_period=2), loss='bce', amp_dtype=None)
    g = torch.Generator(device=DEV).manual_seed(0)
    batches = [S.make_batch(cfg, g, DEV) for _ in range(5)]
    for b in batches:
        l1 = t1.step(b)
        l2 = t2.step(b)
        assert abs(l1.item() - l2.item()) < 1e-4 * max(1.0, abs(l1.item()))
    s1, s2 = m1.state_dict(), m2.state_dict()
    for k in s1:
        if k in ('item_emb.weight', 'user_emb.weight'):
            continue  # held as shards by the sharded optimizer
        torch.testing.assert_close(s1[k].float(), s2[k].float(), rtol=1e-3, atol=2e-5, msg=k)
    # the shards (deferred rows flushed) == the fused optimizer's full tables at G = 1
    for k in ('item_emb', 'user_emb'):
        torch.testing.assert_close(t2.opt.shard_table(k).float(), s1[f'{k}.weight'].float(), rtol=1e-3, atol=2e-5,
                                   msg=k)
    grp, _ = t2.opt.shards['item_emb']
    torch.testing.assert_close(grp.flat.float(), t1.opt.groups[0].flat.float(), rtol=1e-3, atol=2e-5)


def test_sharded_graph_and_lookahead_equal_eager(pg):
    """Row-sharded training with the forward + backward captured in a HIP graph
    (exchange into fixed buffers before each replay, gradient exchange and
    updates after it) and the next batch routed ahead (prefetch on its own
    communicator) == the plain eager sharded step, bit for bit."""
    from tencent_recommendation_2025_amd import synthetic as S
    from tencent_recommendation_2025_amd.sharding import ShardedFusedAdamW
    from tencent_recommendation_2025_amd.train import Trainer
    runs = []
    for graph in (False, True):
        m, cfg = build()
        opt = ShardedFusedAdamW(m, lr=2e-3, defer_period=3)
        tr = Trainer(m, opt, loss='bce', graph=graph, graph_warmup=2)
        g = torch.Generator(device=DEV).manual_seed(0)
        batches = [S.make_batch(cfg, g, DEV) for _ in range(4)]
        losses = []
        for i in range(8):
            nxt = batches[(i + 1) % 4] if graph else None   # eager run: no lookahead
            losses.append(tr.step(batches[i % 4], next_batch=nxt).clone())
        if graph:
            assert tr._g is not None
        sd = {k: v.clone() for k, v in m.state_dict().items()}
        tabs = {k: opt.shard_table(k).clone() for k in ('item_emb', 'user_emb')}
        torch.cuda.synchronize()
        runs.append((torch.stack(losses), sd, tabs))
    assert torch.equal(runs[0][0], runs[1][0]), (runs[0][0], runs[1][0])
    for k in runs[0][1]:
        assert torch.equal(runs[0][1][k], runs[1][1][k]), k
    for k in runs[0][2]:
        assert torch.equal(runs[0][2][k], runs[1][2][k]), k


def test_shards_built_directly_equal_materialized_table(pg):
    """args.shard_tables: the sharded optimizer builds only its rows (never the
    whole table, config 3); it trains like FusedAdamW on the materialized twin
    (materialize_tables_, the same per-row init) -- G = 1."""
    from tencent_recommendation_2025_amd import synthetic as S
    from tencent_recommendation_2025_amd.model import BaselineModel, init_reference_, materialize_tables_
    from tencent_recommendation_2025_amd.optim import FusedAdamW
    from tencent_recommendation_2025_amd.sharding import ShardedFusedAdamW
    from tencent_recommendation_2025_amd.train import Trainer
    cfg = S.SyntheticConfig(batch_size=8, maxlen=40, num_items=3000, num_users=400, min_len=8)
    stats, types = S.feature_schema(cfg)
    models = []
    for _ in range(2):
        args = S.make_args(hidden_units=64, maxlen=40, num_blocks=1, num_heads=2)
        args.shard_tables = True
        torch.manual_seed(0)
        m = BaselineModel(cfg.num_users, cfg.num_items, stats, types, args).to(DEV)
        init_reference_(m, seed=0, live_norms=True)
        models.append(m)
    m1, m2 = models
    materialize_tables_(m1, seed=5)
    assert m2.item_emb.weight.numel() == 0
    t1 = Trainer(m1, FusedAdamW(m1, lr=2e-3, table_dtype=torch.float32, defer_period=2), loss='bce',
                 amp_dtype=None)
    opt2 = ShardedFusedAdamW(m2, lr=2e-3, table_dtype=torch.float32, defer_period=2, init_seed=5)
    for k in ('item_emb', 'user_emb'):
        assert torch.equal(opt2.shard_table(k), getattr(m1, k).weight.detach()), k
    t2 = Trainer(m2, opt2, loss='bce', amp_dtype=None)
    g = torch.Generator(device=DEV).manual_seed(0)
    for _ in range(4):
        b = S.make_batch(cfg, g, DEV)
        l1, l2 = t1.step(b), t2.step(b)
        assert abs(l1.item() - l2.item()) < 1e-4 * max(1.0, abs(l1.item()))
    s1 = m1.state_dict()
    for k in ('item_emb', 'user_emb'):
        torch.testing.assert_close(opt2.shard_table(k).float(), s1[f'{k}.weight'].float(), rtol=1e-3, atol=2e-5,
                                   msg=k)


def test_capture_stream_is_private_never_a_pool_stream(pg):
    """Deterministic check of the r2s7 capture abort's mechanism (DESIGN.md §5b
    item 4): a collective's end event is recorded on a torch pool stream (the
    process group takes its streams from torch's round-robin pool, and so would
    the Trainer if it called torch.cuda.Stream()).  Capturing the step on such a
    stream makes the watchdog's query of that event illegal.  The Trainer must
    capture (and warm up) on the process's own grk_stream_create stream, which is
    none of the pool's streams however many the process has handed out."""
    from tencent_recommendation_2025_amd import synthetic as S
    from tencent_recommendation_2025_amd.optim import FusedAdamW
    from tencent_recommendation_2025_amd.train import Trainer, private_stream
    pool = [torch.cuda.Stream() for _ in range(96)]      # every stream of torch's pool, several times over
    pool_handles = {s.cuda_stream for s in pool}
    x = torch.ones(4, device=DEV)
    with torch.cuda.stream(pool[0]):                     # a collective's event on a pool stream
        dist.all_reduce(x)
        ev = torch.cuda.Event()
        ev.record(pool[0])
    m, cfg = build()
    tr = Trainer(m, FusedAdamW(m, lr=1e-3, defer_period=4), loss='bce', graph=True, graph_warmup=1)
    g = torch.Generator(device=DEV).manual_seed(0)
    for _ in range(3):
        tr.step(S.make_batch(cfg, g, DEV))
        ev.query()                                       # the watchdog's poll: legal outside our capture
    assert tr._g is not None
    side = tr._side.cuda_stream
    assert side == private_stream(torch.device(DEV)).cuda_stream
    assert side not in pool_handles and side != torch.cuda.current_stream().cuda_stream
    torch.cuda.synchronize()
    assert float(x[0]) == 1.0


# Jagged rows under the row-sharded optimizer (train.jagged_remaps).  Its first
# hardware run (round 4) found the graph replays of the first capacity stepping
# with the gradient buffers of the second capacity's graph (one capture state per
# optimizer): the states are now kept per graph (Trainer._cap_states).
def test_sharded_jagged_equals_sharded_padded_and_graph_replay(pg):
    """World 1, fp32: the row-sharded trainer on jagged rows tracks it on the padded
    batch (losses 5e-4) and equals the non-sharded fused trainer on the same jagged
    rows (parameters and shards within the world-1 bounds of
    test_sharded_optimizer_world1_equals_fused); the jagged sharded step replayed
    from HIP graphs (two capacities) == its eager step, bitwise.  (Parameters of the
    padded and jagged trajectories are not compared: after the first step they are
    two trajectories, and Adam turns the rounding noise of a near-zero gradient
    element into a +-lr move -- tests/test_gpu_jagged.py compares the two layouts
    from identical parameters instead.)"""
    from tencent_recommendation_2025_amd import jagged as J
    from tencent_recommendation_2025_amd import synthetic as S
    from tencent_recommendation_2025_amd.optim import FusedAdamW
    from tencent_recommendation_2025_amd.sharding import ShardedFusedAdamW
    from tencent_recommendation_2025_amd.train import Trainer
    runs = {}
    for name, jagged, graph, amp, sharded in (('padded', False, False, None, True), ('jagged', True, False, None, True),
                                              ('fused_jagged', True, False, None, False),
                                              ('jagged_bf16', True, False, torch.bfloat16, True),
                                              ('jagged_graph', True, True, torch.bfloat16, True)):
        m, cfg = build()
        tdt = torch.float32 if amp is None else torch.bfloat16
        if sharded:
            opt = ShardedFusedAdamW(m, lr=2e-3, table_dtype=tdt, defer_period=3)
        else:
            opt = FusedAdamW(m, lr=2e-3, table_dtype=tdt, defer_period=3)
        tr = Trainer(m, opt, loss='bce', amp_dtype=amp, graph=graph, graph_warmup=1, jagged=jagged,
                     jagged_quantum=64)
        g = torch.Generator(device=DEV).manual_seed(0)
        batches = [S.make_batch(cfg, g, DEV) for _ in range(3)]
        short = S.SyntheticConfig(**{**cfg.__dict__, 'min_len': 2})
        batches.append(S.make_batch(short, g, DEV))
        rows = [J.span_rows(b[3]) for b in batches]
        losses = [tr.step(batches[i % 4], next_batch=batches[(i + 1) % 4] if graph else None,
                          rows=rows[i % 4] if jagged else None).clone() for i in range(8)]
        if graph:
            assert len(tr._graphs) >= 2, tr._graphs.keys()
        sd = {k: v.clone() for k, v in m.state_dict().items()}
        if sharded:
            tabs = {k: opt.shard_table(k).clone() for k in ('item_emb', 'user_emb')}
        else:
            tabs = {k: sd[f'{k}.weight'] for k in ('item_emb', 'user_emb')}
        torch.cuda.synchronize()
        runs[name] = (torch.stack(losses), sd, tabs)
    assert torch.equal(runs['jagged_bf16'][0], runs['jagged_graph'][0])
    for i in (1, 2):
        for k in runs['jagged_bf16'][i]:
            assert torch.equal(runs['jagged_bf16'][i][k], runs['jagged_graph'][i][k]), k
    lp, lj = runs['padded'][0], runs['jagged'][0]
    rel = (lj - lp).abs() / lp.abs()
    # step 1 sees identical parameters: the same loss up to the order of the sums over
    # rows; later steps follow two trajectories (measured on MI355X, round 4: 0, 2e-5,
    # 1e-5, 1.6e-4, 4e-6, 3e-5, 1e-4, 3e-5 over the 8 steps)
    assert rel[0].item() < 1e-6, (lp, lj)
    assert rel.max().item() < 5e-4, (lp, lj)
    lf = runs['fused_jagged'][0]
    assert ((lj - lf).abs() < 1e-4 * lf.abs().clamp(min=1.0)).all(), (lj, lf)
    for k in runs['fused_jagged'][1]:
        if k in ('item_emb.weight', 'user_emb.weight'):
            continue   # held as shards by the sharded optimizer: compared below
        torch.testing.assert_close(runs['jagged'][1][k].float(), runs['fused_jagged'][1][k].float(), rtol=1e-3,
                                   atol=2e-5, msg=k)
    for k in runs['fused_jagged'][2]:
        torch.testing.assert_close(runs['jagged'][2][k].float(), runs['fused_jagged'][2][k].float(), rtol=1e-3,
                                   atol=2e-5, msg=k)

def test_sharded_dense_flat_equals_torch_adamw_and_shadows_match(pg):
    """the row-sharded optimizer's dense parameters on the flat multi-range
    AdamW (dense_flat=True, the default: gradients are views of the all-reduce
    buckets, bf16 GEMM shadows written by the update) against dense_flat=False
    (torch's fused AdamW) over 4 bf16 steps: losses, and the parameters after the first step, within the flat
    update's few-ulp deviation (hardware sqrt / reciprocal), and every
    shadow == its parameter rounded to bf16, bit for bit."""
    from tencent_recommendation_2025_amd import functional as G
    from tencent_recommendation_2025_amd import synthetic as S
    from tencent_recommendation_2025_amd.sharding import ShardedFusedAdamW
    from tencent_recommendation_2025_amd.train import Trainer
    runs = []
    for flat in (True, False):
        m, cfg = build()
        opt = ShardedFusedAdamW(m, lr=2e-3, defer_period=3, dense_flat=flat)
        assert (opt._flat is not None) == flat
        tr = Trainer(m, opt, loss='bce')
        g = torch.Generator(device=DEV).manual_seed(0)
        losses, first = [], None
        for i in range(4):
            losses.append(tr.step(S.make_batch(cfg, g, DEV)).item())
            if i == 0:   # parameters after step 1 (same gradients in both runs)
                first = {k: v.float().clone() for k, v in m.state_dict().items()}
        if flat:
            for p in opt._flat.params:
                assert torch.equal(G.bf16_shadow(p), p.detach().bfloat16())
        runs.append((losses, first))
    (l1, s1), (l2, s2) = runs
    assert all(abs(a - b) < 1e-3 * max(1.0, abs(b)) for a, b in zip(l1, l2)), (l1, l2)
    for k in s1:
        if k in ('item_emb.weight', 'user_emb.weight'):
            continue
        torch.testing.assert_close(s1[k], s2[k], rtol=2e-3, atol=1e-4, msg=k)


def _route_reference(ids, world, global_rows):
    """The routing plan of ShardExchange._route_torch restated on the host: distinct
    in-range ids ordered by (owner = id % world, id), each id's slot, per-owner counts."""
    import numpy as np
    ok = (ids >= 0) & (ids < global_rows)
    uniq = sorted(set(ids[ok].tolist()), key=lambda v: (v % world, v))
    slot = {v: i for i, v in enumerate(uniq)}
    inverse = np.array([slot[v] if 0 <= v < global_rows else -1 for v in ids.tolist()], dtype=np.int64)
    counts = np.bincount(np.array([v % world for v in uniq], dtype=np.int64), minlength=world)[:world]
    return np.array(uniq, dtype=np.int64), inverse, counts, int((~ok).sum())


@pytest.mark.parametrize('world,rows,n', [(1, 1_000_001, 41472), (2, 1_000_001, 30000), (3, 1000, 5000),
                                          (8, 50_000_017, 20000), (5, 7, 64), (4, 100, 0)])
def test_grk_route_equals_sort_route(world, rows, n):
    """grk_route (the presence-bitmap route of the row-sharded tables) == the sort-based
    plan: send order, slots, split sizes, out-of-range count -- duplicates, ids past the
    last row and negative ids included."""
    import numpy as np
    from tencent_recommendation_2025_amd import kernels as K
    rng = np.random.default_rng(world * 7 + n)
    ids = rng.integers(0, rows, n)
    if n:
        ids[rng.integers(0, n, n // 3)] = ids[0]                        # duplicates
        ids[rng.integers(0, n, max(1, n // 100))] = rng.integers(0, min(rows, 50), max(1, n // 100))
    if n >= 64:
        ids[5], ids[9], ids[11] = -1, rows, rows + 12                   # out of range
    R = -(-rows // world)
    got = K.route(torch.tensor(ids, device=DEV), world, R, rows)
    uniq, inverse, counts, bad = _route_reference(ids, world, rows)
    nu = len(uniq)
    assert int(got['n_uniq'].item()) == nu and int(got['bad'].item()) == bad
    assert np.array_equal(got['send_ids'][:nu].cpu().numpy(), uniq)
    assert np.array_equal(got['inverse'].cpu().numpy(), inverse)
    assert np.array_equal(got['send_counts'].cpu().numpy(), counts)


def test_flat_pack_equals_cat():
    """grk_flat_pack: a bucket's bf16 / fp32 gradients (and a missing one, zeros) into the
    fp32 flat buffer == torch.cat of the fp32 casts, more than 64 parts (two launches)."""
    from tencent_recommendation_2025_amd import kernels as K
    g = torch.Generator(device=DEV).manual_seed(3)
    shapes = [(512, 2048), (512,), (7,), (552, 512), (1, 33), (2049,)] * 12
    parts, ref, off = [], [], 0
    for i, sh in enumerate(shapes):
        n = int(torch.tensor(sh).prod())
        if i % 11 == 5:
            src = None
            ref.append(torch.zeros(n, device=DEV))
        else:
            src = torch.randn(sh, device=DEV, generator=g)
            if i % 2:
                src = src.bfloat16()
            ref.append(src.float().reshape(-1))
        parts.append((src, off, n))
        off += n
    flat = torch.full((off,), float('nan'), device=DEV)
    K.flat_pack(flat, parts)
    assert torch.equal(flat, torch.cat(ref))


def test_grk_jagged_remap_equals_torch_remap():
    """train.jagged_remaps on the device (grk_jagged_remap, one launch for every role) ==
    its torch form: span rows follow the row map, dead rows read the role's first
    padding slot (position 0 when a role has no padding id)."""
    from tencent_recommendation_2025_amd.sharding import ShardedFusedAdamW
    from tencent_recommendation_2025_amd.train import jagged_remaps
    g = torch.Generator().manual_seed(5)
    B, T, cap = 16, 40, 640
    starts = torch.randint(0, T - 3, (B,), generator=g).tolist()
    starts[3] = 0
    tt = torch.zeros(B, T, dtype=torch.int64)
    for b, s0 in enumerate(starts):
        tt[b, s0:] = 1
        tt[b, s0] = 2
    seq = torch.randint(1, 500, (B, T), generator=g) * (tt != 0)
    pos = torch.randint(1, 500, (B, T), generator=g) * (tt != 0)
    neg = torch.randint(1, 500, (B, T), generator=g)              # no padding id at all
    batch = tuple(t.to(DEV) for t in (seq, pos, neg, tt))
    parts = ShardedFusedAdamW._parts(batch)
    remaps, fetched = {}, object()
    for name, plist in parts.items():
        for role, idx, mode, v in plist:
            inv = torch.randint(0, 10_000, (B * T,), generator=g).to(DEV)
            remaps[(name, role, mode)] = (fetched, inv.view(B, T))
    span = [(b, t) for b in range(B) for t in range(starts[b], T)]
    row_map = torch.full((cap,), -1, dtype=torch.int32)
    row_map[:len(span)] = torch.tensor([b * T + t for b, t in span], dtype=torch.int32)
    row_map = row_map.to(DEV)
    want = jagged_remaps(remaps, parts, row_map)                  # torch form (no token_type)
    got = jagged_remaps(remaps, parts, row_map, batch[3])         # grk_jagged_remap
    assert set(got) == set(want)
    for k in want:
        assert got[k][0] is want[k][0] and torch.equal(got[k][1], want[k][1]), k


def test_torch_route_switch_equals_grk_route(pg, monkeypatch):
    """GRK_ROUTE=torch (sharding.ROUTE_TORCH): the sort-based torch route on device ids
    trains bit for bit like grk_route (the same plan: owner order, ascending ids)."""
    from tencent_recommendation_2025_amd import sharding
    from tencent_recommendation_2025_amd import synthetic as S
    from tencent_recommendation_2025_amd.train import Trainer
    out = []
    for torch_route in (False, True):
        monkeypatch.setattr(sharding, 'ROUTE_TORCH', torch_route)
        m, cfg = build()
        tr = Trainer(m, sharding.ShardedFusedAdamW(m, lr=2e-3, defer_period=2), loss='bce')
        g = torch.Generator(device=DEV).manual_seed(4)
        losses = [float(tr.step(S.make_batch(cfg, g, DEV))) for _ in range(4)]
        state = {k: v.detach().clone() for k, v in m.state_dict().items()
                 if k not in ('item_emb.weight', 'user_emb.weight')}
        state.update({k: tr.opt.shard_table(k).clone() for k in ('item_emb', 'user_emb')})
        out.append((losses, state))
    assert out[0][0] == out[1][0]
    for k in out[0][1]:
        assert torch.equal(out[0][1][k], out[1][1][k]), k
