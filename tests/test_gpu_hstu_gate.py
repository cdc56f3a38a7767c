"""GPU parity of the fused HSTU output gate (grk_norm_gate_fwd/bwd):
y = dropout(LayerNorm(o) * SiLU(u)) against a plain PyTorch fp32 reference of
the same op (HSTU itself is parity-unpinned: no reference implementation).

Tolerances: y and dout/du are bf16 outputs -> 1e-2 normwise (bf16 rounding
of outputs ~ 2^-9 relative per element); dgamma/dbeta are fp32 sums of
bf16-input products -> 1e-3 normwise."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = 'cuda'


@pytest.fixture(scope='module')
def K():
    from tencent_recommendation_2025_amd import _lib, kernels
    _lib.lib()
    return kernels


def nrel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def keep_np(seed, rows, dim, p):
    """numpy replica of drop8() in grk_hstu.hip (test infrastructure): one splitmix64
    finalisation per 4 consecutive elements, 16-bit uniforms, kept iff >= ceil(p 2^16)."""
    with np.errstate(over='ignore'):
        j = np.arange(rows * dim // 4, dtype=np.uint64)
        x = np.uint64(seed) ^ (j * np.uint64(0x9E3779B97F4A7C15))
        x ^= x >> np.uint64(30); x *= np.uint64(0xBF58476D1CE4E5B9)
        x ^= x >> np.uint64(27); x *= np.uint64(0x94D049BB133111EB)
        x ^= x >> np.uint64(31)
    u16 = np.stack([(x >> np.uint64(16 * e)) & np.uint64(0xFFFF) for e in range(4)], 1).reshape(rows, dim)
    return torch.from_numpy(u16 >= np.ceil(np.float32(p) * np.float32(65536)))


def reference(o, u, w, b, eps, gy, keep, p):
    """fp32 torch: y = LN(o) * bf16(SiLU(u)) * keep / (1-p), grads by autograd + dSiLU(u)."""
    o32 = o.float().requires_grad_(True)
    w32 = w.clone().requires_grad_(True)
    b32 = b.clone().requires_grad_(True)
    u32 = u.float()
    su = F.silu(u32).bfloat16().float()
    m = keep.to(DEV).float() / (1.0 - p) if p > 0 else torch.ones_like(su)
    z = F.layer_norm(o32, (o.shape[1],), w32, b32, eps)
    y = z * su * m
    do, dw, db = torch.autograd.grad(y, (o32, w32, b32), gy.float())
    s = torch.sigmoid(u32)
    du = gy.float() * m * z.detach() * (s * (1 + u32 * (1 - s)))
    return y.detach(), do, du, dw, db


@pytest.mark.parametrize('rows,dim,p', [(1000, 512, 0.0), (777, 64, 0.0), (300, 1024, 0.0), (513, 512, 0.3),
                                        (5, 2048, 0.1)])
def test_norm_gate_matches_torch(K, rows, dim, p):
    g = torch.Generator(device=DEV).manual_seed(rows + dim)
    o = torch.randn(rows, dim, device=DEV, generator=g).bfloat16()
    pre = torch.randn(rows, 4 * dim, device=DEV, generator=g).bfloat16()  # u = first D columns (strided view)
    u = pre[:, :dim]
    w = 1 + 0.1 * torch.randn(dim, device=DEV, generator=g)
    b = 0.1 * torch.randn(dim, device=DEV, generator=g)
    gy = torch.randn(rows, dim, device=DEV, generator=g).bfloat16()
    seed = 987654321
    y, stats = K.norm_gate_fwd(o, u, w, b, 1e-8, p, seed)
    dpre = torch.zeros(rows, 4 * dim, dtype=torch.bfloat16, device=DEV)
    do, du, dw, db = K.norm_gate_bwd(gy, o, u, w, b, stats, p, seed, du=dpre[:, :dim])
    keep = keep_np(seed, rows, dim, p) if p > 0 else None
    ry, rdo, rdu, rdw, rdb = reference(o, u, w, b, 1e-8, gy, keep, p)
    assert nrel(y.float(), ry) < 1e-2
    assert nrel(do.float(), rdo) < 1e-2
    assert nrel(dpre[:, :dim].float(), rdu) < 1e-2
    assert torch.all(dpre[:, dim:] == 0)  # wrote only its own columns
    assert nrel(dw, rdw) < 1e-3 and nrel(db, rdb) < 1e-3
    mean = o.float().mean(1)
    torch.testing.assert_close(stats[:, 0], mean, rtol=1e-4, atol=1e-5)
    if p > 0:
        zero = ~keep.to(DEV)
        assert torch.all(y[zero] == 0) and torch.all(du[zero] == 0)


def test_norm_gate_deterministic_and_empty(K):
    g = torch.Generator(device=DEV).manual_seed(1)
    o = torch.randn(4000, 512, device=DEV, generator=g).bfloat16()
    u = torch.randn(4000, 512, device=DEV, generator=g).bfloat16()
    gy = torch.randn(4000, 512, device=DEV, generator=g).bfloat16()
    w, b = torch.ones(512, device=DEV), torch.zeros(512, device=DEV)
    y, st = K.norm_gate_fwd(o, u, w, b, 1e-8)
    r1 = K.norm_gate_bwd(gy, o, u, w, b, st)
    r2 = K.norm_gate_bwd(gy, o, u, w, b, st)
    for a, c in zip(r1, r2):
        assert torch.equal(a, c)
    e = torch.empty(0, 512, dtype=torch.bfloat16, device=DEV)
    ye, ste = K.norm_gate_fwd(e, e, w, b, 1e-8)
    _, _, dwe, dbe = K.norm_gate_bwd(e, e, e, w, b, ste)
    assert ye.shape == (0, 512) and torch.all(dwe == 0) and torch.all(dbe == 0)


@pytest.mark.parametrize('nbt', [0, 40], ids=['pos', 'pos+time'])
def test_hstu_core_matches_unfused_torch(K, nbt):
    """functional.hstu_core (attention SiLU-on-load + norm gate) vs the eager
    formulation (oracle.model_ref.RefHSTU math) in fp32 on bf16-rounded inputs;
    nbt > 0 adds the time bias rab_t[h, time_bucket(t_q - t_k)] (buckets from
    oracle/hstu.py, gathered in torch so that autograd gives drab_t)."""
    from oracle import hstu as ohstu
    from tencent_recommendation_2025_amd import functional as G
    B, T, H, hd = 3, 90, 2, 64
    D = H * hd
    g = torch.Generator(device=DEV).manual_seed(7)
    pre = torch.randn(B * T, 4 * D, device=DEV, generator=g).bfloat16().float().requires_grad_(True)
    rab = (0.3 * torch.randn(H, T, device=DEV, generator=g)).requires_grad_(True)
    w = (1 + 0.1 * torch.randn(D, device=DEV, generator=g)).requires_grad_(True)
    b = (0.1 * torch.randn(D, device=DEV, generator=g)).requires_grad_(True)
    lens = [90, 50, 3]
    kv = torch.zeros(B, T, dtype=torch.uint8, device=DEV)
    for i, n in enumerate(lens):
        kv[i, T - n:] = 1
    tkw, ts_np = {}, None
    if nbt:
        ts_np = 1_600_000_000 + np.cumsum(np.random.default_rng(5).integers(0, 10 ** 6, (B, T)), 1)
        rab_t = (0.3 * torch.randn(H, nbt, device=DEV, generator=g)).requires_grad_(True)
        tkw = dict(timestamps=torch.from_numpy(ts_np).to(DEV), rab_t=rab_t)
    y = G.hstu_core(pre, rab, w, b, kv, B, T, H, hd, 1.0 / T, 1e-8, precise=True, **tkw)
    gy = torch.randn(B * T, D, device=DEV, generator=g).bfloat16().float()
    params = (pre, rab, w, b) + ((rab_t,) if nbt else ())
    grads = torch.autograd.grad(y, params, gy)
    # eager reference
    p2 = pre.detach().clone().requires_grad_(True)
    r2, w2, b2 = (t.detach().clone().requires_grad_(True) for t in (rab, w, b))
    rt2 = rab_t.detach().clone().requires_grad_(True) if nbt else None
    act = F.silu(p2)
    u, v, q, k = torch.split(act, D, dim=-1)
    sh = lambda x: x.view(B, T, H, hd).transpose(1, 2)
    i = torch.arange(T, device=DEV)[:, None]
    j = torch.arange(T, device=DEV)[None, :]
    s = sh(q) @ sh(k).transpose(-1, -2) * hd ** -0.5 + r2[:, (i - j).clamp(0, T - 1)][None]
    if nbt:
        _, bt = ohstu._time_bias(ts_np, kv.cpu().numpy(), np.zeros((H, nbt)))
        s = s + rt2[:, torch.from_numpy(bt).to(DEV)].transpose(0, 1)
    mask = (j <= i)[None, None] & kv.bool()[:, None, None, :]
    a = F.silu(s) / T * mask
    o = (a @ sh(v)).transpose(1, 2).reshape(B * T, D)
    yr = F.layer_norm(o, (D,), w2, b2, 1e-8) * u
    rg = torch.autograd.grad(yr, (p2, r2, w2, b2) + ((rt2,) if nbt else ()), gy)
    assert nrel(y.detach(), yr.detach()) < 2e-2
    for name, a_, b_ in zip(('dpre', 'drab', 'dgamma', 'dbeta', 'drab_t'), grads, rg):
        assert nrel(a_, b_) < 2e-2, name


@pytest.mark.parametrize('with_y', [False, True])
@pytest.mark.parametrize('x_dtype', [torch.bfloat16, torch.float32])
def test_add_norm_matches_torch(with_y, x_dtype):
    """functional.add_norm (grk_add_norm fwd/bwd) against the eager autocast
    composition it replaces: s_new = bf16(s + y); x = LayerNorm(s_new) in fp32;
    gradients of s, y, gamma, beta in fp32."""
    from tencent_recommendation_2025_amd import functional as G
    g = torch.Generator(device='cuda').manual_seed(8)
    N, D = 333, 512
    s = torch.randn(N, D, device='cuda', generator=g).bfloat16().requires_grad_()
    y = torch.randn(N, D, device='cuda', generator=g).bfloat16().requires_grad_() if with_y else None
    w = (1 + 0.1 * torch.randn(D, device='cuda', generator=g)).requires_grad_()
    b = (0.1 * torch.randn(D, device='cuda', generator=g)).requires_grad_()
    out = G.add_norm(s, y, w, b, 1e-8, x_dtype=x_dtype)
    s_new, x = out if with_y else (None, out)
    gx = torch.randn(N, D, device='cuda', generator=g).to(x_dtype)
    gs = torch.randn(N, D, device='cuda', generator=g).bfloat16() if with_y else None
    torch.autograd.backward([x] + ([s_new] if with_y else []), [gx] + ([gs] if with_y else []))
    # reference: fp32 math on the same bf16 values
    s2 = s.detach().float().requires_grad_()
    y2 = y.detach().float().requires_grad_() if with_y else None
    w2, b2 = w.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    sn = (s2 + y2) if with_y else s2
    if with_y:  # autocast adds in bf16: the LayerNorm sees the rounded sum (straight-through gradient)
        sn = sn + (sn.bfloat16().float() - sn).detach()
    x2 = torch.nn.functional.layer_norm(sn, (D,), w2, b2, 1e-8)
    torch.autograd.backward([x2] + ([sn] if with_y else []), [gx.float()] + ([gs.float()] if with_y else []))
    if with_y:
        assert torch.equal(s_new, (s.detach().float() + y.detach().float()).bfloat16())
    tol = dict(rtol=2e-2, atol=2e-2) if x_dtype == torch.bfloat16 else dict(rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(x.float(), x2.detach(), **tol)
    torch.testing.assert_close(s.grad.float(), s2.grad, rtol=2e-2, atol=3e-2)
    if with_y:
        torch.testing.assert_close(y.grad.float(), y2.grad, rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(w.grad, w2.grad, rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(b.grad, b2.grad, rtol=1e-3, atol=1e-2)


def test_device_seed_equals_host_seed(K):
    """A dropout seed held in device memory (read by the kernels at run time,
    model.dropout_seed) gives bitwise the masks of the same seed passed by value:
    norm gate forward / backward and softmax attention forward / backward."""
    from tencent_recommendation_2025_amd import _lib as L
    g = torch.Generator(device=DEV).manual_seed(11)
    rows, dim, p, seed = 300, 256, 0.2, 1234567890123
    o = torch.randn(rows, dim, device=DEV, generator=g).bfloat16()
    u = torch.randn(rows, dim, device=DEV, generator=g).bfloat16()
    w = torch.randn(dim, device=DEV, generator=g)
    b = torch.randn(dim, device=DEV, generator=g)
    gy = torch.randn(rows, dim, device=DEV, generator=g).bfloat16()
    dseed = torch.tensor([seed], dtype=torch.int64, device=DEV)
    outs = []
    for s in (seed, dseed):
        y, st = K.norm_gate_fwd(o, u, w, b, 1e-8, p, s)
        do, du, dw, db = K.norm_gate_bwd(gy, o, u, w, b, st, p, s)
        outs.append((y, do, du, dw, db))
    for a, c in zip(*outs):
        assert torch.equal(a, c)
    B, T, H, hd = 3, 97, 2, 32
    D = H * hd
    x = torch.randn(B * T, 3 * D, device=DEV, generator=g).bfloat16()
    kv = torch.ones(B, T, dtype=torch.uint8, device=DEV)
    kv[1, :40] = 0
    dout = torch.randn(B * T, D, device=DEV, generator=g).bfloat16()
    res = []
    for s in (seed, dseed):
        args = K.attn_args(L.ATTN_SOFTMAX, x[:, :D], x[:, D:2 * D], x[:, 2 * D:], B, T, H, hd, key_valid=kv,
                           dropout_p=0.2, seed=s)
        out = torch.empty(B * T, D, dtype=torch.bfloat16, device=DEV)
        lse = torch.empty(B, H, T, device=DEV)
        K.attention_fwd(args, out, lse)
        grads = [torch.empty(B * T, D, dtype=torch.bfloat16, device=DEV) for _ in range(3)]
        K.attention_bwd(args, out, dout, lse, torch.empty(B, H, T, device=DEV), *grads)
        res.append([out, *grads])
    for a, c in zip(*res):
        assert torch.equal(a, c)
