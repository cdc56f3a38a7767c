"""GPU parity of the loss kernels: fused pair logits + BCE (reference loss,
model/BaseLine/main.py:177-182) and the in-batch sampled softmax (north star,
parity unpinned vs the reference; checked against oracle/loss.py in fp64 on the
same bf16-rounded inputs: loss and gradients within 1e-3 relative (normwise)
-- the north star's bf16 loss tolerance; the fused backward feeds G to the MFMA
as bf16 hi + lo, so the gradients are in fact fp32-accurate)."""
import numpy as np
import pytest
import torch

from oracle import loss as oloss
from oracle.embedding import to_bf16_f32

pytestmark = pytest.mark.gpu
DEV = 'cuda'


@pytest.fixture(scope='module')
def K():
    from tencent_recommendation_2025_amd import _lib, kernels
    _lib.lib()
    return kernels


def nrel(a, b):
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(np.asarray(a, np.float64) - b) / max(np.linalg.norm(b), 1e-30))


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_pair_logits_and_bce(K, dtype):
    from tencent_recommendation_2025_amd import functional as G
    rng = np.random.default_rng(0)
    N, D = 1003, 64
    h, ep, en = (to_bf16_f32(rng.standard_normal((N, D)).astype(np.float32) * 0.3) for _ in range(3))
    ntt = (rng.random(N) < 0.7).astype(np.int64)
    loss, pos, neg, dh, dep, den = oloss.bce(h, ep, en, ntt)
    t = lambda x: torch.from_numpy(x).to(DEV).to(dtype).requires_grad_(True)
    th, tp, tn = t(h), t(ep), t(en)
    got = G.bce_loss(th, tp, tn, torch.from_numpy(ntt).to(DEV))
    got.backward()
    assert abs(got.item() - loss) < 1e-5 * abs(loss)
    # fp32: 1e-5 normwise; bf16: the gradients are computed in fp32 and rounded once,
    # so they are held at the north star's 1e-3 against the oracle rounded to bf16 alike
    tol = 1e-5 if dtype == torch.float32 else 1e-3
    rnd = (lambda x: x) if dtype == torch.float32 else (lambda x: to_bf16_f32(np.asarray(x, np.float32)))
    for a, b in ((th.grad, dh), (tp.grad, dep), (tn.grad, den)):
        assert nrel(a.float().cpu().numpy(), rnd(b)) < tol
    th.grad = None
    pl, nl = G.pair_logits(th, tp, tn, torch.from_numpy(ntt).to(DEV))
    np.testing.assert_allclose(pl.detach().cpu().numpy(), pos, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(nl.detach().cpu().numpy(), neg, rtol=1e-4, atol=1e-5)
    (pl.sum() * 2 + nl.sum()).backward()
    want = 2 * ep * (ntt == 1)[:, None] + en * (ntt == 1)[:, None]
    assert nrel(th.grad.float().cpu().numpy(), rnd(want)) < tol


def test_bce_mixed_dtypes_equal_promoted(K):
    """fp32 h with bf16 item embeddings (the bench's autocast dtypes): the kernels
    read them as they are (GRK_F32_BF16) -- loss and dh bitwise those of promoting
    e to fp32, de_pos / de_neg the promoted run's fp32 gradients rounded to bf16."""
    from tencent_recommendation_2025_amd import functional as G
    rng = np.random.default_rng(2)
    N, D = 2050, 512
    h = torch.from_numpy(rng.standard_normal((N, D)).astype(np.float32) * 0.3).to(DEV)
    ep, en = (torch.from_numpy(rng.standard_normal((N, D)).astype(np.float32) * 0.3).to(DEV).bfloat16()
              for _ in range(2))
    ntt = torch.from_numpy((rng.random(N) < 0.7).astype(np.int64)).to(DEV)
    runs = []
    for mixed in (True, False):
        th = h.clone().requires_grad_(True)
        tp = (ep if mixed else ep.float()).clone().requires_grad_(True)
        tn = (en if mixed else en.float()).clone().requires_grad_(True)
        loss = G.bce_loss(th, tp, tn, ntt)
        loss.backward()
        runs.append((loss.detach(), th.grad, tp.grad, tn.grad))
    (lm, hm, pm, nm), (lf, hf, pf, nf) = runs
    assert torch.equal(lm, lf) and torch.equal(hm, hf)
    assert pm.dtype == torch.bfloat16 and torch.equal(pm, pf.bfloat16()) and torch.equal(nm, nf.bfloat16())


def sampled_case(M, D, seed, frac_valid=0.6, dup_every=7):
    rng = np.random.default_rng(seed)
    h = to_bf16_f32(rng.standard_normal((M, D)).astype(np.float32) * 0.2)
    e = to_bf16_f32(rng.standard_normal((M, D)).astype(np.float32) * 0.2)
    ids = rng.integers(1, 5000, M)
    ids[::dup_every] = ids[1::dup_every][:len(ids[::dup_every])]   # in-batch collisions
    valid = rng.random(M) < frac_valid
    return h, e, ids, valid


@pytest.mark.parametrize('M,D', [(77, 32), (600, 64), (1000, 512), (333, 128), (2100, 256), (45, 512), (3001, 512)])
def test_sampled_softmax_matches_oracle(K, M, D):
    """fp32 gradients of the fused backward vs the fp64 oracle at 1e-4 (the
    bf16-output gradients of the autograd path at 1e-3 below)."""
    from tencent_recommendation_2025_amd import functional as G
    h, e, ids, valid = sampled_case(M, D, seed=M)
    tau = 0.05
    loss, dh, de = oloss.sampled_softmax(h, e, ids, valid, tau)
    th = torch.from_numpy(h).to(DEV).to(torch.bfloat16).requires_grad_(True)
    te = torch.from_numpy(e).to(DEV).to(torch.bfloat16).requires_grad_(True)
    ids_d = torch.from_numpy(ids).to(DEV)
    ntt = torch.from_numpy(valid.astype(np.int64)).to(DEV)
    got = G.sampled_softmax_loss(th, te, ids_d, ntt, tau)
    got.backward()
    assert abs(got.item() - loss) < 1e-4 * abs(loss), (got.item(), loss)
    # bf16 gradients (h's dtype) vs the oracle rounded the same way (at M = 45 a handful
    # of one-ulp rounding differences of large elements make the whole normwise figure:
    # the fp32 gradients below are held to 1e-4 there as everywhere)
    if M >= 100:
        assert nrel(th.grad.float().cpu().numpy(), to_bf16_f32(dh.astype(np.float32))) < 1e-3
        assert nrel(te.grad.float().cpu().numpy(), to_bf16_f32(de.astype(np.float32))) < 1e-3
    v8 = torch.from_numpy(valid.astype(np.uint8)).to(DEV)
    l2, lse2, cnt = K.sampled_softmax_fwd(th.detach(), te.detach(), ids_d, v8, tau)
    fdh, fde = K.sampled_softmax_bwd(th.detach(), te.detach(), ids_d, v8, tau, lse2)
    assert int(cnt.item()) == int(valid.sum())
    assert nrel(fdh.cpu().numpy(), dh) < 1e-4 and nrel(fde.cpu().numpy(), de) < 1e-4
    assert torch.all(fdh[~v8.bool()] == 0) and torch.all(fde[~v8.bool()] == 0)
    again = K.sampled_softmax_bwd(th.detach(), te.detach(), ids_d, v8, tau, lse2)
    assert torch.equal(again[0], fdh) and torch.equal(again[1], fde)      # deterministic


@pytest.mark.parametrize('M,D', [(600, 64), (1000, 512), (2100, 256)])
def test_sampled_softmax_logq_matches_oracle(K, M, D):
    """logQ correction (z_ij -= log q_j): loss and fp32 gradients
    vs the fp64 oracle at 1e-4, bf16 gradients at 1e-3 (oracle rounded alike);
    log q = 0 is bitwise the uncorrected kernel."""
    from tencent_recommendation_2025_amd import functional as G
    h, e, ids, valid = sampled_case(M, D, seed=M + 1)
    lq = np.log(np.random.default_rng(M).uniform(1e-4, 0.2, M)).astype(np.float32)
    tau = 0.05
    loss, dh, de = oloss.sampled_softmax(h, e, ids, valid, tau, log_q=lq)
    th = torch.from_numpy(h).to(DEV).to(torch.bfloat16).requires_grad_(True)
    te = torch.from_numpy(e).to(DEV).to(torch.bfloat16).requires_grad_(True)
    ids_d = torch.from_numpy(ids).to(DEV)
    ntt = torch.from_numpy(valid.astype(np.int64)).to(DEV)
    lq_d = torch.from_numpy(lq).to(DEV)
    got = G.sampled_softmax_loss(th, te, ids_d, ntt, tau, log_q=lq_d)
    got.backward()
    assert abs(got.item() - loss) < 1e-4 * abs(loss), (got.item(), loss)
    assert nrel(th.grad.float().cpu().numpy(), to_bf16_f32(dh.astype(np.float32))) < 1e-3
    assert nrel(te.grad.float().cpu().numpy(), to_bf16_f32(de.astype(np.float32))) < 1e-3
    v8 = torch.from_numpy(valid.astype(np.uint8)).to(DEV)
    l2, lse2, _ = K.sampled_softmax_fwd(th.detach(), te.detach(), ids_d, v8, tau, log_q=lq_d)
    fdh, fde = K.sampled_softmax_bwd(th.detach(), te.detach(), ids_d, v8, tau, lse2, log_q=lq_d)
    assert nrel(fdh.cpu().numpy(), dh) < 1e-4 and nrel(fde.cpu().numpy(), de) < 1e-4
    zero = torch.zeros(M, device=DEV)
    a = K.sampled_softmax_fwd(th.detach(), te.detach(), ids_d, v8, tau, log_q=zero)
    b = K.sampled_softmax_fwd(th.detach(), te.detach(), ids_d, v8, tau)
    nv = int(valid.sum())                 # lse2 holds the nv valid rows (compact index)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1][:nv], b[1][:nv])
    ga = K.sampled_softmax_bwd(th.detach(), te.detach(), ids_d, v8, tau, a[1], log_q=zero)
    gb = K.sampled_softmax_bwd(th.detach(), te.detach(), ids_d, v8, tau, b[1])
    assert torch.equal(ga[0], gb[0]) and torch.equal(ga[1], gb[1])


@pytest.mark.parametrize('D', [64, 512])
def test_sampled_softmax_no_valid_rows(K, D):
    M = 64
    h = torch.randn(M, D, device=DEV).bfloat16()
    ids = torch.arange(M, device=DEV)
    v8 = torch.zeros(M, dtype=torch.uint8, device=DEV)
    loss, lse2, cnt = K.sampled_softmax_fwd(h, h, ids, v8, 0.1)
    dh, de = K.sampled_softmax_bwd(h, h, ids, v8, 0.1, lse2)
    assert loss.item() == 0 and cnt.item() == 0 and torch.all(dh == 0) and torch.all(de == 0)


def test_sampled_softmax_full_size_vs_torch_fp32(K):
    """BASELINE config 2 size (M = 128 x 201 positions, D = 512) against a torch
    fp32 restatement on the device (oracle/model_ref.sampled_softmax_loss)."""
    from oracle import model_ref
    from tencent_recommendation_2025_amd import functional as G
    g = torch.Generator(device=DEV).manual_seed(0)
    M, D = 128 * 201, 512
    h = (torch.randn(M, D, device=DEV, generator=g) * 0.05).to(torch.bfloat16)
    e = (torch.randn(M, D, device=DEV, generator=g) * 0.05).to(torch.bfloat16)
    ids = torch.randint(1, 1_000_000, (M,), device=DEV, generator=g)
    ntt = (torch.rand(M, device=DEV, generator=g) < 0.58).long()
    th, te = h.clone().requires_grad_(True), e.clone().requires_grad_(True)
    got = G.sampled_softmax_loss(th, te, ids, ntt, 0.05)
    got.backward()
    rh, re_ = h.float().requires_grad_(True), e.float().requires_grad_(True)
    ref = model_ref.sampled_softmax_loss(rh, re_, ids, ntt, 0.05)
    ref.backward()
    assert abs(got.item() - ref.item()) < 1e-4 * abs(ref.item())
    for a, b in ((th.grad, rh.grad), (te.grad, re_.grad)):   # bf16 grads vs fp32 rounded to bf16
        err = float((a.float() - b.bfloat16().float()).norm() / b.norm())
        assert err < 1e-3, err


@pytest.mark.parametrize('log_q', [None, 'batch'])
def test_trainer_sampled_softmax_learns(log_q):
    from tencent_recommendation_2025_amd import synthetic as S
    from tencent_recommendation_2025_amd.model import BaselineModel
    from tencent_recommendation_2025_amd.optim import FusedAdamW
    from tencent_recommendation_2025_amd.train import Trainer
    cfg = S.SyntheticConfig(batch_size=16, maxlen=60, num_items=5000, num_users=500)
    stats, types = S.feature_schema(cfg)
    torch.manual_seed(0)
    m = BaselineModel(cfg.num_users, cfg.num_items, stats, types,
                      S.make_args(hidden_units=64, maxlen=60, num_blocks=2, num_heads=2)).to(DEV)
    tr = Trainer(m, FusedAdamW(m, lr=3e-3), loss='sampled_softmax', log_q=log_q)
    batch = S.make_batch(cfg, torch.Generator(device=DEV).manual_seed(0), DEV)
    losses = [tr.step(batch).item() for _ in range(6)]
    assert all(np.isfinite(losses)) and losses[-1] < losses[0] - 0.1, losses
