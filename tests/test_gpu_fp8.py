"""Config C5 (BASELINE.json configs[4]): HSTU d=1024, T=1025 with fp8
attention.  The fp8 layer quantises its SiLU'd v|q|k to OCP e4m3 once
(grk_silu_fp8) and runs the fp8 attention kernels; the backward is
straight-through at the quantiser (grk_dsilu_mul).  The oracle
(oracle/model_ref.RefHSTU(fp8=True)) rounds the same activations to e4m3 with
the same straight-through gradient, in fp32 everywhere else."""
import contextlib

import numpy as np
import pytest
import torch

from oracle import model_ref

pytestmark = pytest.mark.gpu
DEV = 'cuda'
# The d = 1024 model tests were opt-in in round 3: their first run hit an illegal
# address in torch's batched bf16 GEMM of the projected feature tables (hipBLASLt
# HIPBLAS_STATUS_INTERNAL_ERROR at m 1024 n 10001 k 1024, then the rocBLAS fallback
# faulted), before any fp8 code ran.  The projections now run on grk's grouped MFMA
# GEMM / grk_gemm; both tests passed on MI355X in round 4
# (gpurun_out r4l) and run by default.


def nrel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.fixture(scope='module')
def K():
    from tencent_recommendation_2025_amd import kernels
    return kernels


def test_silu_fp8_and_dsilu_mul(K):
    """e4m3(SiLU(x)) against torch's e4m3 cast of the fp32 SiLU (equal except where
    the ~1-ulp hardware sigmoid moves a value across a rounding boundary: then one
    e4m3 step), saturated beyond +-448, column views; g * dSiLU(x) within bf16."""
    g = torch.Generator(device=DEV).manual_seed(0)
    pre = (3 * torch.randn(3000, 4 * 96, device=DEV, generator=g)).bfloat16()
    pre[0, 96:104] = torch.tensor([500., -500., 1e4, 0., -0., 1e-8, 600., -3.], device=DEV).bfloat16()
    view = pre[:, 96:]
    got = K.silu_fp8(view).float()
    want = torch.nn.functional.silu(view.float()).clamp(-448, 448).to(torch.float8_e4m3fn).float()
    diff = (got - want).abs()
    assert float((diff > 0).float().mean()) < 1e-3
    assert bool(torch.all(diff <= 0.07 * want.abs() + 2 ** -9))
    assert got[0, :8].tolist() == want[0, :8].tolist()
    gr = torch.randn(3000, 4 * 96, device=DEV, generator=g).bfloat16()
    gv = gr[:, 96:]
    ref = (gv.float() * torch.sigmoid(view.float()) * (1 + view.float() * (1 - torch.sigmoid(view.float()))))
    out = K.dsilu_mul_(gv.clone(), view).float()
    assert nrel(out.cpu(), ref.cpu()) < 4e-3
    keep = gr[:, :96].clone()
    K.dsilu_mul_(gv, view)
    assert torch.equal(gr[:, :96], keep)           # columns outside the view untouched


def _c5_models(B, blocks, seed=5):
    from tencent_recommendation_2025_amd import synthetic as S
    from tencent_recommendation_2025_amd.model import BaselineModel
    cfg = S.SyntheticConfig(batch_size=B, maxlen=1024, num_items=3000, num_users=400, min_len=300)
    stats, types = S.feature_schema(cfg)
    args = S.make_args(hidden_units=1024, maxlen=1024, num_blocks=blocks, num_heads=8, hstu_fp8=True)
    ref = model_ref.RefBaselineModel(cfg.num_users, cfg.num_items, stats, types, args, variant='o1', block='hstu')
    model_ref.init_params(ref, seed=seed)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for n, p in ref.named_parameters():
            if p.dim() == 1 and 'norm' in n and n.endswith('weight'):
                p.fill_(1.0)
            elif p.dim() == 1:
                p.copy_(0.02 * torch.randn(p.shape, generator=g))
            elif n.endswith('.rab'):
                p.copy_(0.3 * torch.randn(p.shape, generator=g))
    m = BaselineModel(cfg.num_users, cfg.num_items, stats, types, args).to(DEV)
    m.load_state_dict(ref.state_dict())
    return cfg, m, ref


# Bounds of the C5 model step (the round-4 bounds -- loss 1e-2, logits
# 5e-2, attention gradients 0.15 -- came from comparing bf16 activations rounded to e4m3
# with fp32 ones rounded to e4m3, where e4m3 flips dominate).  Now:
# * the fp32 model against the oracle fed the core's own rounding points (RefHSTU
#   bf16_core + fp8: bf16 pre-activation, e4m3(SiLU) in one rounding, bf16 gate, o, y
#   and gradients) -- what is left is the kernels' math and the rare e4m3 flips of the
#   hardware SiLU's last bit (tests/test_silu_fp8_and_dsilu_mul: < 1e-3 of elements);
# * the bf16-autocast model (the bench's) against the fp32 oracle, held to the oracle's
#   own bf16-autocast error (the reference's --use_amp), as the bench-config tests.
# measured on MI355X (round 5, gpurun_out r5a): core loss 3.2e-6, logits 9.0e-5, gradients
# <= 1.7e-3 (the rab and uvqk weight of the second block); autocast loss 1.2e-4 (AMP 1.1e-5),
# logits 2.8e-3 (AMP 2.8e-3), gradients <= 9.5e-2 (AMP <= 9.8e-2: the user-side feature
# tables at B = 2, one token per row)
C5_CORE_TOL = dict(loss=1e-4, logits=1e-3, grad=5e-3)
C5_AMP_FACTOR = 1.5
C5_AMP_FLOOR = dict(logits=5e-3, grad=2.5e-2)


def _c5_oracles(ref, cpu):
    """(fp32 oracle, bf16-core oracle, AMP oracle): loss, logits, gradients of each."""
    out = {}
    for mode in ('fp32', 'core', 'amp'):
        for blk in ref.attention_layers:
            blk.bf16_core = mode == 'core'
        ref.zero_grad(set_to_none=True)
        ctx = torch.autocast('cpu', dtype=torch.bfloat16) if mode == 'amp' else contextlib.nullcontext()
        with ctx:
            rpl, rnl = ref(cpu[0], cpu[1], cpu[2], cpu[3], cpu[4], cpu[6], cpu[7], cpu[8])
            rloss = model_ref.bce_loss(rpl.float(), rnl.float(), cpu[4])
        rloss.backward()
        out[mode] = (rloss.item(), rpl.detach().float(), rnl.detach().float(),
                     {n: p.grad.detach().float().clone() for n, p in ref.named_parameters() if p.grad is not None})
    for blk in ref.attention_layers:
        blk.bf16_core = False
    return out


def _c5_errors(loss, pl, nl, grads, want):
    wl, wpl, wnl, wg = want
    e = {'loss': abs(loss - wl) / abs(wl), 'logits': max(nrel(pl, wpl), nrel(nl, wnl))}
    g = {n: nrel(grads[n], w) for n, w in wg.items() if float(w.norm()) > 0}
    return e, g


def test_c5_fp8_model_step_matches_oracle():
    """C5 shape (d=1024 = 8 heads x 128, T=1025) at reduced B=2 and 2 blocks: the
    drop-in model with fp8 HSTU layers against the oracle with the same e4m3
    rounding of q/k/v: loss, logits and EVERY gradient, twice -- the fp32 model
    against the oracle fed the core's rounding points (C5_CORE_TOL), the bf16
    autocast model against the fp32 oracle within its AMP reference's error."""
    from tencent_recommendation_2025_amd import functional as G
    from tencent_recommendation_2025_amd import synthetic as S
    cfg, m, ref = _c5_models(B=2, blocks=2)
    batch = S.make_batch(cfg, torch.Generator(device=DEV).manual_seed(7), DEV)
    seq, pos, neg, tt, ntt, _nat, sf, pf, nf = batch
    cpu = [x.cpu() if torch.is_tensor(x) else {k: v.cpu() for k, v in x.items()} for x in batch]
    want = _c5_oracles(ref, cpu)
    m.train()
    res = {}
    for amp in (False, True):
        m.zero_grad(set_to_none=True)
        ctx = torch.autocast('cuda', dtype=torch.bfloat16) if amp else contextlib.nullcontext()
        with ctx:
            h, pe, ne = m.encode(seq, pos, neg, tt, sf, pf, nf)
            loss = G.bce_loss(h, pe, ne, ntt)
        pl, nl = G.pair_logits(h.detach().float(), pe.detach().float(), ne.detach().float(), ntt)
        loss.backward()
        assert np.isfinite(loss.item())
        res[amp] = (loss.item(), pl.cpu(), nl.cpu(),
                    {n: p.grad.float().cpu() for n, p in m.named_parameters() if p.grad is not None})
    # (1) fp32 model vs the bf16-core oracle
    e, g = _c5_errors(*res[False], want['core'])
    worst = sorted(g.items(), key=lambda kv: -kv[1])[:6]
    print('C5 fp32 model vs bf16-core fp8 oracle:', e, 'worst grads', worst)
    assert len(want['core'][3]) == sum(1 for _ in ref.parameters())   # every parameter's gradient compared
    assert e['loss'] < C5_CORE_TOL['loss'] and e['logits'] < C5_CORE_TOL['logits'], e
    bad = {k: v for k, v in g.items() if v >= C5_CORE_TOL['grad']}
    assert not bad, bad
    # (2) bf16-autocast model vs the fp32 oracle, within the AMP oracle's own error
    e, g = _c5_errors(*res[True], want['fp32'])
    ea, ga = _c5_errors(*want['amp'], want['fp32'])
    print('C5 autocast model vs fp32 oracle:', e, '; AMP oracle:', ea)
    print('   worst grads (grk, amp):', sorted(((v, ga.get(k), k) for k, v in g.items()), reverse=True)[:6])
    assert e['loss'] < 1e-3, (e, ea)                                        # the north star's loss bound
    assert e['logits'] <= max(C5_AMP_FACTOR * ea['logits'], C5_AMP_FLOOR['logits']), (e, ea)
    over = [(k, v, ga[k]) for k, v in g.items() if v > max(C5_AMP_FACTOR * ga[k], C5_AMP_FLOOR['grad'])]
    assert not over, over


def test_c5_fp8_trainer_graph_equals_eager():
    """The fused trainer with fp8 HSTU layers at the C5 shape (B=2, 1 block):
    the HIP-graph replayed step equals the eager step bitwise (losses and every
    parameter after two steps)."""
    from tencent_recommendation_2025_amd import synthetic as S
    from tencent_recommendation_2025_amd.optim import FusedAdamW
    from tencent_recommendation_2025_amd.train import Trainer
    out = []
    for graph in (False, True):
        cfg, m, _ = _c5_models(B=2, blocks=1, seed=9)
        opt = FusedAdamW(m, lr=1e-3)
        tr = Trainer(m, opt, loss='bce', graph=graph, graph_warmup=1)
        gen = torch.Generator(device=DEV).manual_seed(3)
        batches = [S.make_batch(cfg, gen, DEV) for _ in range(3)]
        losses = [tr.step(b).item() for b in batches]
        opt.flush()
        out.append((losses, {k: v.detach().float().cpu() for k, v in m.state_dict().items()}))
    assert np.isfinite(out[0][0]).all()
    assert out[0][0] == out[1][0]
    for k in out[0][1]:
        assert torch.equal(out[0][1][k], out[1][1][k]), k
