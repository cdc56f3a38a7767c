"""The benched configuration at its OWN size against the oracle (VERDICT r4 item 1,
VERDICT r5 item 1: also at B = 32 and at BASELINE config 4).

``bench.py`` times BASELINE config 2: O1 + HSTU d=512 (8 heads x hd 64), 4 blocks,
maxlen 200 (T = 201), 1M-item and 1M-user bf16 tables, the jagged (span-row)
layout, bf16 autocast GEMMs, the grouped MFMA projections, the merged
projected-row backward, the flat dense AdamW and the deferred dense-parity table
AdamW.  Here exactly that model and optimizer take ONE training step at B = 8 and
B = 32 (and config 4: the same model with 3 RQ-VAE semantic-id levels as O1
item_sparse features) with dropout 0 (the oracle cannot draw grk's dropout masks),
and are compared with ``oracle/model_ref.py`` -- the fp32 torch-CPU restatement of
the reference step (``model/BaseLine/main.py:163-190``: forward, BCE, backward,
``torch.optim.AdamW`` with betas (0.9, 0.98), weight decay 0.01) -- on the same
parameters and batch:

* loss and logits against the fp32 oracle;
* the error budget is the reference's own mixed precision: the oracle step run
  under CPU bf16 autocast (the reference's ``--use_amp``, ``main.py:139-141,173``)
  is measured against the fp32 oracle on the same inputs, and grk may not exceed
  BENCH_AMP_FACTOR x that (or a floor, stated per quantity);
* the dnn ReLUs: a pre-activation within its own rounding error of 0 takes either
  side of the ReLU, and each such flip moves a whole table row's gradient by the
  flipped element's gradient -- a few dozen flips among 10^5-10^6 elements decide the
  normwise error of the tables read by few tokens (the user-side tables at B = 8: 8
  rows; round-6 diagnosis: scripts/diag/user_grad_trace.py).  So the forward's flip
  COUNT is held to the AMP step's (each against the fp32 oracle's own masks), and the
  gradients / updates are compared with the fp32 and AMP oracle steps fed grk's own
  ReLU masks (``RefBaselineModel.relu_masks``): the smooth arithmetic error, without
  the discontinuity;
* every gradient (dense parameters and each table, padding rows excluded), and every
  parameter after the update (deferred rows flushed);
* rows the batch does not touch take the g = 0 AdamW step (decay only): after the
  flush they must equal the fp32 oracle's rows rounded to bf16 BIT FOR BIT.

HSTU has no reference implementation: the oracle's HSTU (``oracle/hstu.py``) is
the HSTU paper restated (parity unpinned against the reference).
"""
import contextlib

import numpy as np
import pytest
import torch

from oracle import model_ref

pytestmark = pytest.mark.gpu
DEV = 'cuda'

B, MAXLEN, D, HEADS, BLOCKS = 8, 200, 512, 8, 4
ITEMS = USERS = 1_000_000
LR, BETAS, EPS, WD = 1e-3, (0.9, 0.98), 1e-8, 0.01

# Bounds.  loss: the north star's 1e-3.  Everything else: BENCH_AMP_FACTOR x the
# AMP reference's own error on the same quantity, or the floor when that is smaller.
BENCH_AMP_FACTOR = 1.5
LOSS_TOL = 1e-3
LOGIT_FLOOR = 5e-3
GRAD_FLOOR = 2.5e-2          # gradients against the oracle fed grk's ReLU masks
RELU_FLIP_FLOOR = 16         # forward ReLU-boundary flips vs the fp32 oracle: max(1.5 x AMP's, 16)
UPDATE_FLOOR = 2.5e-2        # the AdamW step-1 update is ~lr * sign(g): sign flips where |g| ~ its error
ROBUST = 0.1                 # updates compared where |g_fp32| >= 0.1 x its rms (the step-1 sign of a
                             # near-zero gradient is rounding noise for grk and the AMP step alike)
TABLE_FLIP_FRAC = 2e-3       # bf16 tables: robust elements whose step-1 update sign flipped (beyond
                             # BENCH_AMP_FACTOR x the AMP step's own gradient sign flips there)
OPT_TOL = 1e-3               # update vs torch AdamW of grk's own gradient (fp32 dense parameters)
DENSE_FLIPS = (2e-3, 1)      # dense parameters: robust elements whose step-1 update sign flipped, at most
                             # max(BENCH_AMP_FACTOR x the AMP step's flips there, 0.2 % of the robust
                             # elements, 1); the rest compared normwise (UPDATE_FLOOR)


def nrel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    d = np.linalg.norm(b)
    return float(np.linalg.norm(a - b) / (d if d > 0 else 1.0))


def oracle_setup(seed=5, batch=None, sid=None, sid_codes=256):
    """The fp32 oracle model at the bench configuration with live parameters (reference
    init, then LayerNorm gains 1 and small random biases / rab: the reference init
    zeroes them, which makes the first step's logits identically zero), tables
    rounded to bf16 (the fused optimizer stores them so).  sid: a semantic-id table
    [items + 1, levels] (BASELINE config 4: RQ-VAE codes as O1 item_sparse features)."""
    from tencent_recommendation_2025_amd import synthetic as S
    cfg = S.SyntheticConfig(batch_size=batch or B, maxlen=MAXLEN, num_items=ITEMS, num_users=USERS,
                            sid_table=sid, sid_codes=sid_codes)
    stats, types = S.feature_schema(cfg)
    args = S.make_args(hidden_units=D, maxlen=MAXLEN, num_blocks=BLOCKS, num_heads=HEADS, dropout_rate=0.0)
    ref = model_ref.RefBaselineModel(USERS, ITEMS, stats, types, args, variant='o1', block='hstu')
    model_ref.init_params(ref, seed=seed)
    g = torch.Generator().manual_seed(seed + 1)
    tables = ('item_emb', 'user_emb', 'pos_emb', 'sparse_emb.')
    with torch.no_grad():
        for n, p in ref.named_parameters():
            if p.dim() == 1 and 'norm' in n and n.endswith('weight'):
                p.fill_(1.0)
            elif p.dim() == 1:
                p.copy_(0.02 * torch.randn(p.shape, generator=g))
            elif n.endswith('.rab'):
                p.copy_(0.3 * torch.randn(p.shape, generator=g))
            if n.startswith(tables):
                p.copy_(p.bfloat16().float())
    return cfg, stats, types, args, ref


def oracle_step(ref, cpu, bf16, masks=None):
    """One oracle forward + BCE + backward (fp32, or under CPU bf16 autocast): loss,
    logits, every parameter gradient, and the dnn pre-activations {(role, which):
    [B, T, d]} (role seq / pos / neg in call order).  masks: RefBaselineModel.relu_masks
    for the step (None: the oracle's own ReLUs)."""
    ref.zero_grad(set_to_none=True)
    pre, order = {}, iter([('seq', 'item'), ('seq', 'user'), ('pos', 'item'), ('neg', 'item')])
    calls = []

    def hook(mod, inp, out):
        calls.append(out.detach().float())
    hs = [ref.itemdnn.register_forward_hook(hook), ref.userdnn.register_forward_hook(hook)]
    ref.relu_masks = masks
    ctx = torch.autocast('cpu', dtype=torch.bfloat16) if bf16 else contextlib.nullcontext()
    try:
        with ctx:
            pl, nl = ref(cpu[0], cpu[1], cpu[2], cpu[3], cpu[4], cpu[6], cpu[7], cpu[8])
            loss = model_ref.bce_loss(pl.float(), nl.float(), cpu[4])
        loss.backward()
    finally:
        ref.relu_masks = None
        for h in hs:
            h.remove()
    for c in calls:
        pre[next(order)] = c
    grads = {n: p.grad.detach().clone() for n, p in ref.named_parameters() if p.grad is not None}
    return loss.detach(), pl.detach().float(), nl.detach().float(), grads, pre


def adamw_step1_update(p, g):
    """The first torch AdamW step's change of p (m_hat = g, v_hat = g^2): restated
    to price the AMP reference's gradient error in parameter space."""
    return -LR * WD * p - LR * g / (g.abs() + EPS)


def _table_rows(grp, key, n):
    off = grp.offsets[key]
    return off, off + n


def semantic_ids(levels=3, codes=256):
    """BASELINE config 4's item tokens: an RQ-VAE (grk_rq_assign code search) trained
    briefly on the items' mm rows and tokenising the whole 1M-item table, as bench.py
    --semantic-ids does -> the [items + 1, levels] semantic-id table."""
    from tencent_recommendation_2025_amd.rqvae import RQVAE, semantic_id_table
    g = torch.Generator(device=DEV).manual_seed(81)
    mm = torch.randn(ITEMS, 32, device=DEV, generator=g)
    torch.manual_seed(4)
    tok = RQVAE(32, hidden=(256, 128), latent_dim=64, levels=levels, codebook_size=codes).to(DEV)
    tok.init_codebooks(mm[:65536], iters=5)
    opt = torch.optim.Adam(tok.parameters(), lr=1e-3)
    for i in range(10):
        opt.zero_grad(set_to_none=True)
        tok(mm[i * 16384:(i + 1) * 16384])[2]['loss'].backward()
        opt.step()
    return semantic_id_table(tok.tokenize(mm), ITEMS)


@pytest.mark.timeout(600)
@pytest.mark.parametrize('bsz,sid_levels', [(8, 0), (32, 0), (8, 3)], ids=['B8', 'B32', 'C4-sid3-B8'])
def test_bench_config_full_size_step_matches_oracle(bsz, sid_levels):
    """batch 8 / 32: BASELINE config 2 (the bench workload); C4: config 4, the same
    model with 3 RQ-VAE semantic-id levels of 256 codes as O1 item_sparse features
    (model/BaseLineO1/model.py:271-280 -- the ids enter as ordinary item sparse
    features, looked up through the projected tables)."""
    from tencent_recommendation_2025_amd import functional as G
    from tencent_recommendation_2025_amd import jagged as J
    from tencent_recommendation_2025_amd import synthetic as S
    from tencent_recommendation_2025_amd.model import BaselineModel
    from tencent_recommendation_2025_amd.optim import FusedAdamW
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    sid = semantic_ids(sid_levels) if sid_levels else None
    cfg, stats, types, args, ref = oracle_setup(batch=bsz, sid=sid)
    if sid is not None:
        assert types['item_sparse'][-sid_levels:] == [f'sid{i}' for i in range(sid_levels)]
    before = {k: v.detach().clone() for k, v in ref.state_dict().items()}
    m = BaselineModel(USERS, ITEMS, stats, types, args).to(DEV)
    m.load_state_dict(ref.state_dict())
    m.train()
    opt = FusedAdamW(m, lr=LR, betas=BETAS, eps=EPS, weight_decay=WD)   # bench defaults: dense_flat, defer 16
    assert opt._flat is not None and set(opt._deferred) == {'item', 'user'}
    batch = S.make_batch(cfg, torch.Generator(device=DEV).manual_seed(7), DEV)

    # the fused trainer's eager step (train.Trainer.compute_loss, jagged layout, quantum 512),
    # opened up to keep the logits and the gradients before the update
    opt.zero_grad()
    opt.begin_step(batch)
    tt = batch[3]
    n_span = J.span_rows(tt)
    jag = J.layout(tt, J.capacity_for(n_span, 512), batch[4])
    seq, pos, neg, tt_j, ntt, _nat, sf, pf, nf, _ts, pidx = J.compact(batch, jag)
    # grk's dnn ReLU masks: the seq side's item / user pre-activations (the inputs of
    # emb_combine, which applies the ReLUs), the pair side's itemdnn output (ReLU in the
    # GEMM's store: > 0 exactly where the pre-activation is)
    gmask = {}
    orig_combine, orig_linear = G.emb_combine, G.linear

    def combine(a, b, *rest, **kw):
        gmask['seq', 'item'], gmask['seq', 'user'] = (a.detach() > 0), (b.detach() > 0)
        return orig_combine(a, b, *rest, **kw)

    def linear(x, weight, bias=None, addend=None, relu=False, in_place=False):
        y = orig_linear(x, weight, bias, addend, relu, in_place)
        if relu:
            assert 'pair' not in gmask, 'one ReLU linear (the pair itemdnn) per forward'
            gmask['pair'] = y.detach() > 0
        return y
    G.emb_combine, G.linear = combine, linear
    try:
        with torch.autocast('cuda', dtype=torch.bfloat16):
            h, pe, ne = m.encode(seq, pos, neg, tt_j, sf, pf, nf, jagged=jag, pos_idx=pidx)
            loss = G.bce_loss(h, pe, ne, ntt)
    finally:
        G.emb_combine, G.linear = orig_combine, orig_linear
    pl, nl = G.pair_logits(h.detach().float(), pe.detach().float(), ne.detach().float(), ntt)
    loss.backward()
    J.check_error(jag.err)
    grads = {n: p.grad.float().cpu() for n, p in m.named_parameters() if p.grad is not None}
    tgrads = {}
    for grp in opt.groups:
        dg = grp.dense_gradient()
        for key in grp.offsets:
            rows = dict(m.table_modules())[key].num_embeddings
            lo, hi = _table_rows(grp, key, rows)
            tgrads[f'{key}.weight'] = dg[lo + 1:hi].cpu()          # padding row excluded
        del dg
    opt.step()
    opt.flush()
    after = {k: v.detach().float().cpu() for k, v in m.state_dict().items()}
    torch.cuda.synchronize()

    # grk's masks as [B, T, d] (+ the rows they cover: the span rows of the jagged layout)
    rm = jag.row_map.cpu().long()
    live = rm >= 0
    assert int(live.sum()) == n_span
    Bq, Tq = tt.shape
    covered = torch.zeros(Bq * Tq, dtype=torch.bool)
    covered[rm[live]] = True
    covered = covered.view(Bq, Tq)

    def to_bt(msk):
        full = torch.zeros(Bq * Tq, msk.shape[-1], dtype=torch.bool)
        full[rm[live]] = msk.reshape(-1, msk.shape[-1]).cpu()[:rm.numel()][live]
        return full.view(Bq, Tq, -1)
    cap = rm.numel()
    pair = gmask.pop('pair').reshape(-1, gmask['seq', 'item'].shape[-1])
    gmask['pos', 'item'], gmask['neg', 'item'] = pair[:cap], pair[cap:2 * cap]
    masks = {k: (to_bt(v), covered) for k, v in gmask.items()}

    # the oracle: the AMP and fp32 steps with their own ReLUs (loss, logits, the
    # forward's ReLU flips), then both fed grk's ReLU masks (gradients), torch AdamW
    # on the fp32 masked gradients
    cpu = [x.cpu() if torch.is_tensor(x) else {k: v.cpu() for k, v in x.items()} for x in batch]
    aloss, apl, anl, _, apre = oracle_step(ref, cpu, bf16=True)
    rloss, rpl, rnl, _, rpre = oracle_step(ref, cpu, bf16=False)
    flips = {}
    for key, (gm, cov) in masks.items():
        want = rpre[key] > 0
        flips[key] = (int((gm != want)[cov].sum()), int(((apre[key] > 0) != want)[cov].sum()), int(cov.sum()))
    agrad = oracle_step(ref, cpu, bf16=True, masks=masks)[3]
    rgrad = oracle_step(ref, cpu, bf16=False, masks=masks)[3]
    torch.optim.AdamW(ref.parameters(), lr=LR, betas=BETAS, eps=EPS, weight_decay=WD).step()
    rafter = {k: v.detach() for k, v in ref.state_dict().items()}
    pl, nl = pl.cpu().reshape(-1)[live], nl.cpu().reshape(-1)[live]
    sel = rm[live]
    rpl, rnl, apl, anl = (x.reshape(-1)[sel] for x in (rpl, rnl, apl, anl))
    errs = {'loss': abs(loss.item() - rloss.item()) / abs(rloss.item()),
            'logits': max(nrel(pl, rpl), nrel(nl, rnl))}
    amp = {'loss': abs(aloss.item() - rloss.item()) / abs(rloss.item()),
           'logits': max(nrel(apl, rpl), nrel(anl, rnl))}

    # gradients: every dense parameter and every table (padding row excluded)
    g_err, g_amp = {}, {}
    for n, want in rgrad.items():
        is_table = n.startswith(('item_emb', 'user_emb', 'pos_emb', 'sparse_emb.'))
        got = tgrads[n] if is_table else grads[n]
        w = want[1:] if is_table else want
        a = agrad[n][1:] if is_table else agrad[n]
        if float(w.norm()) == 0:
            assert float(got.norm()) == 0, n
            continue
        g_err[n] = nrel(got, w)
        g_amp[n] = nrel(a.float(), w)
    assert set(g_err) | {n for n in rgrad if n not in g_err} == set(rgrad)
    assert len(rgrad) == sum(1 for _ in ref.parameters())

    # parameters after the update: grk (bf16 tables, fp32 dense) vs the oracle rounded
    # alike; the change is compared (the parameters themselves are mostly unchanged)
    u_err, u_amp, u_opt, exact_rows, ulp_off, flip_over = {}, {}, {}, {}, {}, []
    for n, p0 in before.items():
        is_table = n.startswith(('item_emb', 'user_emb', 'pos_emb', 'sparse_emb.'))
        want = rafter[n].bfloat16().float() if is_table else rafter[n]
        du_grk = after[n] - p0
        du_ref = want - p0
        # compared where the sign of the fp32 gradient is robust (|g| >= ROBUST x its rms):
        # the step-1 update is ~lr * sign(g), so where |g| is at its own error level the
        # sign -- and the update -- is rounding noise for grk and the AMP step alike
        rg = rgrad.get(n)
        if rg is not None and float(rg.norm()) > 0:
            nz = rg[rg != 0]                   # rms over the elements with a gradient (tables: touched rows)
            robust = rg.abs() >= ROBUST * float(nz.pow(2).mean().sqrt())
        else:
            robust = torch.ones_like(p0, dtype=torch.bool)
        if n in agrad:
            du_amp = adamw_step1_update(p0, agrad[n].float())
            du_fp = adamw_step1_update(p0, rgrad[n])
            u_amp[n] = nrel(du_amp[robust], du_fp[robust])
        else:
            u_amp[n] = 0.0
        if is_table:
            # bf16 rows: grk's and the oracle's new values are each rounded to bf16, so
            # where the two fp32 results straddle a rounding boundary they differ by one
            # bf16 ulp of the row value (~2^-8 |p|, a large fraction of the ~lr update):
            # every robust element within one ulp, and the count of those off by one
            # ulp reported
            d = (after[n] - want).abs()
            ulp = torch.maximum(want.abs(), after[n].abs()) * 2.0 ** -7 + 1e-9   # + slack << lr near 0
            off = int((d[robust] > 0).sum())
            far = int((d[robust] > ulp[robust]).sum())   # beyond one ulp: a step-1 sign flip (|du| ~ 2 lr)
            # the AMP step's own sign flips of the gradient on the same elements: its budget
            amp_flips = int((((agrad[n].float() > 0) != (rg > 0)) & robust).sum()) if n in agrad else 0
            ulp_off[n] = (off, far, int(robust.sum()), amp_flips)
            if far > max(BENCH_AMP_FACTOR * amp_flips, TABLE_FLIP_FRAC * int(robust.sum())):
                flip_over.append((n, far, amp_flips, int(robust.sum())))
            u_err[n] = 0.0
        else:
            flip = robust & ((du_grk > 0) != (du_ref > 0)) & (du_ref != 0)
            nflip = int(flip.sum())
            amp_flips = int((((agrad[n].float() > 0) != (rg > 0)) & robust).sum()) if n in agrad else 0
            if nflip > max(BENCH_AMP_FACTOR * amp_flips, DENSE_FLIPS[0] * int(robust.sum()), DENSE_FLIPS[1]):
                flip_over.append((n, nflip, amp_flips, int(robust.sum())))
            ulp_off[n] = (0, nflip, int(robust.sum()), amp_flips)
            keep = robust & ~flip
            u_err[n] = nrel(du_grk[keep], du_ref[keep])
        if not is_table and n in grads:
            # the optimizer itself: the change grk applied == torch AdamW's step-1 change
            # computed from grk's own gradient, on every element
            u_opt[n] = nrel(du_grk, adamw_step1_update(p0, grads[n].float()))
        if n in ('item_emb.weight', 'user_emb.weight'):
            untouched = rgrad[n].abs().amax(1) == 0        # g = 0 rows: decay only, deferred then flushed
            untouched[0] = False
            exact_rows[n] = (int(untouched.sum()),
                             int((after[n][untouched] != want[untouched]).any(1).sum()))
    worst_g = sorted(((e, g_amp[k], k) for k, e in g_err.items()), reverse=True)[:6]
    worst_u = sorted(((e, u_amp[k], k) for k, e in u_err.items()), reverse=True)[:6]
    print(f'bench-size step (B={bsz}, sid levels {sid_levels}, {n_span} span rows): grk {errs}, AMP {amp}')
    print('  dnn ReLU flips vs the fp32 oracle (grk, AMP, rows):', flips)
    print('  worst grads (grk, amp, name):', worst_g)
    print('  worst updates (grk, amp, name):', worst_u)
    print('  untouched table rows (count, mismatching):', exact_rows)
    print('  optimizer (update vs AdamW of grk gradients), worst:', max(u_opt.values()) if u_opt else None)
    print('  table + dense elements (one ulp off, sign-flipped, robust, AMP sign flips):',
          [sum(v[i] for v in ulp_off.values()) for i in range(4)])
    print('  per table (one ulp off, sign-flipped, robust, AMP sign flips):',
          {k: v for k, v in ulp_off.items() if k.startswith(('item_emb', 'user_emb', 'sparse_emb.'))})
    print('  worst grads vs AMP (grk / AMP, name):',
          sorted(((e / max(g_amp[k], 1e-30), k) for k, e in g_err.items()), reverse=True)[:8])
    assert not flip_over, flip_over

    assert errs['loss'] < LOSS_TOL, (errs, amp)
    over = [(k, f) for k, f in flips.items() if f[0] > max(BENCH_AMP_FACTOR * f[1], RELU_FLIP_FLOOR)]
    assert not over, over
    assert errs['logits'] <= max(BENCH_AMP_FACTOR * amp['logits'], LOGIT_FLOOR), (errs, amp)
    over = [(k, e, g_amp[k]) for k, e in g_err.items() if e > max(BENCH_AMP_FACTOR * g_amp[k], GRAD_FLOOR)]
    assert not over, over
    over = [(k, e, u_amp[k]) for k, e in u_err.items() if e > max(BENCH_AMP_FACTOR * u_amp[k], UPDATE_FLOOR)]
    assert not over, over
    over = [(k, e) for k, e in u_opt.items() if e > OPT_TOL]
    assert not over, over
    for n, (cnt, bad) in exact_rows.items():
        assert cnt > ITEMS // 2 and bad == 0, (n, cnt, bad)
