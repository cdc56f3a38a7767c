"""GPU diagnostic (round 6): where does grk's gradient error on the USER token's rows
come from?  tests/test_gpu_bench_size.py measures the user-side tables at 3.8e-2
normwise against the fp32 oracle where the AMP oracle step has 2.4e-2 (the item side:
3.9e-2 vs 4.3e-2); scripts/diag/proj_rounding.py shows on the CPU that neither the
projected tables' bf16 roundings nor the bf16 residual stream explain it (1.5e-2).

One bench-config step (B = 8) of grk and of the fp32 / AMP oracle with hooks on the
gradient of (a) every HSTU layer's input (the LayerNorm output) and (b) the first
block's input (the embedding combine output); per layer, the normwise error of that
gradient over the user-token rows and over the item-token rows.

    python scripts/diag/user_grad_trace.py
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))

import test_gpu_bench_size as TB  # noqa: E402
from oracle import model_ref  # noqa: E402


def hook_oracle(ref, store):
    orig = model_ref.RefHSTU.forward

    def fwd(self, query, key, value, *a, **kw):
        i = list(ref.attention_layers).index(self)
        query.register_hook(lambda g, i=i: store.__setitem__(f'x{i}', g.detach().float().reshape(-1, g.shape[-1])))
        return orig(self, query, key, value, *a, **kw)
    return orig, fwd


def main():
    from tencent_recommendation_2025_amd import functional as G
    from tencent_recommendation_2025_amd import jagged as J
    from tencent_recommendation_2025_amd import synthetic as S
    from tencent_recommendation_2025_amd import model as Mm
    from tencent_recommendation_2025_amd.model import BaselineModel
    from tencent_recommendation_2025_amd.optim import FusedAdamW
    torch.set_num_threads(16)
    cfg, stats, types, args, ref = TB.oracle_setup()
    m = BaselineModel(TB.USERS, TB.ITEMS, stats, types, args).to('cuda')
    m.load_state_dict(ref.state_dict())
    m.train()
    opt = FusedAdamW(m, lr=TB.LR, betas=TB.BETAS, eps=TB.EPS, weight_decay=TB.WD)
    batch = S.make_batch(cfg, torch.Generator(device='cuda').manual_seed(7), 'cuda')
    grk = {}
    layers = list(m.attention_layers)
    orig_fwd = type(layers[0]).forward

    def gfwd(self, x, *a, **kw):
        i = layers.index(self)
        x.register_hook(lambda g, i=i: grk.__setitem__(f'x{i}', g.detach().float().reshape(-1, g.shape[-1])))
        return orig_fwd(self, x, *a, **kw)
    type(layers[0]).forward = gfwd
    orig_combine = G.emb_combine

    def combine(*a, **kw):
        xi, xu = a[0], a[1]
        grk['fwd_xi'] = xi.detach().float().reshape(-1, xi.shape[-1]).clone()
        grk['fwd_xu'] = xu.detach().float().reshape(-1, xu.shape[-1]).clone()
        xi.register_hook(lambda g: grk.__setitem__('xi', g.detach().float().reshape(-1, g.shape[-1])))
        xu.register_hook(lambda g: grk.__setitem__('xu', g.detach().float().reshape(-1, g.shape[-1])))
        y = orig_combine(*a, **kw)
        y.register_hook(lambda g: grk.__setitem__('emb', g.detach().float().reshape(-1, g.shape[-1])))
        return y
    G.emb_combine = combine
    Mm.G.emb_combine = combine
    opt.zero_grad()
    opt.begin_step(batch)
    tt = batch[3]
    jag = J.layout(tt, J.capacity_for(J.span_rows(tt), 512), batch[4])
    seq, pos, neg, tt_j, ntt, _nat, sf, pf, nf, _ts, pidx = J.compact(batch, jag)
    with torch.autocast('cuda', dtype=torch.bfloat16):
        h, pe, ne = m.encode(seq, pos, neg, tt_j, sf, pf, nf, jagged=jag, pos_idx=pidx)
        loss = G.bce_loss(h, pe, ne, ntt)
    loss.backward()
    torch.cuda.synchronize()
    type(layers[0]).forward = orig_fwd
    G.emb_combine = orig_combine
    Mm.G.emb_combine = orig_combine
    rm = jag.row_map.cpu().long()
    live = rm >= 0
    Bt = tt.numel()
    full = {}
    for k, g in grk.items():
        f = torch.zeros(Bt, g.shape[1])
        f[rm[live]] = g.cpu()[:rm.numel()][live]
        full[k] = f

    cpu = [x.cpu() if torch.is_tensor(x) else {k: v.cpu() for k, v in x.items()} for x in batch]
    res = {}
    for tag, bf16 in (('fp32', False), ('amp', True)):
        st = {}
        o, f = hook_oracle(ref, st)
        model_ref.RefHSTU.forward = f
        o_l2f = model_ref.RefBaselineModel.log2feats

        def l2f(self, log_seqs, mask, feats, timestamps=None):
            orig_drop = self.emb_dropout.forward

            def drop(x):
                x.register_hook(lambda g: st.__setitem__('emb', g.detach().float().reshape(-1, g.shape[-1])))
                return orig_drop(x)
            self.emb_dropout.forward = drop
            try:
                return o_l2f(self, log_seqs, mask, feats, timestamps)
            finally:
                self.emb_dropout.forward = orig_drop
        model_ref.RefBaselineModel.log2feats = l2f
        hooks = []
        for nm, mod in (('xi', ref.itemdnn), ('xu', ref.userdnn)):
            def fh(m_, inp, out, nm=nm):
                if 'fwd_' + nm in st:
                    return            # the seq-side call only (log2feats runs first)
                st['fwd_' + nm] = out.detach().float().reshape(-1, out.shape[-1]).clone()
                out.register_hook(lambda g, nm=nm: st.__setitem__(nm, g.detach().float().reshape(-1, g.shape[-1])))
            hooks.append(mod.register_forward_hook(fh))
        TB.oracle_step(ref, cpu, bf16=bf16)
        for hk in hooks:
            hk.remove()
        model_ref.RefHSTU.forward = o
        model_ref.RefBaselineModel.log2feats = o_l2f
        res[tag] = st
    ttf = tt.cpu().reshape(-1)
    user, item = ttf == 2, ttf == 1
    print(f'user rows {int(user.sum())}, item rows {int(item.sum())}')
    print('gradient of            rows   grk err   AMP err   (normwise vs fp32 oracle)')
    # self-consistency of the combine backward: dxu == (xu > 0) * g_emb * sqrt(d), for grk and the oracle
    sc = m.item_emb.embedding_dim ** 0.5
    for tag, src in (('grk', full), ('fp32', res['fp32']), ('amp', res['amp'])):
        for nm, sel in (('user', user), ('item', item)):
            want_xu = (src['fwd_xu'][sel] > 0).float() * src['emb'][sel] * sc
            print(f'  consistency {tag:5s} {nm}: |dxu - mask*g*scale| / |dxu| = '
                  f'{TB.nrel(src["xu"][sel].numpy(), want_xu.numpy()):.3e}')
    want = res['fp32']
    for nm, sel in (('user', user), ('item', item)):
        mk = (want['fwd_xu'][sel] > 0)
        e = [TB.nrel((x['emb'][sel] * mk).numpy(), (want['emb'][sel] * mk).numpy()) for x in (full, res['amp'])]
        print(f'  emb grad on the fp32 xu>0 mask, {nm}: grk {e[0]:.4e} AMP {e[1]:.4e}')
    for k in ['fwd_xi', 'fwd_xu', 'xi', 'xu', 'emb'] + [f'x{i}' for i in range(len(layers))]:
        want = res['fp32'][k]
        for nm, sel in (('user', user), ('item', item)):
            e = [TB.nrel(x[sel].numpy(), want[sel].numpy()) for x in (full[k], res['amp'][k])]
            extra = ''
            if k.startswith('fwd_'):     # ReLU mask flips of the pre-activation against fp32
                fl = [int(((x[sel] > 0) != (want[sel] > 0)).sum()) for x in (full[k], res['amp'][k])]
                extra = f'   relu flips grk {fl[0]} AMP {fl[1]} of {int(sel.sum()) * want.shape[1]}'
            print(f'  {k:20s} {nm:5s} {e[0]:.4e} {e[1]:.4e}{extra}')


if __name__ == '__main__':
    main()
