"""Where do the bf16 jagged and padded training steps part?  (round 4 diagnostic)

One bf16-autocast fused-trainer step of the test_gpu_jagged configuration, padded
and jagged, from the same parameters; every intermediate the model hands between
modules (the feat2emb outputs, each HSTU layer's input / output, log_feats, the
pos / neg embeddings) is kept with its gradient, and the jagged rows are compared
with the padded rows they hold (jagged.row_map), forward and backward, in the
order the backward visits them.

    python scripts/diag/jagged_vs_padded.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

DEV = 'cuda'


def nrel(a, b):
    a, b = a.double(), b.double()
    d = b.norm()
    return float((a - b).norm() / (d if d > 0 else 1.0))


def run(jagged, batch, state):
    from tencent_recommendation_2025_amd import synthetic as S
    from tencent_recommendation_2025_amd.model import BaselineModel, init_reference_
    from tencent_recommendation_2025_amd.optim import FusedAdamW
    from tencent_recommendation_2025_amd.train import Trainer
    cfg = S.SyntheticConfig(batch_size=16, maxlen=60, num_items=4000, num_users=500, min_len=4)
    stats, types = S.feature_schema(cfg)
    m = BaselineModel(cfg.num_users, cfg.num_items, stats, types,
                      S.make_args(hidden_units=128, maxlen=60, num_blocks=2, num_heads=2)).to(DEV)
    if state is None:
        torch.manual_seed(0)
        init_reference_(m, seed=0, live_norms=True)
        state = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m.load_state_dict(state)
    opt = FusedAdamW(m, lr=1e-3, defer_period=4)
    tr = Trainer(m, opt, loss='bce', jagged=jagged, jagged_quantum=128)
    kept = {}

    def keep(name, t):
        if isinstance(t, torch.Tensor) and t.requires_grad:
            t.retain_grad()
            kept.setdefault(name, []).append(t)

    hooks = []
    for i, layer in enumerate(m.attention_layers):
        hooks.append(layer.register_forward_hook(
            lambda mod, inp, out, i=i: (keep(f'layer{i}.in', inp[0]), keep(f'layer{i}.out', out[0]))))
    orig_embed = m._embed

    def embed(*a, **kw):
        x, pos_rows = orig_embed(*a, **kw)
        keep(f"embed.{kw.get('role', 'seq')}", x)
        return x, pos_rows
    m._embed = embed
    orig_encode = m.encode

    def encode(*a, **kw):
        h, pe, ne = orig_encode(*a, **kw)
        keep('log_feats', h)
        keep('pos_emb_out', pe)
        keep('neg_emb_out', ne)
        return h, pe, ne
    m.encode = encode
    opt.zero_grad()
    opt.begin_step(batch)
    loss = tr.compute_loss(batch)
    loss.backward()
    jag = None
    if jagged:
        from tencent_recommendation_2025_amd import jagged as J
        jag = J.layout(batch[3], J.capacity_for(J.span_rows(batch[3]), 128), batch[4])
    grads = {n: p.grad.detach().float().clone() for n, p in m.named_parameters() if p.grad is not None}
    for grp in opt.groups:
        grads['group.' + grp.name] = grp.dense_gradient().float().clone()
    return state, float(loss), kept, grads, jag


def main():
    from tencent_recommendation_2025_amd import synthetic as S
    cfg = S.SyntheticConfig(batch_size=16, maxlen=60, num_items=4000, num_users=500, min_len=4)
    g = torch.Generator(device=DEV).manual_seed(3)
    batch = S.make_batch(cfg, g, DEV)
    state, lp, kp, gp, _ = run(False, batch, None)
    _, lj, kj, gj, jag = run(True, batch, state)
    B, T = batch[0].shape
    rm = jag.row_map.long()
    live = rm >= 0
    src = rm[live]
    print(f'loss padded {lp:.8f} jagged {lj:.8f} rel {abs(lp - lj) / abs(lp):.2e}')
    for name in kp:
        for idx, (tp, tj) in enumerate(zip(kp[name], kj.get(name, []))):
            D = tp.shape[-1]
            P = tp.detach().reshape(-1, D)
            Jt = tj.detach().reshape(-1, D)
            reps = P.shape[0] // (B * T)      # the pair lookups stack pos | neg
            if reps != 1:
                src2 = torch.cat([src + r * B * T for r in range(reps)])
                live2 = live.repeat(reps)
            else:
                src2, live2 = src, live
            fw = nrel(Jt[live2].float(), P[src2].float())
            gline = ''
            if tp.grad is not None and tj.grad is not None:
                Gp = tp.grad.reshape(-1, D).float()
                Gj = tj.grad.reshape(-1, D).float()
                diff = (Gj[live2] - Gp[src2]).abs()
                dead = Gj[~live2].abs().max().item() if (~live2).any() else 0.0
                # padded rows no jagged row holds (the padding before each span)
                held = torch.zeros(P.shape[0], dtype=torch.bool, device=P.device)
                held[src2] = True
                pad = Gp[~held].abs().max().item() if (~held).any() else 0.0
                gline = (f' grad nrel {nrel(Gj[live2], Gp[src2]):.2e} diff>0 {int((diff > 0).sum())}/{diff.numel()}'
                         f' | jagged dead-row grad max {dead:.2e} | padded padding-row grad max {pad:.2e}')
            print(f'{name}[{idx}]: fwd nrel {fw:.2e}{gline}')
    for k in sorted(gp, key=lambda k: -nrel(gj[k], gp[k]))[:12]:
        print(f'param {k}: {nrel(gj[k], gp[k]):.2e}')


if __name__ == '__main__':
    main()
