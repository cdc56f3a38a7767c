"""Generate the golden vectors by IMPORTING THE REFERENCE (run in the dev container only).

    python tests/golden/make_golden.py            # writes tests/golden/*.npz

The reference (/root/reference, GPL-3.0) never travels: only these small
input/output arrays are committed.  Everything is CPU fp32 with
``torch.set_num_threads(1)`` and fixed seeds.

Fixtures:
  emb_ops.npz      -- the reference model's own ``sparse_emb`` / ``item_emb``
                      modules (model/BaseLine/model.py:115,159-165): gather,
                      ``.sum(2)`` bag-sum, dense backward with padding_idx=0.
  mha_h1.npz, mha_h4.npz
                   -- ``FlashMultiHeadAttention`` (model/BaseLine/model.py:10-62)
                      fwd + grads, left-padded causal mask as log2feats builds it.
  model_baseline.npz, model_o1.npz
                   -- one full training step of the reference ``BaselineModel``
                      (BaseLine and BaseLineO1) on a batch produced by the
                      reference ``MyDataset`` + ``collate_fn`` + ``feat2tensor``:
                      state before, logits, loss (main.py:177-185 semantics),
                      every grad, params after one AdamW step.
  dataset.npz      -- ``MyDataset.__getitem__`` + ``collate_fn`` + ``feat2tensor``
                      outputs on a synthetic TencentGR directory.
  save_emb.bin     -- bytes written by the reference ``save_emb``.
  retrieval.npz    -- retrieval file formats: item / id / query files written
                      by the reference ``save_emb`` (as save_item_emb and
                      infer.py:205-209 write them) and a result-id file read
                      back by the reference ``read_result_ids`` (infer.py:51-65);
                      the exact top-10 (float64) the HNSW search approximates.
                      ``python tests/golden/make_golden.py retrieval`` writes
                      only this fixture.
  model_baseline_nf_live.npz, model_o1_nf_live.npz
                   -- the same training step with ``norm_first=True`` (pre-LN
                      blocks, model/BaseLine/model.py:338-342); written by
                      ``python tests/golden/make_golden.py norm_first``.
"""
from __future__ import annotations

import importlib.util
import sys
import tempfile
from pathlib import Path
from types import SimpleNamespace

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
REF = Path('/root/reference/model')
sys.path.insert(0, str(REPO))


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def ref_modules():
    sys.path.insert(0, str(REF / 'BaseLine'))
    ds = _load('dataset', REF / 'BaseLine' / 'dataset.py')
    sys.modules['dataset'] = ds  # O1's model.py does `from dataset import save_emb`
    base = _load('ref_baseline_model', REF / 'BaseLine' / 'model.py')
    o1 = _load('ref_o1_model', REF / 'BaseLineO1' / 'model.py')
    return ds, base, o1


def ref_init(model):
    """model/BaseLine/main.py:95-111 verbatim semantics."""
    for _, p in model.named_parameters():
        if p.dim() >= 2:
            torch.nn.init.xavier_normal_(p.data)
        elif p.dim() == 1:
            torch.nn.init.constant_(p.data, 0.0)
    model.pos_emb.weight.data[0, :] = 0
    model.item_emb.weight.data[0, :] = 0
    model.user_emb.weight.data[0, :] = 0
    for k in model.sparse_emb:
        model.sparse_emb[k].weight.data[0, :] = 0


def save(name, **arrays):
    path = HERE / name
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrays.items()})
    print(f'{path.name}: {path.stat().st_size / 1024:.1f} KiB')


def flat_feats(prefix, feats):
    return {f'{prefix}.{k}': v.numpy() for k, v in feats.items()}


def model_step_fixture(tag, mod, wd, l2, live, args, dset, ft, batch):
    """One full training step of the reference BaselineModel -> model_<tag>.npz."""
    seq, pos, neg, tt, ntt, nat, sf, pf, nf = batch
    torch.manual_seed(0)
    m = mod.BaselineModel(dset.usernum, dset.itemnum, dset.feat_statistics, ft, args)
    ref_init(m)
    if live:
        gl = torch.Generator().manual_seed(7)
        with torch.no_grad():
            for mm in m.modules():
                if isinstance(mm, torch.nn.LayerNorm):
                    mm.weight.fill_(1.0)
            for _, p in m.named_parameters():
                if p.dim() == 1 and not torch.all(p == 1.0):
                    p.copy_(torch.randn(p.shape, generator=gl) * 0.05)
    before = {k: v.detach().clone().numpy() for k, v in m.state_dict().items()}
    opt = torch.optim.AdamW(m.parameters(), lr=args.lr, betas=(0.9, 0.98), weight_decay=wd)
    m.train()
    pl, nl = m(seq, pos, neg, tt, ntt, nat, sf, pf, nf)
    # loss: model/BaseLine/main.py:177-185 (O1 main.py:233-245 has no l2 term)
    crit = torch.nn.BCEWithLogitsLoss(reduction='mean')
    idx = np.where(ntt == 1)
    loss = crit(pl[idx], torch.ones_like(pl)[idx]) + crit(nl[idx], torch.zeros_like(nl)[idx])
    if l2:
        for p in m.item_emb.parameters():
            loss = loss + l2 * torch.norm(p)
    opt.zero_grad()
    loss.backward()
    grads = {f'grad.{k}': p.grad.detach().clone().numpy() for k, p in m.named_parameters() if p.grad is not None}
    opt.step()
    after = {f'after.{k}': v.detach().clone().numpy() for k, v in m.state_dict().items()}
    save(f'model_{tag}.npz', loss=loss.detach().numpy(), pos_logits=pl.detach().numpy(),
         neg_logits=nl.detach().numpy(), weight_decay=wd, l2_emb=l2, lr=args.lr,
         hidden_units=args.hidden_units, num_blocks=args.num_blocks, num_heads=args.num_heads,
         maxlen=args.maxlen, norm_first=bool(getattr(args, 'norm_first', False)),
         **{f'before.{k}': v for k, v in before.items()}, **grads, **after)


def norm_first_golden():
    """model_baseline_nf_live.npz, model_o1_nf_live.npz: the pre-LN blocks
    (``--norm_first``, model/BaseLine/model.py:338-342, BaseLineO1/model.py:451),
    same dataset batch and live init as the other model fixtures."""
    torch.set_num_threads(1)
    ds_mod, base_mod, o1_mod = ref_modules()
    from tencent_recommendation_2025_amd.dataset import write_synthetic_tencentgr
    tmp = Path(tempfile.mkdtemp(prefix='grk_golden_'))
    write_synthetic_tencentgr(tmp, num_users=24, num_items=300, max_events=40, seed=0,
                              sparse_card=(10, 50, 100), user_card=100)
    args = SimpleNamespace(maxlen=20, mm_emb_id=['81'], hidden_units=32, num_blocks=2, num_heads=2,
                           dropout_rate=0.0, norm_first=True, device='cpu', l2_emb=0.001, lr=0.001)
    np.random.seed(0)
    dset = ds_mod.MyDataset(tmp, args)
    batch = ds_mod.MyDataset.collate_fn([dset[u] for u in range(8)])
    ft = dset.feature_types
    for tag, mod, wd, l2 in (('baseline_nf_live', base_mod, 0.01, args.l2_emb), ('o1_nf_live', o1_mod, args.l2_emb, 0.0)):
        model_step_fixture(tag, mod, wd, l2, True, args, dset, ft, batch)


def main():
    torch.set_num_threads(1)
    ds_mod, base_mod, o1_mod = ref_modules()
    from tencent_recommendation_2025_amd.dataset import write_synthetic_tencentgr

    tmp = Path(tempfile.mkdtemp(prefix='grk_golden_'))
    write_synthetic_tencentgr(tmp, num_users=24, num_items=300, max_events=40, seed=0,
                              sparse_card=(10, 50, 100), user_card=100)
    args = SimpleNamespace(maxlen=20, mm_emb_id=['81'], hidden_units=32, num_blocks=2, num_heads=2,
                           dropout_rate=0.0, norm_first=False, device='cpu', l2_emb=0.001, lr=0.001)

    # ---------------- dataset -------------------------------------------------
    np.random.seed(0)
    dset = ds_mod.MyDataset(tmp, args)
    uids = list(range(8))
    samples = [dset[u] for u in uids]
    batch = ds_mod.MyDataset.collate_fn(samples)
    seq, pos, neg, tt, ntt, nat, sf, pf, nf = batch
    ft = dset.feature_types
    model_for_t = base_mod.BaselineModel(dset.usernum, dset.itemnum, dset.feat_statistics, ft, args)
    item_f = ft['item_sparse'] + ft['item_array']
    user_f = ft['user_sparse'] + ft['user_array']

    def t2(feats, fids):
        out = {k: model_for_t.feat2tensor(feats, k) for k in fids}
        for k in ft['item_emb']:  # mm loop of model.py:281-296
            arr = np.zeros((len(feats), len(feats[0]), 32), np.float32)
            for i, s in enumerate(feats):
                for j, d in enumerate(s):
                    if k in d:
                        arr[i, j] = d[k]
            out[k] = torch.from_numpy(arr)
        return out

    seq_t, pos_t, neg_t = t2(sf, item_f + user_f), t2(pf, item_f), t2(nf, item_f)
    save('dataset.npz', uids=np.array(uids), seq=seq, pos=pos, neg=neg, token_type=tt, next_token_type=ntt,
         next_action_type=nat, itemnum=dset.itemnum, usernum=dset.usernum,
         feat_stats=np.array([[int(k), v] for k, v in dset.feat_statistics.items()]),
         **flat_feats('seq_feat', seq_t), **flat_feats('pos_feat', pos_t), **flat_feats('neg_feat', neg_t))
    # the directory generator is deterministic: tests regenerate it with the same seed.

    # ---------------- full training step (BaseLine and O1) --------------------
    # The reference init zeroes every 1-D parameter, LayerNorm gamma included
    # (main.py:100-102), which makes the first step's logits and table grads
    # exactly zero.  The "_live" fixtures apply the same init and then set
    # gamma = 1 and small random biases so that every gradient is non-zero.
    runs = []
    for tag, mod, wd, l2 in (('baseline', base_mod, 0.01, args.l2_emb), ('o1', o1_mod, args.l2_emb, 0.0)):
        runs += [(tag, mod, wd, l2, False), (tag + '_live', mod, wd, l2, True)]
    for tag, mod, wd, l2, live in runs:
        model_step_fixture(tag, mod, wd, l2, live, args, dset, ft, batch)

    # ---------------- embedding ops on the reference's own modules -------------
    torch.manual_seed(1)
    eargs = SimpleNamespace(**{**vars(args), 'hidden_units': 64, 'maxlen': 50})
    stats = dict(dset.feat_statistics)
    stats['106'] = 1000  # user-array table of 1001 rows
    em = base_mod.BaselineModel(dset.usernum, 1000, stats, ft, eargs)
    ref_init(em)
    tab = em.sparse_emb['106']
    g = torch.Generator().manual_seed(2)
    idx = torch.randint(0, 1001, (4, 51), generator=g)
    idx[:, :10] = 0                      # left padding
    idx[0, 10:20] = 7                    # duplicates
    idx[1, 30:40] = idx[1, 20:30]
    idx_arr = torch.randint(0, 1001, (4, 51, 4), generator=g)
    idx_arr[..., 2:] = torch.where(torch.rand(4, 51, 2, generator=g) < 0.5, 0, idx_arr[..., 2:])
    idx_arr[2, :, 1] = 5
    out = tab(idx)
    gout = torch.randn(out.shape, generator=g)
    out.backward(gout)
    dgrad = tab.weight.grad.clone(); tab.weight.grad = None
    bag = tab(idx_arr).sum(2)
    gbag = torch.randn(bag.shape, generator=g)
    bag.backward(gbag)
    dgrad_bag = tab.weight.grad.clone(); tab.weight.grad = None
    item = em.item_emb
    isx = torch.randint(1, 1001, (3, 51), generator=g)
    isx[:, :5] = 0
    multi = [item(isx), item(isx.flip(1)), item(isx.roll(7, 1))]  # three lookups of one table (seq/pos/neg)
    gm = [torch.randn(x.shape, generator=g) for x in multi]
    sum(((x * gg).sum() for x, gg in zip(multi, gm))).backward()
    save('emb_ops.npz', table=tab.weight.detach().numpy(), idx=idx.numpy(), out=out.detach().numpy(),
         gout=gout.numpy(), dgrad=dgrad.numpy(), idx_arr=idx_arr.numpy(), bag=bag.detach().numpy(),
         gbag=gbag.numpy(), dgrad_bag=dgrad_bag.numpy(), item_table=item.weight.detach().numpy(),
         item_idx=np.stack([isx.numpy(), isx.flip(1).numpy(), isx.roll(7, 1).numpy()]),
         item_gout=np.stack([x.numpy() for x in gm]), item_dgrad=item.weight.grad.numpy())

    # ---------------- FlashMultiHeadAttention ---------------------------------
    for H in (1, 4):
        torch.manual_seed(3 + H)
        mha = base_mod.FlashMultiHeadAttention(64, H, 0.0)
        for _, p in mha.named_parameters():
            if p.dim() >= 2:
                torch.nn.init.xavier_normal_(p.data)
            else:
                torch.nn.init.normal_(p.data, std=0.1)
        B, T = 4, 51
        lens = [51, 40, 13, 1]
        token_type = torch.zeros(B, T, dtype=torch.long)
        for b, n in enumerate(lens):
            token_type[b, T - n:] = 1
        x = torch.randn(B, T, 64, requires_grad=True)
        mask = torch.tril(torch.ones(T, T, dtype=torch.bool)).unsqueeze(0) & (token_type != 0).unsqueeze(1)
        y, _ = mha(x, x, x, attn_mask=mask)
        gy = torch.randn(y.shape)
        y.backward(gy)
        save(f'mha_h{H}.npz', x=x.detach().numpy(), token_type=token_type.numpy(), y=y.detach().numpy(),
             gy=gy.numpy(), dx=x.grad.numpy(),
             **{f'p.{k}': v.detach().numpy() for k, v in mha.named_parameters()},
             **{f'g.{k}': v.grad.numpy() for k, v in mha.named_parameters()})

    # ---------------- save_emb bytes ------------------------------------------
    arr = np.arange(12, dtype=np.float32).reshape(3, 4) * 0.5
    ds_mod.save_emb(arr, HERE / 'save_emb.bin')
    print('torch', torch.__version__)


def retrieval_golden():
    ds_mod, base, _ = ref_modules()
    sys.modules['model'] = base  # infer.py: `from model import BaselineModel`
    infer = _load('ref_infer', REF / 'BaseLine' / 'infer.py')
    from oracle.retrieval import mips_topk
    rng = np.random.default_rng(7)
    items = rng.standard_normal((300, 64)).astype(np.float32)
    queries = rng.standard_normal((9, 64)).astype(np.float32)
    ids = (rng.permutation(300) + 1000).astype(np.uint64).reshape(-1, 1)
    out = {}
    with tempfile.TemporaryDirectory() as d:
        for name, arr in (('items', items), ('queries', queries), ('ids', ids)):
            ds_mod.save_emb(arr, Path(d, name))
            out[f'{name}_bytes'] = np.frombuffer(Path(d, name).read_bytes(), dtype=np.uint8)
        scores, top = mips_topk(queries, items, 10, ids.reshape(-1).astype(np.int64))
        res = np.concatenate([np.array([9, 10], dtype=np.uint32).view(np.uint8),
                              top.astype(np.uint64).view(np.uint8).reshape(-1)])
        Path(d, 'res').write_bytes(res.tobytes())
        read = infer.read_result_ids(Path(d, 'res'))
    save('retrieval.npz', items=items, queries=queries, ids=ids, top10_scores=scores, top10_ids=top,
         result_bytes=res, result_read_by_reference=read, **out)


if __name__ == '__main__':
    if sys.argv[1:] == ['retrieval']:
        retrieval_golden()
    elif sys.argv[1:] == ['norm_first']:
        norm_first_golden()
    else:
        main()
