"""CPU experiment (round 6): does the projected-table restatement's extra bf16
rounding of the dnn pre-activation explain grk's user-table gradient error at the
bench configuration (tests/test_gpu_bench_size.py: user tables 3.8e-2 vs the AMP
step's 2.4e-2)?

Runs the fp32 oracle step, the AMP (CPU bf16 autocast) oracle step, and the AMP step
with feat2emb restated as grk computes it (P_f = bf16(E_f W_f^T), the bag sum of P
rounded to bf16 in the gather buffer, added to the bf16 [row | 1] GEMM in the
store), and prints each table's normwise gradient error against fp32.

    python scripts/diag/proj_rounding.py [B]
"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), 'tests'))

from oracle import model_ref  # noqa: E402
import test_gpu_bench_size as T  # noqa: E402


def r16(x):
    return x.to(torch.bfloat16).to(torch.float32)


def dnn_projected(dnn, row, feats, d, mode):
    """relu(dnn(cat(row, feats...))) as grk's projection restatement computes it.
    feats: list of ('sparse'|'array', embedding module, idx) then ('dense', tensor)."""
    W, b = dnn.weight, dnn.bias
    blocks = [row]
    col = d
    acc = None
    dense_cols = []
    for kind, emb, t in feats:
        if kind == 'dense':
            dense_cols.append((col, t))
            col += d
            continue
        Wf = W[:, col:col + d]
        col += d
        P = emb.weight @ Wf.t()                         # autocast: bf16 out (P_f in bf16)
        g = F.embedding(t, P.float())
        if kind == 'array':
            g = g.sum(2)
        acc = g if acc is None else acc + g
    parts = [row] + [x for _, x in dense_cols]
    Wm = torch.cat([W[:, :d]] + [W[:, c:c + d] for c, _ in dense_cols], 1)
    y = F.linear(torch.cat(parts, 2), Wm, b)           # autocast: bf16 GEMM of the direct blocks
    if acc is None:
        return torch.relu(y)
    if mode == 'proj':
        pre = r16(y.float() + r16(acc))                # sum of P rounded (gather buffer), one store rounding
    else:                                              # 'proj_f32sum': the bag sum kept in fp32
        pre = r16(y.float() + acc)
    return torch.relu(pre)


def make_feat2emb(mode):
    def feat2emb(self, seq, feats, mask=None, include_user=False, role=None):
        d = self.item_emb.embedding_dim
        if include_user:
            irow, urow = self.item_emb((mask == 1) * seq), self.user_emb((mask == 2) * seq)
        else:
            irow = self.item_emb(seq)
        ifeats = [('sparse', self.sparse_emb[k], feats[k]) for k in self.ITEM_SPARSE_FEAT]
        ifeats += [('array', self.sparse_emb[k], feats[k]) for k in self.ITEM_ARRAY_FEAT]
        ifeats += [('dense', None, self.emb_transform[k](feats[k])) for k in self.ITEM_EMB_FEAT]
        x = dnn_projected(self.itemdnn, irow, ifeats, d, mode)
        if include_user:
            ufeats = [('sparse', self.sparse_emb[k], feats[k]) for k in self.USER_SPARSE_FEAT]
            ufeats += [('array', self.sparse_emb[k], feats[k]) for k in self.USER_ARRAY_FEAT]
            x = x + dnn_projected(self.userdnn, urow, ufeats, d, mode)
        return x
    return feat2emb


def main():
    from tencent_recommendation_2025_amd import synthetic as S
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    T.B = B
    torch.set_num_threads(8)
    cfg, stats, types, args, ref = T.oracle_setup()
    cfg.batch_size = B
    batch = S.make_batch(cfg, torch.Generator().manual_seed(7), 'cpu')
    cpu = list(batch)
    g32 = T.oracle_step(ref, cpu, bf16=False)[3]
    gamp = T.oracle_step(ref, cpu, bf16=True)[3]
    orig = model_ref.RefBaselineModel.feat2emb
    res = {}
    for mode in ('proj', 'proj_f32sum'):
        model_ref.RefBaselineModel.feat2emb = make_feat2emb(mode)
        res[mode] = T.oracle_step(ref, cpu, bf16=True)[3]
    model_ref.RefBaselineModel.feat2emb = orig
    # the grk HSTU core's bf16 storage points (RefHSTU.bf16_core), with and without the projection
    for layer in ref.attention_layers:
        layer.bf16_core = True
    res['core'] = T.oracle_step(ref, cpu, bf16=True)[3]
    model_ref.RefBaselineModel.feat2emb = make_feat2emb('proj')
    res['core+proj'] = T.oracle_step(ref, cpu, bf16=True)[3]
    model_ref.RefBaselineModel.feat2emb = orig
    for layer in ref.attention_layers:
        layer.bf16_core = False
    # grk's bf16 residual stream (model.log2feats: add_norm keeps seqs in bf16; its
    # gradient is a bf16 tensor too)
    orig_l2f = model_ref.RefBaselineModel.log2feats

    def log2feats_bf16res(self, log_seqs, mask, feats, timestamps=None):
        B_, T_ = log_seqs.shape
        rb = model_ref._RoundBF16.apply
        seqs = self.feat2emb(log_seqs, feats, mask=mask, include_user=True)
        seqs = seqs * self.item_emb.embedding_dim ** 0.5
        poss = torch.arange(1, T_ + 1).unsqueeze(0).expand(B_, -1) * (log_seqs != 0)
        seqs = rb(self.emb_dropout(seqs + self.pos_emb(poss)))
        attn_mask = torch.tril(torch.ones((T_, T_), dtype=torch.bool)).unsqueeze(0) & (mask != 0).unsqueeze(1)
        for i in range(len(self.attention_layers)):
            y, _ = self.attention_layers[i](*(3 * (self.attention_layernorms[i](seqs),)), attn_mask=attn_mask,
                                            timestamps=timestamps, key_valid=(mask != 0))
            seqs = rb(seqs + y)
        return self.last_layernorm(seqs)
    model_ref.RefBaselineModel.log2feats = log2feats_bf16res
    res['bf16res'] = T.oracle_step(ref, cpu, bf16=True)[3]
    model_ref.RefBaselineModel.feat2emb = make_feat2emb('proj')
    res['bf16res+proj'] = T.oracle_step(ref, cpu, bf16=True)[3]
    model_ref.RefBaselineModel.feat2emb = orig
    model_ref.RefBaselineModel.log2feats = orig_l2f
    user = set(types['user_sparse']) | set(types['user_array'])
    cols = (gamp, res['proj'], res['proj_f32sum'], res['bf16res'], res['bf16res+proj'])
    print(f'B={B}: table, group, AMP, AMP+proj, AMP+proj(fp32 bag sum), AMP+bf16 residual, AMP+bf16 residual+proj')
    for n, w in g32.items():
        if not n.startswith(('sparse_emb.', 'item_emb', 'user_emb')) or float(w[1:].norm()) == 0:
            continue
        key = n.split('.')[1] if n.startswith('sparse_emb.') else n
        e = [T.nrel(x[n][1:].float(), w[1:]) for x in cols]
        print(f'  {n:28s} {"user" if key in user or n.startswith("user") else "item":4s} '
              + ' '.join(f'{v:.4e}' for v in e))
    for n in ('itemdnn.weight', 'userdnn.weight', 'attention_layers.0.uvqk.weight'):
        e = [T.nrel(x[n].float(), g32[n]) for x in cols]
        print(f'  {n:28s} dense ' + ' '.join(f'{v:.4e}' for v in e))


if __name__ == '__main__':
    main()
