"""fp32 torch-CPU restatement of the reference model + training step.  TEST INFRASTRUCTURE ONLY.

This is (1) the full-model checker for the HIP path and (2) ``bench.py``'s
``cpu_baseline`` leg (kind "port").  It is an independent restatement of the
reference's ``BaselineModel`` (``model/BaseLine/model.py:81-433``,
``model/BaseLineO1/model.py:167-555``) operating on tensorised features
(``{fid: LongTensor[B,T] | LongTensor[B,T,A] | FloatTensor[B,T,E]}``) instead of
lists of dicts; ``feat2tensor`` (``model/BaseLine/model.py:186-224``) is
restated by ``tensorize_features`` for the golden comparison.  Parameter names
equal the reference's state_dict keys, so a reference checkpoint loads as is.

Pinned: the softmax variants ("baseline" = Conv1d FFN, "o1" = SwiGLU FFN)
against ``tests/golden/model_*.npz`` produced by the imported reference.
The "hstu" block and the sampled-softmax loss are north-star only
(**parity unpinned**) and restate ``oracle/hstu.py`` / ``oracle/loss.py``.
"""
from __future__ import annotations

import math
from types import SimpleNamespace

import numpy as np
import torch
import torch.nn.functional as F

from . import hstu

EMB_SHAPE = {"81": 32, "82": 1024, "83": 3584, "84": 4096, "85": 3584, "86": 3584}  # model/BaseLine/model.py:183


class RefMHA(torch.nn.Module):
    """FlashMultiHeadAttention restated (model/BaseLine/model.py:10-62)."""

    def __init__(self, d, h, p):
        super().__init__()
        self.hidden_units, self.num_heads, self.head_dim, self.dropout_rate = d, h, d // h, p
        self.q_linear = torch.nn.Linear(d, d)
        self.k_linear = torch.nn.Linear(d, d)
        self.v_linear = torch.nn.Linear(d, d)
        self.out_linear = torch.nn.Linear(d, d)

    def forward(self, query, key, value, attn_mask=None):
        B, T, _ = query.shape
        sh = lambda x: x.view(B, T, self.num_heads, self.head_dim).transpose(1, 2)
        q, k, v = sh(self.q_linear(query)), sh(self.k_linear(key)), sh(self.v_linear(value))
        o = F.scaled_dot_product_attention(q, k, v, dropout_p=self.dropout_rate if self.training else 0.0,
                                           attn_mask=attn_mask.unsqueeze(1))
        return self.out_linear(o.transpose(1, 2).contiguous().view(B, T, self.hidden_units)), None


class _RoundBF16(torch.autograd.Function):
    """x rounded to bf16 (kept in x's dtype); the gradient rounded to bf16 as well."""

    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).to(g.dtype)


class RefHSTU(torch.nn.Module):
    """HSTU layer (parity unpinned; see oracle/hstu.py).  Same math, torch autograd.

    bf16_core=True: the fp32 math fed the grk HSTU core's bf16 storage points
    (ops.hstu_core: the u|v|q|k pre-activation, the attention output o and the
    gated output y are bf16 tensors, and so are their gradients dpre, do, dy;
    the MFMA operands SiLU(q), SiLU(k), SiLU(v) and the gate SiLU(u) are bf16
    values, csrc/grk_hstu.hip k_ng_fwd) -- the checker that separates that
    rounding from the kernels' math.  With fp8=True the same points as
    functional._HSTUFp8Fn: SiLU(v|q|k) of the bf16 pre-activation rounded once
    to e4m3, their gradients stored as bf16."""

    def __init__(self, d, h, p, num_buckets, num_time_buckets=0, fp8=False):
        super().__init__()
        self.hidden_units, self.num_heads, self.head_dim, self.dropout_rate = d, h, d // h, p
        self.fp8 = fp8  # config C5: SiLU'd q/k/v rounded to OCP e4m3, straight-through gradient
        self.bf16_core = False
        self.uvqk = torch.nn.Linear(d, 4 * d)
        self.rab = torch.nn.Parameter(torch.zeros(h, num_buckets))
        self.rab_t = torch.nn.Parameter(torch.zeros(h, num_time_buckets)) if num_time_buckets else None
        self.attn_norm = torch.nn.LayerNorm(d, eps=1e-8)
        self.out_linear = torch.nn.Linear(d, d)

    def forward(self, query, key, value, attn_mask=None, timestamps=None, key_valid=None):
        B, T, D = query.shape
        rb = _RoundBF16.apply if self.bf16_core else (lambda x: x)
        u, v, q, k = torch.split(F.silu(rb(self.uvqk(query))), D, dim=-1)
        r16 = lambda x: x + (x.to(torch.bfloat16).to(x.dtype) - x).detach()
        if self.fp8:
            # e4m3(SiLU(pre)) in ONE rounding from the fp32 SiLU of the (bf16) pre-activation, as
            # grk_silu_fp8 does; straight-through gradient.  bf16_core: the gate SiLU(u) is a bf16
            # value (k_ng_fwd) and the attention's dq / dk / dv are stored as bf16 before
            # grk_dsilu_mul (rb on the e4m3 values: identity forward, every e4m3 value is a bf16 one)
            r8 = lambda x: x + (x.clamp(-448, 448).to(torch.float8_e4m3fn).to(x.dtype) - x).detach()
            v, q, k = r8(v), r8(q), r8(k)
            if self.bf16_core:
                u = r16(u)
                v, q, k = rb(v), rb(q), rb(k)
        elif self.bf16_core:   # SiLU(v), SiLU(q), SiLU(k) (MFMA operands) and the gate SiLU(u) are bf16 values
            u, v, q, k = (r16(x) for x in (u, v, q, k))
        sh = lambda x: x.reshape(B, T, self.num_heads, self.head_dim).transpose(1, 2)
        q, k, v = sh(q), sh(k), sh(v)
        nb = self.rab.shape[1]
        i = torch.arange(T)[:, None]
        j = torch.arange(T)[None, :]
        bucket = (i - j).clamp(0, nb - 1)
        s = torch.matmul(q, k.transpose(-1, -2)) * self.head_dim ** -0.5 + self.rab[:, bucket][None]
        if timestamps is not None and self.rab_t is not None:   # time bias (hstu.py _time_bias)
            _, bt = hstu._time_bias(np.asarray(timestamps), np.asarray(key_valid), np.zeros(self.rab_t.shape))
            s = s + self.rab_t[:, torch.from_numpy(bt)].transpose(0, 1)
        a = F.silu(s) * (1.0 / T) * attn_mask.unsqueeze(1).to(s.dtype)
        o = rb(torch.matmul(a, v).transpose(1, 2).contiguous().view(B, T, D))
        y = rb(self.attn_norm(o) * u)
        y = F.dropout(y, self.dropout_rate, self.training)
        return self.out_linear(y), None


class RefConvFFN(torch.nn.Module):
    """PointWiseFeedForward restated (model/BaseLine/model.py:65-78)."""

    def __init__(self, d, p):
        super().__init__()
        self.conv1 = torch.nn.Conv1d(d, d, kernel_size=1)
        self.dropout1 = torch.nn.Dropout(p)
        self.relu = torch.nn.ReLU()
        self.conv2 = torch.nn.Conv1d(d, d, kernel_size=1)
        self.dropout2 = torch.nn.Dropout(p)

    def forward(self, x):
        y = self.dropout2(self.conv2(self.relu(self.dropout1(self.conv1(x.transpose(-1, -2))))))
        return y.transpose(-1, -2)


def swiglu_hidden(d, multiple_of=256):
    """Hidden width of PackedSwiGLUFFN (model/BaseLineO1/model.py:128-133)."""
    h = 4 * d
    return multiple_of * ((h + multiple_of - 1) // multiple_of)


class RefSwiGLU(torch.nn.Module):
    """PackedSwiGLUFFN restated (model/BaseLineO1/model.py:103-164)."""

    def __init__(self, d, p):
        super().__init__()
        hid = swiglu_hidden(d)
        self.w13 = torch.nn.Linear(d, 2 * hid, bias=False)
        self.w2 = torch.nn.Linear(hid, d, bias=False)
        self.dropout = torch.nn.Dropout(p) if p > 0 else None

    def forward(self, x):
        a, b = torch.chunk(self.w13(x), 2, dim=-1)
        y = self.w2(F.silu(a) * b)
        return self.dropout(y) if self.dropout is not None else y


class RefBaselineModel(torch.nn.Module):
    """BaselineModel restated (model/BaseLine/model.py:104-167; O1 :176-260).

    ``variant``: "baseline" (Conv1d FFN) | "o1" (SwiGLU FFN).
    ``block``:   "softmax" (reference) | "hstu" (north star, no FFN).
    """

    def __init__(self, user_num, item_num, feat_statistics, feat_types, args, variant="baseline", block="softmax"):
        super().__init__()
        d = args.hidden_units
        self.maxlen, self.norm_first, self.block, self.variant = args.maxlen, args.norm_first, block, variant
        self.item_emb = torch.nn.Embedding(item_num + 1, d, padding_idx=0)
        self.user_emb = torch.nn.Embedding(user_num + 1, d, padding_idx=0)
        self.pos_emb = torch.nn.Embedding(2 * args.maxlen + 1, d, padding_idx=0)
        self.emb_dropout = torch.nn.Dropout(p=args.dropout_rate)
        self.sparse_emb = torch.nn.ModuleDict()
        self.emb_transform = torch.nn.ModuleDict()
        self.attention_layernorms = torch.nn.ModuleList()
        self.attention_layers = torch.nn.ModuleList()
        self.forward_layernorms = torch.nn.ModuleList()
        self.forward_layers = torch.nn.ModuleList()
        self.USER_SPARSE_FEAT = {k: feat_statistics[k] for k in feat_types['user_sparse']}
        self.USER_CONTINUAL_FEAT = feat_types['user_continual']
        self.ITEM_SPARSE_FEAT = {k: feat_statistics[k] for k in feat_types['item_sparse']}
        self.ITEM_CONTINUAL_FEAT = feat_types['item_continual']
        self.USER_ARRAY_FEAT = {k: feat_statistics[k] for k in feat_types['user_array']}
        self.ITEM_ARRAY_FEAT = {k: feat_statistics[k] for k in feat_types['item_array']}
        self.ITEM_EMB_FEAT = {k: EMB_SHAPE[k] for k in feat_types['item_emb']}
        userdim = d * (len(self.USER_SPARSE_FEAT) + 1 + len(self.USER_ARRAY_FEAT)) + len(self.USER_CONTINUAL_FEAT)
        itemdim = (d * (len(self.ITEM_SPARSE_FEAT) + 1 + len(self.ITEM_ARRAY_FEAT)) + len(self.ITEM_CONTINUAL_FEAT)
                   + d * len(self.ITEM_EMB_FEAT))
        self.userdnn = torch.nn.Linear(userdim, d)
        self.itemdnn = torch.nn.Linear(itemdim, d)
        self.last_layernorm = torch.nn.LayerNorm(d, eps=1e-8)
        T = args.maxlen + 1
        for _ in range(args.num_blocks):
            self.attention_layernorms.append(torch.nn.LayerNorm(d, eps=1e-8))
            if block == "hstu":
                self.attention_layers.append(RefHSTU(d, args.num_heads, args.dropout_rate, T,
                                                     getattr(args, 'hstu_time_buckets', 0) or 0,
                                                     fp8=bool(getattr(args, 'hstu_fp8', False))))
                continue
            self.attention_layers.append(RefMHA(d, args.num_heads, args.dropout_rate))
            self.forward_layernorms.append(torch.nn.LayerNorm(d, eps=1e-8))
            self.forward_layers.append(RefConvFFN(d, args.dropout_rate) if variant == "baseline"
                                       else RefSwiGLU(d, args.dropout_rate))
        for group in (self.USER_SPARSE_FEAT, self.ITEM_SPARSE_FEAT, self.ITEM_ARRAY_FEAT, self.USER_ARRAY_FEAT):
            for k in group:
                self.sparse_emb[k] = torch.nn.Embedding(group[k] + 1, d, padding_idx=0)
        for k in self.ITEM_EMB_FEAT:
            self.emb_transform[k] = torch.nn.Linear(self.ITEM_EMB_FEAT[k], d)

    # The dnn outputs' ReLU masks may be given (``relu_masks``): {(role, 'item' | 'user'):
    # (mask bool [B, T, d], rows bool [B, T])} replaces relu(y) by y * mask on those rows
    # of that call (the own y > 0 elsewhere) -- role 'seq' (log2feats), 'pos', 'neg'
    # (forward).  Test infrastructure: fed the HIP model's own masks, the oracle's
    # gradients separate the forward's ReLU-boundary flips (a discontinuous function of
    # the forward rounding) from the smooth arithmetic error (tests/test_gpu_bench_size.py).
    relu_masks = None

    def _act(self, y, role, which):
        m = None if self.relu_masks is None else self.relu_masks.get((role, which))
        if m is None:
            return torch.relu(y)
        keep = torch.where(m[1][..., None], m[0], y > 0)
        return y * keep.to(y.dtype)

    # --- model/BaseLine/model.py:226-310 -------------------------------------
    def feat2emb(self, seq, feats, mask=None, include_user=False, role=None):
        if include_user:
            item_list = [self.item_emb((mask == 1) * seq)]
            user_list = [self.user_emb((mask == 2) * seq)]
        else:
            item_list = [self.item_emb(seq)]
        groups = [(self.ITEM_SPARSE_FEAT, 'sparse', item_list), (self.ITEM_ARRAY_FEAT, 'array', item_list)]
        if include_user:
            groups += [(self.USER_SPARSE_FEAT, 'sparse', user_list), (self.USER_ARRAY_FEAT, 'array', user_list)]
        for group, kind, out in groups:
            for k in group:
                t = feats[k]
                out.append(self.sparse_emb[k](t) if kind == 'sparse' else self.sparse_emb[k](t).sum(2))
        for k in self.ITEM_EMB_FEAT:
            item_list.append(self.emb_transform[k](feats[k]))
        x = self._act(self.itemdnn(torch.cat(item_list, dim=2)), role, 'item')
        if include_user:
            x = x + self._act(self.userdnn(torch.cat(user_list, dim=2)), role, 'user')
        return x

    # --- model/BaseLine/model.py:312-350 -------------------------------------
    def log2feats(self, log_seqs, mask, feats, timestamps=None):
        B, T = log_seqs.shape
        seqs = self.feat2emb(log_seqs, feats, mask=mask, include_user=True, role='seq')
        seqs = seqs * self.item_emb.embedding_dim ** 0.5
        poss = torch.arange(1, T + 1).unsqueeze(0).expand(B, -1) * (log_seqs != 0)
        seqs = self.emb_dropout(seqs + self.pos_emb(poss))
        attn_mask = torch.tril(torch.ones((T, T), dtype=torch.bool)).unsqueeze(0) & (mask != 0).unsqueeze(1)
        for i in range(len(self.attention_layers)):
            if self.block == "hstu":
                y, _ = self.attention_layers[i](*(3 * (self.attention_layernorms[i](seqs),)), attn_mask=attn_mask,
                                                timestamps=timestamps, key_valid=(mask != 0))
                seqs = seqs + y
            elif self.norm_first:
                x = self.attention_layernorms[i](seqs)
                seqs = seqs + self.attention_layers[i](x, x, x, attn_mask=attn_mask)[0]
                seqs = seqs + self.forward_layers[i](self.forward_layernorms[i](seqs))
            else:
                seqs = self.attention_layernorms[i](seqs + self.attention_layers[i](seqs, seqs, seqs, attn_mask=attn_mask)[0])
                seqs = self.forward_layernorms[i](seqs + self.forward_layers[i](seqs))
        return self.last_layernorm(seqs)

    # --- model/BaseLine/model.py:352-384 -------------------------------------
    def forward(self, seq, pos, neg, token_type, next_token_type, seq_feat, pos_feat, neg_feat, return_embs=False,
                timestamps=None):
        h = self.log2feats(seq, token_type, seq_feat, timestamps)
        lm = (next_token_type == 1)
        pe = self.feat2emb(pos, pos_feat, include_user=False, role='pos')
        ne = self.feat2emb(neg, neg_feat, include_user=False, role='neg')
        pl = (h * pe).sum(-1) * lm
        nl = (h * ne).sum(-1) * lm
        if return_embs:
            return pl, nl, h, pe, ne
        return pl, nl

    def predict(self, log_seqs, seq_feat, mask):
        return self.log2feats(log_seqs, mask, seq_feat)[:, -1, :]


def init_params(model, seed=0):
    """Reference init (model/BaseLine/main.py:95-111): xavier_normal_ for dim>=2,
    zeros for 1-D, then zero the padding rows of every table."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for _, p in model.named_parameters():
            if p.dim() >= 2:
                fan_in, fan_out = torch.nn.init._calculate_fan_in_and_fan_out(p)
                std = math.sqrt(2.0 / float(fan_in + fan_out))
                p.copy_(torch.randn(p.shape, generator=g) * std)
            elif p.dim() == 1:
                p.zero_()
        for t in [model.pos_emb, model.item_emb, model.user_emb] + list(model.sparse_emb.values()):
            t.weight[0].zero_()


def bce_loss(pos_logits, neg_logits, next_token_type, model=None, l2_emb=0.0):
    """Training loss (model/BaseLine/main.py:177-185; O1 main.py:233-245)."""
    sel = next_token_type == 1
    loss = F.binary_cross_entropy_with_logits(pos_logits[sel], torch.ones_like(pos_logits[sel]))
    loss = loss + F.binary_cross_entropy_with_logits(neg_logits[sel], torch.zeros_like(neg_logits[sel]))
    if l2_emb and model is not None:  # BaseLine only: main.py:184-185
        loss = loss + l2_emb * torch.norm(model.item_emb.weight)
    return loss


def sampled_softmax_loss(h, pos_emb, pos_ids, next_token_type, tau, log_q=None):
    """In-batch sampled softmax (parity unpinned; oracle/loss.py); log_q: the logQ
    correction subtracted from every logit of a column."""
    D = h.shape[-1]
    hv = h.reshape(-1, D); ev = pos_emb.reshape(-1, D)
    ids = pos_ids.reshape(-1); valid = (next_token_type.reshape(-1) == 1)
    n = hv.shape[0]
    z = hv @ ev.t() / tau
    if log_q is not None:
        z = z - log_q.reshape(1, -1).to(z.dtype)
    same = (ids[:, None] == ids[None, :]) & ~torch.eye(n, dtype=torch.bool, device=hv.device)
    z = z.masked_fill(~valid[None, :] | same, float('-inf'))
    lse = torch.logsumexp(z, dim=1)
    per = lse - z.diagonal()
    cnt = valid.sum().clamp(min=1)
    return torch.where(valid, per, torch.zeros_like(per)).sum() / cnt


def tensorize_features(feat_list, fids, array_fids=(), emb_fids=()):
    """Restates feat2tensor (model/BaseLine/model.py:186-224) and the mm loop
    (:281-296): list of per-sequence object arrays of dicts -> tensors."""
    out = {}
    B = len(feat_list)
    for k in fids:
        if k in array_fids:
            A = max(max(len(d[k]) for d in s) for s in feat_list)
            T = max(len(s) for s in feat_list)
            arr = np.zeros((B, T, A), np.int64)
            for i, s in enumerate(feat_list):
                for j, d in enumerate(s):
                    v = d[k][:A]
                    arr[i, j, :len(v)] = v
            out[k] = torch.from_numpy(arr)
        elif k in emb_fids:
            T = len(feat_list[0])
            arr = np.zeros((B, T, EMB_SHAPE[k]), np.float32)
            for i, s in enumerate(feat_list):
                for j, d in enumerate(s):
                    if k in d:
                        arr[i, j] = d[k]
            out[k] = torch.from_numpy(arr)
        else:
            arr = np.array([[d[k] for d in s] for s in feat_list], dtype=np.int64)
            out[k] = torch.from_numpy(arr)
    return out


def make_args(**kw):
    base = dict(hidden_units=64, maxlen=50, num_blocks=2, num_heads=4, dropout_rate=0.0, norm_first=False,
                device='cpu', l2_emb=0.0, lr=1e-3)
    base.update(kw)
    return SimpleNamespace(**base)
