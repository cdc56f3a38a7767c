"""Drop-in ``BaselineModel`` for the TencentGR training script, on the grk HIP path.

Keeps the reference's module surface:
``BaselineModel(user_num, item_num, feat_statistics, feat_types, args)``,
``forward(user_item, pos_seqs, neg_seqs, mask, next_mask, next_action_type,
seq_feature, pos_feature, neg_feature) -> (pos_logits, neg_logits)``,
``predict``, ``save_item_emb``, the sub-module contract
``attention_layers[i](q, k, v, attn_mask=[B,T,T]) -> (out, None)`` and every
state_dict key (``model/BaseLine/model.py:81-433``,
``model/BaseLineO1/model.py:167-555``).  ``args`` may carry three optional
fields the reference does not have:

* ``variant``: "baseline" (Conv1d FFN, default) | "o1" (PackedSwiGLUFFN);
* ``block``:   "softmax" (reference attention, default) | "hstu" (north-star
  HSTU layer; no FFN, pre-norm residual);
* ``hstu_num_buckets``: relative-position buckets (default maxlen + 1).

Device work: all table lookups of a feat2emb call are ONE fused gather
launch (``grk_embedding_gather``) writing the concatenated itemdnn/userdnn
operands in place; attention is ``grk_attention_*``; logits are
``grk_pair_logits_*``.  Features may be the reference's lists of dicts (they
are tensorised on the host, as ``feat2tensor`` does) or dicts of tensors
(``MyDataset.collate_tensor_fn``).
"""
from __future__ import annotations

import contextlib
from pathlib import Path

import numpy as np
import torch
import torch.nn.functional as F

from . import _lib as L
from . import functional as G
from . import kernels as K
from .dataset import MM_SHAPE, save_emb, tensorize


class FlashMultiHeadAttention(torch.nn.Module):
    """Softmax MHA (model/BaseLine/model.py:10-62) on grk_attention_fwd/bwd.

    Q/K/V come from one GEMM with the three weights concatenated at call time
    (state_dict keys unchanged); the kernel reads the packed [B*T, 3D] result
    directly, with the mask given as causal + per-key validity instead of a
    materialised [B,T,T] tensor."""

    def __init__(self, hidden_units, num_heads, dropout_rate):
        super().__init__()
        assert hidden_units % num_heads == 0, 'hidden_units must be divisible by num_heads'
        self.hidden_units, self.num_heads = hidden_units, num_heads
        self.head_dim = hidden_units // num_heads
        self.dropout_rate = dropout_rate
        self.q_linear = torch.nn.Linear(hidden_units, hidden_units)
        self.k_linear = torch.nn.Linear(hidden_units, hidden_units)
        self.v_linear = torch.nn.Linear(hidden_units, hidden_units)
        self.out_linear = torch.nn.Linear(hidden_units, hidden_units)

    def forward(self, query, key, value, attn_mask=None, key_valid=None, seq_range=None, row_base=None):
        """row_base (with key_valid [B, T] and seq_range): query / key / value hold the
        jagged rows of the batch (jagged.py) as [1, rows, D]."""
        B, T, D = query.shape
        if row_base is not None:
            B, T = key_valid.shape
        elif key_valid is None:
            key_valid = key_valid_from_mask(attn_mask, B, T)
        N = query.shape[0] * query.shape[1]
        if query is key and key is value:
            w = torch.cat([self.q_linear.weight, self.k_linear.weight, self.v_linear.weight], 0)
            b = torch.cat([self.q_linear.bias, self.k_linear.bias, self.v_linear.bias], 0)
            qkv = _linear(query, w, b)
        else:
            qkv = torch.cat([self.q_linear(query), self.k_linear(key), self.v_linear(value)], -1)
        p = self.dropout_rate if self.training else 0.0
        seed = dropout_seed(qkv.device) if p > 0 else 0
        o = G.softmax_mha(qkv.reshape(N, 3 * D), key_valid, B, T, self.num_heads, self.head_dim, p, seed,
                          seq_range=seq_range, row_base=row_base)
        return _linear(o.view(query.shape), self.out_linear.weight, self.out_linear.bias), None


# The dropout seeds of one forward, drawn in ONE launch (seed_pool): dropout_seed
# hands out [1] views of it in call order.
_SEED_POOL = {'buf': None, 'next': 0}


@contextlib.contextmanager
def seed_pool(device, n):
    """Within the block, dropout_seed(device) takes its seeds from n values drawn in
    one torch.randint launch (then falls back to one launch per seed)."""
    if device.type != 'cuda' or n <= 0 or torch.compiler.is_compiling():
        yield
        return
    prev = dict(_SEED_POOL)
    _SEED_POOL['buf'] = torch.randint(0, 2 ** 62, (int(n),), device=device, dtype=torch.int64)
    _SEED_POOL['next'] = 0
    try:
        yield
    finally:
        _SEED_POOL.update(prev)


def dropout_seed(device):
    """The grk dropout seed of one launch: an int64 [1] drawn on the device from
    torch's generator and read by the kernels when they run.  No host round
    trip, and a step replayed from a HIP graph draws a fresh one every replay
    (torch registers its generator with the graph), exactly as the eager step
    would draw it.  Inside seed_pool: the pool's next value."""
    if device.type != 'cuda':
        return int(torch.randint(0, 2 ** 62, (1,)).item())
    buf, i = _SEED_POOL['buf'], _SEED_POOL['next']
    if buf is not None and buf.device == device and i < buf.numel() and not torch.compiler.is_compiling():
        _SEED_POOL['next'] = i + 1
        return buf[i:i + 1]
    return torch.randint(0, 2 ** 62, (1,), device=device, dtype=torch.int64)


def key_valid_from_mask(attn_mask, B, T):
    """Recover per-key validity from a log2feats-style mask (tril AND key_valid)
    and reject any other mask -- the kernels implement exactly that form."""
    if attn_mask is None:
        return None
    kv = attn_mask[:, -1, :]
    expect = torch.tril(torch.ones(T, T, dtype=torch.bool, device=attn_mask.device)).unsqueeze(0) & kv.unsqueeze(1)
    if not torch.equal(attn_mask.bool(), expect):
        raise NotImplementedError('grk attention supports the causal AND key-padding mask of log2feats only')
    return kv.to(torch.uint8).contiguous()


def _valid_bytes(token_type):
    """uint8 [B, T] = token_type != 0: the bool bytes viewed as uint8 (0 / 1, no cast
    kernel) in eager mode; a cast when traced (inductor cannot lower a bool -> uint8
    dtype view)."""
    kv = (token_type != 0).contiguous()
    return kv.to(torch.uint8) if torch.compiler.is_compiling() else kv.view(torch.uint8)


_UNIT_ROWS = {}


def _unit_row(w, device):
    """Cached fp32 [1, w] = [1, 0, ..., 0] on the device: the dnn operand's bias column and
    its padding, broadcast over the tokens by functional.write_extras."""
    key = (int(w), str(device))
    t = _UNIT_ROWS.get(key)
    if t is None:
        t = torch.zeros(1, w)
        t[0, 0] = 1.0
        t = _UNIT_ROWS[key] = t.to(device)
    return t


def _grk_gemm_ok(x):
    """Dense layers run on grk_gemm (hipBLASLt, stream-K eligible) under bf16
    autocast on the GPU -- the training regime of the reference and the
    bench; fp32 runs keep torch's fp32 GEMMs (the fp32 parity tests)."""
    return x.is_cuda and torch.is_autocast_enabled('cuda') and torch.get_autocast_dtype('cuda') == torch.bfloat16


def _linear(x, weight, bias=None):
    return G.linear(x, weight, bias) if _grk_gemm_ok(x) else F.linear(x, weight, bias)


class HSTUAttention(torch.nn.Module):
    """HSTU layer (north star; no reference -- oracle/hstu.py, oracle/model_ref.RefHSTU):

        u, v, q, k = split(SiLU(uvqk(x)))
        y = out_linear(dropout(LayerNorm(HSTU-attn(q, k, v, rab)) * u))

    The SiLU, LayerNorm, gating and dropout run inside the grk kernels
    (functional.hstu_core); dropout uses grk's counter-hash mask (seeded from
    torch's generator on the device), not torch's Philox stream.
    """

    def __init__(self, hidden_units, num_heads, dropout_rate, num_buckets, num_time_buckets=0, fp8=False):
        super().__init__()
        assert hidden_units % num_heads == 0, 'hidden_units must be divisible by num_heads'
        if fp8 and num_time_buckets:
            raise NotImplementedError('fp8 q/k/v (config C5) run without the time bias')
        self.fp8 = fp8  # config C5: q/k/v quantised to e4m3 after the SiLU (functional.hstu_core_fp8)
        self.hidden_units, self.num_heads = hidden_units, num_heads
        self.head_dim = hidden_units // num_heads
        self.dropout_rate = dropout_rate
        self.uvqk = torch.nn.Linear(hidden_units, 4 * hidden_units)
        self.rab = torch.nn.Parameter(torch.zeros(num_heads, num_buckets))
        # time bias rab_t[h, half-octave bucket of |t_q - t_k| + 1] (only with timestamps)
        self.rab_t = torch.nn.Parameter(torch.zeros(num_heads, num_time_buckets)) if num_time_buckets else None
        self.attn_norm = torch.nn.LayerNorm(hidden_units, eps=1e-8)
        self.out_linear = torch.nn.Linear(hidden_units, hidden_units)

    def forward(self, query, key=None, value=None, attn_mask=None, key_valid=None, seq_range=None, timestamps=None,
                row_base=None):
        """row_base (with key_valid [B, T] and seq_range): query holds the jagged rows
        of the batch (jagged.py) as [1, rows, D]; timestamps stay [B, T]."""
        B, T, D = query.shape
        if row_base is not None:
            B, T = key_valid.shape
        elif key_valid is None:
            key_valid = key_valid_from_mask(attn_mask, B, T)
        N = query.shape[0] * query.shape[1]
        rab_t = self.rab_t if timestamps is not None else None
        if rab_t is None:
            timestamps = None
        pre = _linear(query, self.uvqk.weight, self.uvqk.bias).reshape(N, 4 * D)
        p = self.dropout_rate if self.training else 0.0
        seed = dropout_seed(pre.device) if p > 0 else 0
        if self.fp8:
            if row_base is not None:
                raise NotImplementedError('fp8 q/k/v take the padded [B, T] layout (chunked kernels)')
            y = G.hstu_core_fp8(pre, self.rab, self.attn_norm.weight, self.attn_norm.bias, key_valid, B, T,
                                self.num_heads, self.head_dim, 1.0 / T, self.attn_norm.eps, dropout_p=p, seed=seed,
                                seq_range=seq_range)
            return _linear(y.view(query.shape), self.out_linear.weight, self.out_linear.bias), None
        y = G.hstu_core(pre, self.rab, self.attn_norm.weight, self.attn_norm.bias, key_valid, B, T,
                        self.num_heads, self.head_dim, 1.0 / T, self.attn_norm.eps, dropout_p=p, seed=seed,
                        seq_range=seq_range, timestamps=timestamps, rab_t=rab_t, row_base=row_base)
        return _linear(y.view(query.shape), self.out_linear.weight, self.out_linear.bias), None


class PointWiseFeedForward(torch.nn.Module):
    """Conv1d(k=1)-ReLU FFN (model/BaseLine/model.py:65-78)."""

    def __init__(self, hidden_units, dropout_rate):
        super().__init__()
        self.conv1 = torch.nn.Conv1d(hidden_units, hidden_units, kernel_size=1)
        self.dropout1 = torch.nn.Dropout(p=dropout_rate)
        self.relu = torch.nn.ReLU()
        self.conv2 = torch.nn.Conv1d(hidden_units, hidden_units, kernel_size=1)
        self.dropout2 = torch.nn.Dropout(p=dropout_rate)

    def forward(self, x):
        # k=1 convolutions are GEMMs on the [.., D] rows: F.linear, no transposes
        h = self.dropout1(_linear(x, self.conv1.weight.squeeze(-1), self.conv1.bias))
        return self.dropout2(_linear(self.relu(h), self.conv2.weight.squeeze(-1), self.conv2.bias))


class PackedSwiGLUFFN(torch.nn.Module):
    """SwiGLU FFN (model/BaseLineO1/model.py:103-164)."""

    def __init__(self, dim, hidden_dim=None, multiple_of=256, ffn_dim_multiplier=None, device=None, dtype=None,
                 dropout_rate=0.0):
        super().__init__()
        if hidden_dim is None:
            hidden_dim = 4 * dim
        else:
            hidden_dim = int(2 * hidden_dim / 3)
        if ffn_dim_multiplier is not None:
            hidden_dim = int(ffn_dim_multiplier * hidden_dim)
        hidden_dim = multiple_of * ((hidden_dim + multiple_of - 1) // multiple_of)
        kw = {'device': device, 'dtype': dtype}
        self.w13 = torch.nn.Linear(dim, 2 * hidden_dim, bias=False, **kw)
        self.w2 = torch.nn.Linear(hidden_dim, dim, bias=False, **kw)
        self.dropout = torch.nn.Dropout(p=dropout_rate) if dropout_rate > 0.0 else None

    def forward(self, x):
        a, b = torch.chunk(_linear(x, self.w13.weight), 2, dim=-1)
        y = _linear(F.silu(a) * b, self.w2.weight)
        return self.dropout(y) if self.dropout is not None else y


class BaselineModel(torch.nn.Module):
    """Two-tower sequence recommender (model/BaseLine/model.py:81-433)."""

    def __init__(self, user_num, item_num, feat_statistics, feat_types, args):
        super().__init__()
        self.user_num, self.item_num = user_num, item_num
        self.dev = getattr(args, 'device', 'cuda')
        self.norm_first = getattr(args, 'norm_first', False)
        self.maxlen = args.maxlen
        self.variant = getattr(args, 'variant', 'baseline')
        self.block = getattr(args, 'block', 'softmax')
        d = args.hidden_units
        self.hidden_units = d
        # feature tables with more rows than this are looked up directly into the
        # dnn operand instead of projected (see _projection): projecting costs
        # ~6 rows d^2 FLOP per forward + backward, a direct block ~6 tokens d^2
        self.proj_max_rows = int(getattr(args, 'proj_max_rows', 100_000))
        # fused path: the projected tables' row gradients of the seq-side and pair
        # lookups reduced in one call (functional.DenseMerge; the default since round 4)
        self.merge_proj = bool(getattr(args, 'merge_proj_backward', True))
        # fused path: the projections on the grouped MFMA GEMMs (functional.project_blocks)
        # instead of torch.bmm over equal-row-count stacks (_grouped_proj)
        self.grouped_proj = bool(getattr(args, 'grouped_proj', True))
        if getattr(args, 'shard_tables', False):
            # row-sharded item / user tables (BASELINE config 3, 50M rows): the full
            # tables are never built on any rank -- ShardedFusedAdamW creates each
            # rank's rows directly (table_init_rows), materialize_tables_ the whole
            # table when one process trains it
            self.item_emb = _placeholder_table(item_num + 1, d)
            self.user_emb = _placeholder_table(user_num + 1, d)
        else:
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
        self._init_feat_info(feat_statistics, feat_types)
        if self.USER_CONTINUAL_FEAT or self.ITEM_CONTINUAL_FEAT:
            raise NotImplementedError('continual features are not supported (empty in the TencentGR schema)')
        userdim = d * (len(self.USER_SPARSE_FEAT) + 1 + len(self.USER_ARRAY_FEAT))
        itemdim = d * (len(self.ITEM_SPARSE_FEAT) + 1 + len(self.ITEM_ARRAY_FEAT)) + d * len(self.ITEM_EMB_FEAT)
        self.userdnn = torch.nn.Linear(userdim, d)
        self.itemdnn = torch.nn.Linear(itemdim, d)
        self.last_layernorm = torch.nn.LayerNorm(d, eps=1e-8)
        nb = getattr(args, 'hstu_num_buckets', None) or args.maxlen + 1
        for _ in range(args.num_blocks):
            self.attention_layernorms.append(torch.nn.LayerNorm(d, eps=1e-8))
            if self.block == 'hstu':
                self.attention_layers.append(HSTUAttention(d, args.num_heads, args.dropout_rate, nb,
                                                           getattr(args, 'hstu_time_buckets', 0) or 0,
                                                           fp8=bool(getattr(args, 'hstu_fp8', False))))
                continue
            self.attention_layers.append(FlashMultiHeadAttention(d, args.num_heads, args.dropout_rate))
            self.forward_layernorms.append(torch.nn.LayerNorm(d, eps=1e-8))
            if self.variant == 'o1':
                self.forward_layers.append(PackedSwiGLUFFN(d, dropout_rate=args.dropout_rate))
            else:
                self.forward_layers.append(PointWiseFeedForward(d, args.dropout_rate))
        for group in (self.USER_SPARSE_FEAT, self.ITEM_SPARSE_FEAT, self.ITEM_ARRAY_FEAT, self.USER_ARRAY_FEAT):
            for k in group:
                self.sparse_emb[k] = torch.nn.Embedding(group[k] + 1, d, padding_idx=0)
        for k in self.ITEM_EMB_FEAT:
            self.emb_transform[k] = torch.nn.Linear(self.ITEM_EMB_FEAT[k], d)
        self._table_refs = None  # set by FusedAdamW (table groups)
        self._fwd_id = None      # projections of the small tables are shared within one forward
        self._proj_cache = {}
        self._proj_off_cache = {}
        self._remaps = None      # set by ShardedFusedAdamW.prepare (rows fetched from other ranks)
        self._flushers = []      # weak refs to optimizers holding deferred table rows (FusedAdamW)

    def flush_tables(self):
        """Bring every deferred table row to the optimizer's current step (FusedAdamW
        keeps rows outside recent batches a few steps behind): called
        before every read of whole tables outside training -- predict,
        save_item_emb, eval() -- and by state_dict (optimizer hook)."""
        alive = []
        for ref in self._flushers:
            fn = ref()
            if fn is not None:
                fn()
                alive.append(ref)
        self._flushers = alive

    def train(self, mode=True):
        if not mode:
            self.flush_tables()
        return super().train(mode)

    def _init_feat_info(self, feat_statistics, feat_types):
        self.USER_SPARSE_FEAT = {k: feat_statistics[k] for k in feat_types['user_sparse']}
        self.USER_CONTINUAL_FEAT = feat_types['user_continual']
        self.ITEM_SPARSE_FEAT = {k: feat_statistics[k] for k in feat_types['item_sparse']}
        self.ITEM_CONTINUAL_FEAT = feat_types['item_continual']
        self.USER_ARRAY_FEAT = {k: feat_statistics[k] for k in feat_types['user_array']}
        self.ITEM_ARRAY_FEAT = {k: feat_statistics[k] for k in feat_types['item_array']}
        self.ITEM_EMB_FEAT = {k: MM_SHAPE[k] for k in feat_types['item_emb']}

    # ------------------------------------------------------------ tables ----
    def table_modules(self):
        """name -> nn.Embedding for every table (state_dict prefix order)."""
        out = {'item_emb': self.item_emb, 'user_emb': self.user_emb, 'pos_emb': self.pos_emb}
        for k, m in self.sparse_emb.items():
            out[f'sparse_emb.{k}'] = m
        return out

    def _ref(self, name):
        if self._table_refs is not None:
            return self._table_refs[name]
        return G.TableRef(self.table_modules()[name].weight)

    def _device(self):
        return self.item_emb.weight.device

    def _feats(self, feature_array, fids, B, T):
        """Device tensors for the requested features (tensorising dict lists on the host)."""
        dev = self._device()
        if isinstance(feature_array, dict):
            out = feature_array
        else:
            arr = set(self.ITEM_ARRAY_FEAT) | set(self.USER_ARRAY_FEAT)
            out = tensorize(list(feature_array), fids, arr, set(self.ITEM_EMB_FEAT))
        res = {}
        for k in fids:
            t = out[k]
            t = t.to(dev, non_blocking=True) if t.device != dev else t
            res[k] = t if (t.is_floating_point() or t.dtype == torch.int64) else t.long()
        return res

    # -------------------------------------------------- model/BaseLine/model.py:226-310
    # feat2emb computes relu(itemdnn(cat(item_emb, sparse/array feature embs,
    # emb_transform(mm)))) (+ relu(userdnn(cat(user_emb, user feature embs)))).
    # Restated exactly (up to fp32 summation order) as
    #     [item_emb rows | mm | 1] @ [W_0 | W_mm Wt | b']^T  +  sum_f P_f[idx_f]
    # with P_f = E_f @ W_f^T the feature table projected through its itemdnn
    # block: the small feature tables are projected once per forward (~25
    # GFLOP at d=512) and their lookups become ONE bag-sum gather of projected
    # rows, so the dnn GEMMs run with K = d + 40 instead of 16d / 9d.  The
    # projections are plain torch ops, so autograd produces dE_f and dW_f.
    # The projection costs rows x d^2 however few rows a batch touches, so tables
    # with more than proj_max_rows rows (real vocabularies) are instead gathered
    # as their own d-column blocks of the GEMM operand (_direct_feats), right
    # after the item / user rows, with their W_f blocks in the composed weight.
    def _dnn_feats(self, which):
        if which == 'item':
            return list(self.ITEM_SPARSE_FEAT) + list(self.ITEM_ARRAY_FEAT)
        return list(self.USER_SPARSE_FEAT) + list(self.USER_ARRAY_FEAT)

    def _direct_feats(self, which):
        """[(feature, dnn block index)] of the tables looked up unprojected."""
        return [(k, j + 1) for j, k in enumerate(self._dnn_feats(which))
                if self.sparse_emb[k].num_embeddings > self.proj_max_rows]

    def _projection(self, which):
        """(P [rows, d], {feature: P row of its table's row 0}) for the item or user dnn.

        P[0] (the first table's padding row, zero) is the shared padding row:
        every feature's index 0 is mapped there (_proj_index), so padding
        occurrences are skipped by the gradient reduction (padding_idx 0) as
        nn.Embedding(padding_idx=0) does."""
        key = (which, self._fwd_id)
        if self._fwd_id is not None and key in self._proj_cache:
            return self._proj_cache[key]
        d = self.hidden_units
        pieces = self._weight_pieces(which)
        if len(pieces) > 2:                     # grouped MFMA projection (_grouped_proj)
            res = pieces[2]
            if self._fwd_id is not None:
                self._proj_cache[key] = res
            return res
        stacks = pieces[1]
        parts, offs, row = [], {}, 0
        for rows, group, refs in self._proj_groups(which):
            grp = next(iter(refs.values())).group
            if grp is not None and all(r.group is grp for r in refs.values()):
                E = G.group_stack(grp, [refs[k].row_offset for k, _ in group], rows)
            else:
                E = torch.stack([refs[k].weight for k, _ in group])
            # the group's itemdnn / userdnn blocks [len(group), d_out, d_in] in E's dtype
            # (functional.weight_blocks: one gradient buffer for the whole dnn weight)
            Wb = stacks[tuple(j for _, j in group)]
            if d >= 1024 and _grk_gemm_ok(E):
                # torch's batched bf16 GEMM faults at this width (d = 1024, C5): hipBLASLt
                # returned HIPBLAS_STATUS_INTERNAL_ERROR for [3 x 10001 x 1024] x [1024 x 1024]
                # and its rocBLAS fallback made an illegal access.  One
                # grk_gemm per block instead (plans validated at first use).
                parts.append(torch.cat([G.linear(E[i], Wb[i]).to(E.dtype) for i in range(len(group))]))
            else:
                parts.append(torch.bmm(E, Wb.transpose(1, 2)).to(E.dtype).reshape(-1, d))
            for k, _ in group:
                offs[k] = row
                row += rows
        res = (torch.cat(parts) if len(parts) > 1 else parts[0]), offs
        if self._fwd_id is not None:
            self._proj_cache[key] = res
        return res

    def _proj_groups(self, which):
        """[(rows, [(feature, dnn block)], {feature: TableRef})] of the projected tables,
        grouped by row count; a group's tables in group-buffer order when they share
        a table group (so group_stack can view them without a copy)."""
        direct = {k for k, _ in self._direct_feats(which)}
        by_rows = {}
        for j, k in enumerate(self._dnn_feats(which)):  # block 0 is item_emb / user_emb
            if k not in direct:
                by_rows.setdefault(self.sparse_emb[k].num_embeddings, []).append((k, j + 1))
        out = []
        for rows, group in by_rows.items():
            refs = {k: self._ref(f'sparse_emb.{k}') for k, _ in group}
            grp = next(iter(refs.values())).group
            if grp is not None and all(r.group is grp for r in refs.values()):
                group = sorted(group, key=lambda kj: refs[kj[0]].row_offset)
            out.append((rows, group, refs))
        return out

    def _grouped_proj(self, which):
        """(tables [(block, group row offset, rows, P row offset)], group, {feature: P
        offset}, P rows) when the projection runs on the grouped MFMA GEMMs
        (functional.project_blocks: every projected table in one bf16 table group, on
        the GPU, d a multiple of 32, at most 32 tables), else None."""
        if torch.compiler.is_compiling():
            return None
        d = self.hidden_units
        grp, entries = None, []
        for rows, group, refs in self._proj_groups(which):
            for k, j in group:
                r = refs[k]
                if r.group is None or (grp is not None and r.group is not grp):
                    return None
                grp = r.group
                entries.append((k, j, r.row_offset, rows))
        if (grp is None or not grp.flat.is_cuda or grp.flat.dtype != torch.bfloat16 or d % 32
                or len(entries) > 32):
            return None
        dnn = self.itemdnn if which == 'item' else self.userdnn
        if dnn.weight.dtype not in (torch.float32, torch.bfloat16) or dnn.weight.shape[0] % 8:
            return None
        entries.sort(key=lambda e: e[2])        # P in group-buffer order; the first table's row 0 is P[0]
        poffs, p_rows = G.proj_layout([e[3] for e in entries])
        tables = [(j, off, rows, po) for (_, j, off, rows), po in zip(entries, poffs)]
        return tables, grp, {k: po for (k, _, _, _), po in zip(entries, poffs)}, p_rows

    def _weight_pieces(self, which):
        """The itemdnn / userdnn weight's column blocks this forward reads, from ONE
        functional.weight_blocks call per forward and side: ({block: fp32 view} for
        W_0, the direct-feature and the mm blocks, {block tuple: [G, d, d] stack in the
        tables' dtype} for the projected groups) -- or, on the grouped MFMA projection
        (functional.project_blocks), ({block: view}, {}, (P, {feature: P offset}))."""
        key = ('wb', which, self._fwd_id)
        if self._fwd_id is not None and key in self._proj_cache:
            return self._proj_cache[key]
        d = self.hidden_units
        dnn = self.itemdnn if which == 'item' else self.userdnn
        singles = [0] + [j for _, j in self._direct_feats(which)]
        if which == 'item':
            base = 1 + len(self.ITEM_SPARSE_FEAT) + len(self.ITEM_ARRAY_FEAT)
            singles += [base + j for j in range(len(self.ITEM_EMB_FEAT))]
        gp = self._grouped_proj(which) if self.grouped_proj else None
        if gp is not None:
            tables, grp, offs, p_rows = gp
            outs = G.project_blocks(dnn.weight, d, singles, tables, grp, p_rows)
            res = ({j: o for j, o in zip(singles, outs)}, {}, (outs[-1], offs))
            if self._fwd_id is not None:
                self._proj_cache[key] = res
            return res
        stacks = [(tuple(j for _, j in group), next(iter(refs.values())).weight.dtype)
                  for _, group, refs in self._proj_groups(which)]
        if torch.compiler.is_compiling():      # traced: the slice form (weight_blocks is a graph break)
            outs = G.weight_blocks_sliced(dnn.weight, d, singles, stacks)
        else:
            outs = G.weight_blocks(dnn.weight, d, singles, stacks)
        res = ({j: o for j, o in zip(singles, outs)},
               {js: o for (js, _), o in zip(stacks, outs[len(singles):])})
        if self._fwd_id is not None:
            self._proj_cache[key] = res
        return res

    def _proj_merge(self, P):
        """The forward's DenseMerge of the projected tables (args.merge_proj_backward, fused
        lookups only: table groups present), with P registered; None otherwise."""
        if not self.merge_proj or self._fwd_id is None or self._table_refs is None or not P.requires_grad:
            return None
        m = self._proj_cache.get(('merge', self._fwd_id))
        if m is None:
            m = self._proj_cache[('merge', self._fwd_id)] = G.DenseMerge()
        m.add(P)
        return m

    def _proj_index(self, feats, names, offs, N):
        """[N, sum of bags] rows of P: feature value v of table k -> offs[k] + v, 0 -> 0
        (grk_proj_index: one launch on the GPU)."""
        blocks = [(feats[k].reshape(N, -1), offs[k]) for k in names]
        if blocks[0][0].is_cuda and not torch.compiler.is_compiling() \
                and len({b.dtype for b, _ in blocks}) == 1 and blocks[0][0].dtype in (torch.int32, torch.int64):
            return K.proj_index(blocks, N)
        x = torch.cat([feats[k].reshape(N, -1) for k in names], 1)
        key = tuple((offs[k], feats[k].reshape(N, -1).shape[1]) for k in names)
        off = self._proj_off_cache.get(key)
        if off is None:
            off = torch.tensor([o for o, w in key for _ in range(w)], dtype=x.dtype).to(x.device)
            self._proj_off_cache[key] = off
        return torch.where(x > 0, x + off, 0)

    def _dnn_weight(self, which, width, dtype=None):
        """[d, width] = [W_0 | W_f (direct features) | W_mm Wt | b' | 0] matching the
        operand [rows | direct feature rows | mm | 1 | pad], in `dtype` (None: fp32)."""
        d = self.hidden_units
        dnn = self.itemdnn if which == 'item' else self.userdnn
        blk = self._weight_pieces(which)[0]
        if dnn.bias.is_cuda and dtype is not None:
            # one autograd node (functional.dnn_weight): the eager composition below
            # costs ~25 small kernels per forward + backward
            blocks = [blk[0]] + [blk[j] for _, j in self._direct_feats(which)]
            mms = []
            if which == 'item':
                base = 1 + len(self.ITEM_SPARSE_FEAT) + len(self.ITEM_ARRAY_FEAT)
                for j, k in enumerate(self.ITEM_EMB_FEAT):
                    et = self.emb_transform[k]
                    mms.append((blk[base + j], et.weight, et.bias))
            return G.dnn_weight(blocks, dnn.bias, mms, width, dtype)
        cols, bias = [blk[0]], dnn.bias[:, None]
        cols += [blk[j] for _, j in self._direct_feats(which)]
        if which == 'item':
            base = 1 + len(self.ITEM_SPARSE_FEAT) + len(self.ITEM_ARRAY_FEAT)
            for j, k in enumerate(self.ITEM_EMB_FEAT):
                Wk = blk[base + j]
                et = self.emb_transform[k]
                # one matrix-matrix product for [Wk Wt | Wk bt] (a matrix-vector product
                # for Wk bt costs milliseconds of host time in its backward on ROCm)
                Mk = Wk @ torch.cat([et.weight, et.bias[:, None]], 1)
                cols.append(Mk[:, :-1])
                bias = bias + Mk[:, -1:]
        cols.append(bias)
        Wc = torch.cat(cols, 1)
        return F.pad(Wc, (0, width - Wc.shape[1]))

    def _embed(self, seq, feature_array, mask=None, include_user=False, with_pos=False, role='seq', pos_idx=None,
               combine=None):
        """pos_idx (jagged rows): the position-embedding index of each row (t + 1 where
        the token is not padding) instead of the positional mode, which derives it from
        the row's place in a [B, T] batch.  combine = (scale, dropout_p): return the
        first block's input dropout((item + user) * scale + pos) itself (and None for
        the position rows) where the grk path runs."""
        dev = self._device()
        seq = seq.to(dev, non_blocking=True).long()
        B, T = seq.shape
        N = B * T
        d = self.hidden_units
        item_f = list(self.ITEM_SPARSE_FEAT) + list(self.ITEM_ARRAY_FEAT)
        user_f = (list(self.USER_SPARSE_FEAT) + list(self.USER_ARRAY_FEAT)) if include_user else []
        feats = self._feats(feature_array, item_f + user_f + list(self.ITEM_EMB_FEAT), B, T)
        tt = mask.to(dev, non_blocking=True) if mask is not None else None
        specs, extras, splits = [], [], []
        col = 0

        def operand(ref, mode, dense, which):
            """gather block [rows | direct feature rows | dense | 1 | pad] feeding one
            dnn GEMM; returns its split.  The dense features are copied into the gather
            buffer as they are, the constant [1 | 0 ...] columns as one broadcast row
            (no ones / cat / pad tensors per step)."""
            nonlocal col
            start = col
            specs.append(G.LookupSpec(ref, seq, col, mode))
            col += d
            for k, _ in self._direct_feats(which):
                idx = feats[k].reshape(N, -1)
                bag = idx.shape[1]
                specs.append(G.LookupSpec(self._ref(f'sparse_emb.{k}'), idx if bag > 1 else idx.reshape(N), col,
                                          L.IDX_PLAIN, bag))
                col += d
            for x in dense:
                extras.append((col, x))
                col += x.shape[1]
            w = 1 + (-(sum(x.shape[1] for x in dense) + 1)) % 8     # the 1 column + padding to a multiple of 8
            extras.append((col, _unit_row(w, dev)))
            col += w
            splits.append((start, col))
            return col - start

        def projected(which, names):
            nonlocal col
            P, offs = self._projection(which)
            idx = self._proj_index(feats, names, offs, N)
            # P = E W is an intermediate: its row sums may use the chunked order (the
            # reference accumulates dE = sum dY W, in no order P's sums could match)
            # P's row 0 is the zero padding row every feature's padding maps to (grk_proj_index):
            # the gather skips those slots (all user-feature slots of an item token)
            specs.append(G.LookupSpec(G.TableRef(P, chunked=True, merge=self._proj_merge(P), zero_row0=True), idx,
                                      col, L.IDX_PLAIN, idx.shape[1]))
            splits.append((col, col + d))
            col += d

        mm = [feats[k].reshape(N, -1).float() for k in self.ITEM_EMB_FEAT]
        direct_i = {k for k, _ in self._direct_feats('item')}
        direct_u = {k for k, _ in self._direct_feats('user')} if include_user else set()
        item_p = [k for k in item_f if k not in direct_i]
        user_p = [k for k in user_f if k not in direct_u]
        wi = operand(self._ref('item_emb'), L.IDX_ITEM_MASK if include_user else L.IDX_PLAIN, mm, 'item')
        if item_p:
            projected('item', item_p)
        if include_user:
            wu = operand(self._ref('user_emb'), L.IDX_USER_MASK, [], 'user')
            if user_p:
                projected('user', user_p)
        if with_pos and pos_idx is not None:
            specs.append(G.LookupSpec(self._ref('pos_emb'), pos_idx.to(dev).reshape(N), col, L.IDX_PLAIN))
            splits.append((col, col + d))
            col += d
        elif with_pos:
            specs.append(G.LookupSpec(self._ref('pos_emb'), seq, col, L.IDX_POSITION))
            splits.append((col, col + d))
            col += d
        if self._remaps is not None or self._table_refs is not None:
            specs = self._remap_specs(specs, role)
        blocks = list(G.feature_lookup(specs, N, col, tt, T, extras, splits))

        def dnn(which, width, has_proj, relu=True):
            a = blocks.pop(0)
            p = blocks.pop(0) if has_proj else None
            # one composed (and cast) dnn weight per forward: the seq-side and the
            # pos/neg feat2emb share it, so its autograd graph runs once
            key = ('w', which, width, a.dtype, self._fwd_id)
            w = self._proj_cache.get(key) if self._fwd_id is not None else None
            if w is None:
                w = self._dnn_weight(which, width, a.dtype) if _grk_gemm_ok(a) else \
                    self._dnn_weight(which, width).to(a.dtype)
                if self._fwd_id is not None:
                    self._proj_cache[key] = w
            if _grk_gemm_ok(a):
                # ReLU in the GEMM's store; the projected rows' sum p (a column block of the
                # gather buffer, read by nothing else) accumulated into where it lies
                return G.linear(a, w, addend=p, relu=relu, in_place=True)
            y = torch.addmm(p, a, w.t()) if p is not None else a @ w.t()
            return torch.relu(y) if relu else y

        if combine is not None and include_user and with_pos and _grk_gemm_ok(blocks[0]):
            # log2feats' first-block input in one pass: the dnn ReLUs, the sum, the
            # sqrt(d) scale, the position rows and the dropout (grk_emb_combine)
            scale, p = combine
            xi = dnn('item', wi, bool(item_p), relu=False)
            xu = dnn('user', wu, bool(user_p), relu=False)
            seed = dropout_seed(dev) if p > 0 else 0
            return G.emb_combine(xi, xu, blocks.pop(0), scale, True, p, seed).view(B, T, d), None
        x = dnn('item', wi, bool(item_p))
        if include_user:
            x = x + dnn('user', wu, bool(user_p))
        pos_rows = blocks.pop(0) if with_pos else None
        return x.view(B, T, d), pos_rows

    def _remap_specs(self, specs, role):
        """Row-sharded tables: read the rows prepare() fetched for this step.
        Remaps are keyed by (table, role, lookup mode) -- role 'seq' (log2feats),
        'pos' / 'neg' (feat2emb) or 'pair' (the stacked pos|neg lookup) -- never by
        tensor address: the batch's int32 ids are widened to int64 separately by
        prepare() and by the forward, so their copies do not share storage."""
        out = []
        for s in specs:
            name = getattr(s.ref, 'name', None)
            if name is None:
                out.append(s)
                continue
            hit = (self._remaps or {}).get((name, role, s.mode))
            if hit is not None and hit[1].numel() != s.idx.numel():
                raise RuntimeError(f'{name}: the batch prepared ({hit[1].numel()} ids) is not the one in forward '
                                   f'({s.idx.numel()} ids)')
            if hit is None:
                raise RuntimeError(f'{name} is row-sharded: call the optimizer\'s prepare(batch) before forward')
            ref, inv = hit
            out.append(G.LookupSpec(ref, inv, s.out_col, L.IDX_PLAIN, 1))
        return out

    def feat2emb(self, seq, feature_array, mask=None, include_user=False):
        return self._embed(seq, feature_array, mask, include_user)[0]

    def feat2emb_pair(self, pos_seqs, pos_feature, neg_seqs, neg_feature):
        """``(feat2emb(pos), feat2emb(neg))`` computed as ONE feat2emb over the
        two batches stacked ([2B, T]): one fused gather and one itemdnn GEMM
        with twice the rows.  Every output row depends on its own token only,
        so this equals the reference's two calls (model/BaseLine/model.py:376-377)."""
        dev = self._device()
        pos = pos_seqs.to(dev, non_blocking=True).long()
        neg = neg_seqs.to(dev, non_blocking=True).long()
        B, T = pos.shape
        fids = list(self.ITEM_SPARSE_FEAT) + list(self.ITEM_ARRAY_FEAT) + list(self.ITEM_EMB_FEAT)
        fp = self._feats(pos_feature, fids, B, T)
        fn = self._feats(neg_feature, fids, B, T)
        feats = _stack_pairs(fp, fn, fids)
        seq2 = _cat0(pos, neg)
        if self._remaps is not None:  # row-sharded tables: the stacked ids read the rows fetched for pos and neg
            for name in ('item_emb',):
                a = self._remaps.get((name, 'pos', L.IDX_PLAIN))
                b = self._remaps.get((name, 'neg', L.IDX_PLAIN))
                if a is not None and b is not None and a[0] is b[0]:
                    self._remaps[(name, 'pair', L.IDX_PLAIN)] = (a[0], torch.cat([a[1], b[1]], 0))
        x = self._embed(seq2, feats, role='pair')[0]
        # split, not x[:B] / x[B:]: its backward is one cat of the two gradients, where two
        # slices' backwards zero-fill a full-size gradient each and add them (same values);
        # on the GPU not even the cat: the fused loss writes the halves into one buffer
        if x.is_cuda and not torch.compiler.is_compiling():
            return G.split_pair(x, B)
        pe, ne = x.split(B, 0)
        return pe, ne

    # -------------------------------------------------- model/BaseLine/model.py:312-350
    def log2feats(self, log_seqs, mask, seq_feature, timestamps=None, jagged=None, pos_idx=None):
        """timestamps (int [B, T] event times, HSTU blocks with hstu_time_buckets > 0
        only): the time bias of every HSTU layer; None = positions only.
        jagged (jagged.Jagged) + pos_idx: log_seqs / mask / seq_feature / pos_idx hold
        the batch's jagged rows as [1, rows] (jagged.compact); the result is [1, rows, D]."""
        dev = self._device()
        B, T = log_seqs.shape
        scale = self.item_emb.embedding_dim ** 0.5
        p = self.emb_dropout.p if self.training else 0.0
        seqs, pos_rows = self._embed(log_seqs, seq_feature, mask=mask, include_user=True, with_pos=True,
                                     pos_idx=pos_idx if jagged is not None else None, combine=(scale, p))
        if pos_rows is not None:
            seqs = seqs * scale + pos_rows.view(B, T, -1)
            seqs = self.emb_dropout(seqs)
        if jagged is not None:
            kw = dict(key_valid=jagged.key_valid, seq_range=jagged.seq_range, row_base=jagged.row_base)
        else:
            key_valid = _valid_bytes(mask.to(dev, non_blocking=True))
            kw = dict(key_valid=key_valid, seq_range=torch.ops.grk.seq_ranges(key_valid))  # one launch serves every layer
        if timestamps is not None and self.block == 'hstu':
            kw['timestamps'] = timestamps.to(dev, torch.int64, non_blocking=True).contiguous()
        if self.block == 'hstu' and _grk_gemm_ok(seqs) and self.hidden_units % 8 == 0:
            # bf16 residual stream: each residual add is fused into the next LayerNorm
            # (grk_add_norm), the last one into last_layernorm (fp32 output, as autocast's)
            y = None
            for i in range(len(self.attention_layers)):
                ln = self.attention_layernorms[i]
                if y is None:
                    x = G.add_norm(seqs, None, ln.weight, ln.bias, ln.eps)
                else:
                    seqs, x = G.add_norm(seqs, y, ln.weight, ln.bias, ln.eps)
                y, _ = self.attention_layers[i](x, **kw)
            ln = self.last_layernorm
            if y is None:
                return G.add_norm(seqs, None, ln.weight, ln.bias, ln.eps, x_dtype=torch.float32)
            return G.add_norm(seqs, y, ln.weight, ln.bias, ln.eps, x_dtype=torch.float32)[1]
        for i in range(len(self.attention_layers)):
            if self.block == 'hstu':
                y, _ = self.attention_layers[i](self.attention_layernorms[i](seqs), **kw)
                seqs = seqs + y
            elif self.norm_first:
                x = self.attention_layernorms[i](seqs)
                seqs = seqs + self.attention_layers[i](x, x, x, **kw)[0]
                seqs = seqs + self.forward_layers[i](self.forward_layernorms[i](seqs))
            else:
                y, _ = self.attention_layers[i](seqs, seqs, seqs, **kw)
                seqs = self.attention_layernorms[i](seqs + y)
                seqs = self.forward_layernorms[i](seqs + self.forward_layers[i](seqs))
        return self.last_layernorm(seqs)

    # -------------------------------------------------- model/BaseLine/model.py:352-384
    def forward(self, user_item, pos_seqs, neg_seqs, mask, next_mask, next_action_type, seq_feature, pos_feature,
                neg_feature, timestamps=None):
        with self._shared_projections():
            log_feats = self.log2feats(user_item, mask, seq_feature, timestamps)
            pos_embs, neg_embs = self.feat2emb_pair(pos_seqs, pos_feature, neg_seqs, neg_feature)
        return G.pair_logits(log_feats, pos_embs, neg_embs, next_mask.to(self._device(), non_blocking=True))

    def encode(self, user_item, pos_seqs, neg_seqs, mask, seq_feature, pos_feature, neg_feature, timestamps=None,
               jagged=None, pos_idx=None):
        """(log_feats, pos_embs, neg_embs) -- the operands of the loss.  jagged / pos_idx:
        the batch fields hold its jagged rows (jagged.compact), so do the three outputs."""
        with self._shared_projections():
            return (self.log2feats(user_item, mask, seq_feature, timestamps, jagged=jagged, pos_idx=pos_idx),
                    *self.feat2emb_pair(pos_seqs, pos_feature, neg_seqs, neg_feature))

    @contextlib.contextmanager
    def _shared_projections(self):
        """One set of projected feature tables for every feat2emb of this forward, and
        its dropout seeds drawn in one launch (training only: the first-block input and
        one per attention layer)."""
        self._fwd_id = object()
        self._proj_cache = {}
        n = len(self.attention_layers) + 1 if self.training and self.emb_dropout.p > 0 else 0
        try:
            with seed_pool(self._device(), n):
                yield
        finally:
            self._fwd_id = None
            self._proj_cache = {}

    def _inference_autocast(self):
        """bf16 tables (fused mode, optim.FusedAdamW) run inference under the bf16
        autocast they train in; fp32 tables (drop-in mode) as the reference, fp32."""
        ref = self._ref('item_emb').weight if self._table_refs is not None else self.item_emb.weight
        if ref.dtype == torch.bfloat16 and ref.is_cuda and not torch.is_autocast_enabled('cuda'):
            return torch.autocast('cuda', dtype=torch.bfloat16)
        return contextlib.nullcontext()

    def predict(self, log_seqs, seq_feature, mask, timestamps=None):
        self.flush_tables()
        with self._inference_autocast():
            return self.log2feats(log_seqs, mask, seq_feature, timestamps)[:, -1, :]

    def save_item_emb(self, item_ids, retrieval_ids, feat_dict, save_path, batch_size=1024):
        """Candidate item embeddings -> embedding.fbin / id.u64bin (model/BaseLine/model.py:402-433)."""
        self.flush_tables()
        embs = []
        for s in range(0, len(item_ids), batch_size):
            e = min(s + batch_size, len(item_ids))
            seq = torch.tensor(item_ids[s:e], device=self._device()).unsqueeze(0)
            feats = [np.array([feat_dict[i] for i in range(s, e)], dtype=object)]
            with self._inference_autocast():
                emb = self.feat2emb(seq, feats, include_user=False)
            embs.append(emb.squeeze(0).detach().float().cpu().numpy())
        save_emb(np.concatenate(embs, 0), Path(save_path, 'embedding.fbin'))
        save_emb(np.array(retrieval_ids, dtype=np.uint64).reshape(-1, 1), Path(save_path, 'id.u64bin'))


def _adjacent(a, b):
    """torch.cat([a, b], 0) as a view when b starts where a ends in one storage
    (jagged.compact lays pos / neg out that way), else None (always when traced)."""
    if torch.compiler.is_compiling():
        return None
    return G._adjacent_rows(a, b)


def _cat0(a, b):
    v = _adjacent(a, b)
    return v if v is not None else torch.cat([a, b], 0)


def _stack_pairs(fa, fb, fids):
    """{k: _stack_padded(fa[k], fb[k])} for every feature with (at most) one
    zero-fill and one multi-tensor copy kernel per dtype instead of a cat (and
    pads) per feature; no copy at all for pairs already adjacent in memory."""
    out, groups, pad = {}, {}, []
    for k in fids:
        a, b = fa[k], fb[k]
        v = _adjacent(a, b)
        if v is not None:
            out[k] = v
            continue
        if a.dim() != b.dim() or a.shape[0] != b.shape[0] or a.shape[1:2] != b.shape[1:2] or a.dtype != b.dtype \
                or (a.dim() == 3 and a.is_floating_point() and a.shape[2] != b.shape[2]) or a.dim() > 3:
            out[k] = _stack_padded(a, b)
            continue
        w = max(a.shape[2], b.shape[2]) if a.dim() == 3 else None
        shp = (a.shape[0] + b.shape[0],) + a.shape[1:2] + ((w,) if w is not None else ())
        o = torch.empty(shp, dtype=a.dtype, device=a.device)
        if w is not None and (a.shape[2] != w or b.shape[2] != w):
            pad.append(o)
        n = a.shape[0]
        for part, t in ((o[:n], a), (o[n:], b)):
            d = part[..., :t.shape[2]] if w is not None and t.shape[2] != w else part
            # one list per (dtype, contiguous destination): the multi-tensor fast path
            g = groups.setdefault((t.dtype, d.is_contiguous()), ([], []))
            g[0].append(d)
            g[1].append(t if t.is_contiguous() else t.contiguous())
        out[k] = o
    if pad:
        torch._foreach_zero_(pad)
    for dst, src in groups.values():
        torch._foreach_copy_(dst, src)
    return out


def _stack_padded(a, b):
    """Stack two feature tensors along the batch dim; array features (bag dim 2)
    are zero-padded to the wider bag (index 0 = the zero padding row)."""
    if a.dim() == 3 and not a.is_floating_point() and a.shape[2] != b.shape[2]:
        w = max(a.shape[2], b.shape[2])
        a = F.pad(a, (0, w - a.shape[2]))
        b = F.pad(b, (0, w - b.shape[2]))
    return torch.cat([a, b], 0)


def _placeholder_table(rows, dim):
    """nn.Embedding(rows, dim, padding_idx=0) with no rows allocated (weight [0, dim])."""
    emb = torch.nn.Embedding(1, dim, padding_idx=0)
    emb.num_embeddings = rows
    emb.weight = torch.nn.Parameter(torch.empty(0, dim), requires_grad=False)
    return emb


def table_init_rows(rows, dim, seed, std, dtype=torch.float32):
    """Rows `rows` (int64, any device) of a [R, dim] table initialised
    N(0, std^2) from a counter-based hash of (seed, row, column): the value of
    a row does not depend on which rank builds it or which other rows are
    built with it, so row shards (rows rank::world) built separately equal the
    slices of the whole table.  Row 0 (padding) is zero.  The reference draws
    the same distribution with torch's generator (xavier_normal_,
    model/BaseLine/main.py:95-111); a sharded run cannot reproduce that stream."""
    M32 = 0xFFFFFFFF

    def mix(x):  # lowbias32 on int64 lanes holding 32-bit values
        x = (x ^ (x >> 16)) & M32
        x = (x * 0x7FEB352D) & M32
        x = (x ^ (x >> 15)) & M32
        x = (x * 0x846CA68B) & M32
        return (x ^ (x >> 16)) & M32

    rows = rows.to(torch.int64).reshape(-1, 1)
    col = torch.arange(dim, device=rows.device, dtype=torch.int64).reshape(1, -1)
    base = mix(mix(rows & M32) ^ mix((rows >> 32) ^ (int(seed) & M32)))
    u1 = (mix(base ^ mix(2 * col)).double() + 1.0) / 4294967296.0           # (0, 1]
    u2 = mix(base ^ mix(2 * col + 1)).double() / 4294967296.0              # [0, 1)
    z = torch.sqrt(-2.0 * torch.log(u1)) * torch.cos(6.283185307179586 * u2) * std
    z = torch.where(rows == 0, torch.zeros_like(z), z)
    return z.to(dtype)


def table_init_std(num_rows, dim):
    """xavier_normal_'s std for a [num_rows, dim] table (model/BaseLine/main.py:95-111)."""
    return (2.0 / float(num_rows + dim)) ** 0.5


def materialize_tables_(model, seed=0, device=None, dtype=torch.float32, chunk=1 << 18):
    """Replace placeholder item / user tables (args.shard_tables) by whole tables
    holding table_init_rows -- what every shard of a row-sharded run holds, in one
    process (the unsharded twin of a sharded run)."""
    dev = torch.device(device) if device is not None else model.pos_emb.weight.device
    for name in ('item_emb', 'user_emb'):
        emb = getattr(model, name)
        if emb.weight.shape[0] != 0:
            continue
        R, D = emb.num_embeddings, emb.embedding_dim
        w = torch.empty(R, D, dtype=dtype, device=dev)
        for s in range(0, R, chunk):
            w[s:s + chunk] = table_init_rows(torch.arange(s, min(R, s + chunk), device=dev), D,
                                             seed + (1 if name == 'user_emb' else 0), table_init_std(R, D), dtype)
        emb.weight = torch.nn.Parameter(w)
    return model


def init_reference_(model, seed=None, live_norms=False):
    """Parameter init of the training script (model/BaseLine/main.py:95-111):
    xavier_normal_ for dim >= 2, zeros for 1-D, padding rows of every table zeroed.

    The reference's rule also zeroes every LayerNorm gamma, which makes the
    first steps' logits exactly 0; ``live_norms=True`` keeps gamma = 1."""
    g = None
    if seed is not None:
        g = torch.Generator(device=model.item_emb.weight.device).manual_seed(seed)
    with torch.no_grad():
        for _, p in model.named_parameters():
            if p.dim() >= 2:
                fan_in, fan_out = torch.nn.init._calculate_fan_in_and_fan_out(p)
                std = (2.0 / float(fan_in + fan_out)) ** 0.5
                p.normal_(0.0, std, generator=g)
            elif p.dim() == 1:
                p.zero_()
        for t in model.table_modules().values():
            if t.weight.shape[0]:      # placeholder (row-sharded) tables hold no rows here
                t.weight[0].zero_()
        if live_norms:
            for mm in model.modules():
                if isinstance(mm, torch.nn.LayerNorm):
                    mm.weight.fill_(1.0)
    return model
