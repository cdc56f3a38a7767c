"""Fused optimizer for the training step: table groups + dense AdamW.

The reference steps ``torch.optim.AdamW(model.parameters(), lr,
betas=(0.9, 0.98), weight_decay)`` over every parameter, embedding tables
included, with dense table gradients (``model/BaseLine/main.py:131,189``;
``model/BaseLineO1/main.py:174,249``).  Here:

* the embedding tables are packed into a few **table groups** (one flat
  ``[rows, D]`` buffer each; every ``nn.Embedding.weight`` becomes a view, so
  state_dict keys and values are unchanged).  Lookups push row-sparse
  gradient sources into their group; ``step()`` reduces each group with ONE
  deterministic ``grk_embedding_backward`` and updates it with ONE
  ``grk_table_adamw``.  ``table_mode="dense"`` moves every row exactly like
  the reference (rows without gradient still decay and update their
  moments); ``"lazy"`` touches only rows that received a gradient (a
  documented deviation);
* the remaining dense parameters use torch's fused AdamW.

Table storage dtype defaults to bf16 (BASELINE config 2); moments are fp32.
"""
from __future__ import annotations

import torch

from . import functional as G
from . import kernels as K


class TableGroup:
    """Several tables in one flat buffer, with their AdamW state."""

    def __init__(self, name, tables, dtype, device):
        self.name = name
        # equal-sized tables adjacent (stable in the given order): the dnn
        # projections read each size class as one contiguous [G, rows, D] view
        tables = sorted(tables, key=lambda kv: kv[1].num_embeddings)
        D = tables[0][1].embedding_dim
        self.dim = D
        self.offsets = {}
        rows = 0
        for key, emb in tables:
            if emb.embedding_dim != D:
                raise ValueError('all tables of a group share the embedding dim')
            self.offsets[key] = rows
            rows += emb.num_embeddings
        self.rows = rows
        self.flat = torch.empty(rows, D, dtype=dtype, device=device)
        self.refs = {}
        for key, emb in tables:
            off = self.offsets[key]
            view = self.flat[off:off + emb.num_embeddings]
            with torch.no_grad():
                view.copy_(emb.weight.detach().to(device=device, dtype=dtype))
            emb.weight = torch.nn.Parameter(view, requires_grad=False)
            self.refs[key] = G.TableRef(emb.weight, self, off)
        self.exp_avg = torch.zeros(rows, D, dtype=torch.float32, device=device)
        self.exp_avg_sq = torch.zeros(rows, D, dtype=torch.float32, device=device)
        self.row_slot = torch.full((rows,), -1, dtype=torch.int32, device=device)
        self.pending = []
        self.token_type = None
        self.seq_len = 0
        self.dense_grads = {}  # row offset -> dense gradient of rows [off, off + len) (tables used in dense ops)
        self._identity = None

    def collect_dense(self, row_offset, grad):
        """Dense gradient (any float dtype) for rows [row_offset, row_offset + len(grad))."""
        prev = self.dense_grads.get(row_offset)
        if prev is not None and prev.shape == grad.shape:
            grad = prev.float() + grad
        elif prev is not None:
            raise RuntimeError(f'table group {self.name}: overlapping dense gradients at row {row_offset}')
        self.dense_grads[row_offset] = grad

    def identity(self):
        if self._identity is None:
            self._identity = torch.arange(self.rows, dtype=torch.int32, device=self.flat.device)
        return self._identity

    def dense_gradient(self, padding_idx=0):
        """fp32 [rows, D]: the row-sparse sources reduced densely plus the dense parts."""
        if self.pending:
            dense = K.embedding_backward(self.pending, self.rows, self.dim, padding_idx=padding_idx,
                                         token_type=self.token_type, seq_len=self.seq_len, dense=True).dense
        else:
            dense = torch.zeros(self.rows, self.dim, dtype=torch.float32, device=self.flat.device)
        for off, g in self.dense_grads.items():
            dense[off:off + g.shape[0]] += g
        return dense

    def step_dense_ranges(self, hp):
        """Dense-parity AdamW when every gradient of the group is dense (no
        row-sparse sources): each range from its own gradient (bf16 or fp32,
        no fp32 staging buffer), rows without gradient with g = 0."""
        pos = 0
        for off in sorted(self.dense_grads):
            g = self.dense_grads[off]
            if off > pos:
                K.table_adamw(self.flat[pos:off], self.exp_avg[pos:off], self.exp_avg_sq[pos:off], hp)
            end = off + g.shape[0]
            K.table_adamw_dense(self.flat[off:end], self.exp_avg[off:end], self.exp_avg_sq[off:end], hp, g)
            pos = end
        if pos < self.rows:
            K.table_adamw(self.flat[pos:], self.exp_avg[pos:], self.exp_avg_sq[pos:], hp)

    def collect(self, src, token_type, seq_len):
        self.pending.append(src)
        if token_type is not None:
            if self.token_type is not None and self.token_type is not token_type:
                raise RuntimeError(f'table group {self.name}: two masked lookups with different token_type in one step')
            self.token_type, self.seq_len = token_type, seq_len
        elif src.mode == 3:  # GRK_IDX_POSITION
            self.seq_len = seq_len

    def clear(self):
        self.pending = []
        self.token_type = None
        self.dense_grads = {}


# pos_emb (row-sparse gradients) apart from the feature tables, whose gradients
# are dense (they feed the dnns through projections: model._projection)
DEFAULT_GROUPS = (('item', ('item_emb',)), ('user', ('user_emb',)), ('pos', ('pos_emb',)), ('small', None))


class FusedAdamW:
    """AdamW over a BaselineModel: table groups on grk kernels, dense params on torch fused AdamW."""

    def __init__(self, model, lr=1e-3, betas=(0.9, 0.98), eps=1e-8, weight_decay=0.01, table_mode='dense',
                 table_dtype=torch.bfloat16, groups=DEFAULT_GROUPS):
        if table_mode not in ('dense', 'lazy'):
            raise ValueError("table_mode must be 'dense' or 'lazy'")
        self.model = model
        self.lr, self.betas, self.eps, self.weight_decay = lr, betas, eps, weight_decay
        self.lazy = table_mode == 'lazy'
        dev = model.item_emb.weight.device
        tables = model.table_modules()
        taken, self.groups, refs = set(), [], {}
        for gname, keys in groups:
            keys = [k for k in tables if k not in taken] if keys is None else list(keys)
            if not keys:
                continue
            taken.update(keys)
            grp = TableGroup(gname, [(k, tables[k]) for k in keys], table_dtype, dev)
            self.groups.append(grp)
            refs.update(grp.refs)
        model._table_refs = refs
        dense = [p for p in model.parameters() if p.requires_grad]
        self.dense = torch.optim.AdamW(dense, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                                       fused=dev.type == 'cuda')
        self.t = 0

    def zero_grad(self, set_to_none=True):
        self.dense.zero_grad(set_to_none=set_to_none)
        for g in self.groups:
            g.clear()

    @torch.no_grad()
    def step(self):
        self.t += 1
        self.dense.step()
        hp = K.adamw_hparams(self.lr, self.betas[0], self.betas[1], self.eps, self.weight_decay, self.t)
        for g in self.groups:
            if g.dense_grads and not g.pending:  # dense gradients only: per-range updates
                g.step_dense_ranges(hp)
            elif g.dense_grads:  # mixed: one dense fp32 gradient
                K.table_adamw(g.flat, g.exp_avg, g.exp_avg_sq, hp, None, g.dense_gradient(), None, 0, g.identity())
            elif g.pending:
                res = K.embedding_backward(g.pending, g.rows, g.dim, padding_idx=0, token_type=g.token_type,
                                           seq_len=g.seq_len, dense=False, sparse=True, row_slot=g.row_slot)
                K.table_adamw(g.flat, g.exp_avg, g.exp_avg_sq, hp, res.ids, res.rows, res.count, res.capacity,
                              None if self.lazy else g.row_slot, lazy=self.lazy)
            elif not self.lazy:
                K.table_adamw(g.flat, g.exp_avg, g.exp_avg_sq, hp)
            g.clear()
