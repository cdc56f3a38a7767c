"""The grk kernels as ``torch.library`` custom operators (namespace ``grk``).

These are what the drop-in model calls, so that the reference's own training
flags work unchanged (``model/BaseLine/run.sh:7``: ``--use_amp
--use_torch_compile``; ``main.py:114-116`` compiles the model, ``:173`` runs the
step under ``torch.amp.autocast('cuda')`` = fp16 with a ``GradScaler``):

* every op has a fake (meta) implementation, so ``torch.compile`` traces the
  model through it instead of breaking the graph at an opaque ctypes call;
* every differentiable op has its backward registered as another custom op
  (``register_autograd``), so AOTAutograd sees the backward too;
* dtypes: the attention ops take fp32 / fp16 / bf16 inputs.  fp32 and fp16
  run the fp32-fidelity kernels (``precise=2``: operands read exactly, split
  into bf16 hi + lo) when the shape allows, bf16 runs the product kernels.
  ``pair_logits`` and ``feature_lookup`` compute in fp32 under autocast (as
  the reference's fp32 embedding tables and its BCE do): an autocast rule
  casts their floating inputs to fp32.

Ops (file:line of the reference call each replaces):
  grk::feature_lookup (+ _backward)   nn.Embedding lookups + array bag-sums of
                                      feat2emb, model/BaseLine/model.py:242-277
  grk::softmax_attention (+ _backward) F.scaled_dot_product_attention with
                                      log2feats' mask, model/BaseLine/model.py:39-43
  grk::hstu_core (+ _backward)        HSTU layer core (north star, oracle/hstu.py)
  grk::pair_logits (+ _backward)      (h * e).sum(-1) * mask, model/BaseLine/model.py:378-384

The fused trainer's table-group path (row-sparse gradients collected by the
optimizer) stays on autograd.Functions in functional.py: it is replayed from a
HIP graph instead of compiled.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
from torch import Tensor

from . import _lib as L
from . import kernels as K

# --------------------------------------------------------------- lookups ----


@torch.library.custom_op('grk::feature_lookup', mutates_args=(), device_types='cuda')
def feature_lookup(tables: List[Tensor], indices: List[Tensor], table_of: List[int], out_cols: List[int],
                   modes: List[int], bags: List[int], token_type: Optional[Tensor], seq_len: int, num_tokens: int,
                   out_ld: int) -> Tensor:
    """out[n, out_cols[i]:+D] = sum over the bag of tables[table_of[i]][row(indices[i][n, a])]
    (one fused grk_embedding_gather; columns no lookup writes are zero)."""
    dt, dev = tables[0].dtype, tables[0].device
    out = torch.zeros(num_tokens, out_ld, dtype=dt, device=dev)
    lookups = [K.Lookup(tables[t], idx, c, m, b) for t, idx, c, m, b in zip(table_of, indices, out_cols, modes, bags)]
    for i in range(0, len(lookups), L.MAX_FEATURES):
        K.embedding_gather(lookups[i:i + L.MAX_FEATURES], out, num_tokens, token_type, seq_len)
    return out


@feature_lookup.register_fake
def _(tables, indices, table_of, out_cols, modes, bags, token_type, seq_len, num_tokens, out_ld):
    return tables[0].new_empty(num_tokens, out_ld)


@torch.library.custom_op('grk::feature_lookup_backward', mutates_args=(), device_types='cuda')
def feature_lookup_backward(grad: Tensor, indices: List[Tensor], table_of: List[int], out_cols: List[int],
                            modes: List[int], bags: List[int], token_type: Optional[Tensor], seq_len: int,
                            table_rows: List[int], dim: int, table_dtypes: List[int]) -> List[Tensor]:
    """Dense gradient of every table (padding row 0 excluded): one deterministic
    grk_embedding_backward over all lookups, tables stacked."""
    offs, total = [], 0
    for r in table_rows:
        offs.append(total)
        total += r
    grad = grad if grad.stride(-1) == 1 else grad.contiguous()
    src = [K.GradSource(idx, grad, c, m, b, offs[t], table_rows[t])
           for t, idx, c, m, b in zip(table_of, indices, out_cols, modes, bags)]
    dense = K.embedding_backward(src, total, dim, padding_idx=0, token_type=token_type, seq_len=seq_len,
                                 dense=True).dense
    # one fresh tensor per table (outputs may not alias each other)
    return [dense[o:o + r].to(_DT[d], copy=True) for o, r, d in zip(offs, table_rows, table_dtypes)]


@feature_lookup_backward.register_fake
def _(grad, indices, table_of, out_cols, modes, bags, token_type, seq_len, table_rows, dim, table_dtypes):
    return [grad.new_empty(r, dim, dtype=_DT[d]) for r, d in zip(table_rows, table_dtypes)]


_DT = {L.GRK_F32: torch.float32, L.GRK_BF16: torch.bfloat16, L.GRK_F16: torch.float16}


def _lookup_setup(ctx, inputs, output):
    tables, indices, table_of, out_cols, modes, bags, token_type, seq_len, num_tokens, out_ld = inputs
    ctx.save_for_backward(*indices, *([token_type] if token_type is not None else []))
    ctx.meta = (len(indices), token_type is not None, list(table_of), list(out_cols), list(modes), list(bags),
                seq_len, [t.shape[0] for t in tables], tables[0].shape[1], [L.dtype_code(t.dtype) for t in tables])


def _lookup_backward(ctx, grad):
    n, has_tt, table_of, out_cols, modes, bags, seq_len, rows, dim, dts = ctx.meta
    saved = ctx.saved_tensors
    indices, token_type = list(saved[:n]), (saved[n] if has_tt else None)
    gt = torch.ops.grk.feature_lookup_backward(grad, indices, table_of, out_cols, modes, bags, token_type, seq_len,
                                               rows, dim, dts)
    # the gradient mirrors the inputs' structure: one entry per element of the tensor lists
    return list(gt), [None] * n, None, None, None, None, None, None, None, None


torch.library.register_autograd('grk::feature_lookup', _lookup_backward, setup_context=_lookup_setup)
torch.library.register_autocast('grk::feature_lookup', 'cuda', torch.float32)


# ------------------------------------------------------------- attention ----
@torch.library.custom_op('grk::seq_ranges', mutates_args=(), device_types='cuda')
def seq_ranges(key_valid: Tensor) -> Tensor:
    """int32 [B, 3]: (first valid key, contiguous flag, longest-first order) (grk_seq_ranges)."""
    return K.seq_ranges(key_valid)


@seq_ranges.register_fake
def _(key_valid):
    return key_valid.new_empty(key_valid.shape[0], 3, dtype=torch.int32)


def _attn_plan(dtype, T, hd, precise):
    """(fidelity, kernel precise mode, kernel output dtype) for q/k/v of `dtype`."""
    if dtype in (torch.float32, torch.float16) and K.fidelity_supported(T, hd):
        return True, 2, torch.float32
    return False, int(precise), (torch.float32 if dtype == torch.float32 else torch.bfloat16)


def _seed_arg(seed, seed_dev):
    return seed_dev if seed_dev is not None else seed


def _softmax_args(qkv, key_valid, heads, head_dim, dropout_p, seed, seed_dev, precise, seq_range, row_base=None):
    B, T = key_valid.shape
    D = heads * head_dim
    fid, prec, kdt = _attn_plan(qkv.dtype, T, head_dim, precise)
    xb = qkv.contiguous() if fid else qkv.to(torch.bfloat16).contiguous()
    args = K.attn_args(L.ATTN_SOFTMAX, xb[:, :D], xb[:, D:2 * D], xb[:, 2 * D:3 * D], B, T, heads, head_dim,
                       key_valid=key_valid, dropout_p=dropout_p, seed=_seed_arg(seed, seed_dev), precise=prec,
                       out_dtype=kdt, seq_range=seq_range, row_base=row_base)
    return args, xb, prec, kdt


@torch.library.custom_op('grk::softmax_attention', mutates_args=(), device_types='cuda')
def softmax_attention(qkv: Tensor, key_valid: Tensor, heads: int, head_dim: int, dropout_p: float, seed: int,
                      seed_dev: Optional[Tensor], precise: int, seq_range: Optional[Tensor],
                      row_base: Optional[Tensor] = None) -> Tuple[Tensor, Tensor]:
    """Causal + key-padding softmax attention of a packed [B*T, 3D] (q|k|v) -- or of
    the batch's jagged rows with row_base (jagged.py).  Returns (out [rows, D] in the
    kernel dtype: fp32 for fp32/fp16 inputs, bf16 for bf16; lse fp32 [B, H, T])."""
    B, T = key_valid.shape
    args, _, _, kdt = _softmax_args(qkv, key_valid, heads, head_dim, dropout_p, seed, seed_dev, precise, seq_range,
                                    row_base)
    out = torch.empty(qkv.shape[0], heads * head_dim, dtype=kdt, device=qkv.device)
    lse = torch.empty(B, heads, T, dtype=torch.float32, device=qkv.device)
    K.attention_fwd(args, out, lse)
    return out, lse


@softmax_attention.register_fake
def _(qkv, key_valid, heads, head_dim, dropout_p, seed, seed_dev, precise, seq_range, row_base=None):
    B, T = key_valid.shape
    kdt = _attn_plan(qkv.dtype, T, head_dim, precise)[2]
    return (qkv.new_empty(qkv.shape[0], heads * head_dim, dtype=kdt), qkv.new_empty(B, heads, T, dtype=torch.float32))


@torch.library.custom_op('grk::softmax_attention_backward', mutates_args=(), device_types='cuda')
def softmax_attention_backward(gout: Tensor, qkv: Tensor, out: Tensor, lse: Tensor, key_valid: Tensor, heads: int,
                               head_dim: int, dropout_p: float, seed: int, seed_dev: Optional[Tensor], precise: int,
                               seq_range: Optional[Tensor], row_base: Optional[Tensor] = None) -> Tensor:
    """d(q|k|v) [rows, 3D] in qkv's dtype."""
    B, T = key_valid.shape
    D = heads * head_dim
    args, xb, prec, kdt = _softmax_args(qkv, key_valid, heads, head_dim, dropout_p, seed, seed_dev, precise,
                                        seq_range, row_base)
    dqkv = torch.empty(qkv.shape[0], 3 * D, dtype=kdt, device=qkv.device)
    delta = torch.empty(B, heads, T, dtype=torch.float32, device=qkv.device)
    g = gout.contiguous()
    if g.dtype not in (torch.float32, torch.bfloat16) or (prec == 2 and g.dtype != torch.float32):
        g = g.float()
    K.attention_bwd(args, out, g, lse, delta, dqkv[:, :D], dqkv[:, D:2 * D], dqkv[:, 2 * D:])
    return dqkv if dqkv.dtype == qkv.dtype else dqkv.to(qkv.dtype)


@softmax_attention_backward.register_fake
def _(gout, qkv, out, lse, key_valid, heads, head_dim, dropout_p, seed, seed_dev, precise, seq_range, row_base=None):
    return torch.empty_like(qkv, memory_format=torch.contiguous_format)


def _softmax_setup(ctx, inputs, output):
    qkv, key_valid, heads, head_dim, dropout_p, seed, seed_dev, precise, seq_range, row_base = inputs
    out, lse = output
    ctx.save_for_backward(qkv, out, lse, key_valid, seed_dev, seq_range, row_base)
    ctx.meta = (heads, head_dim, dropout_p, seed, precise)


def _softmax_backward(ctx, gout, glse):
    qkv, out, lse, key_valid, seed_dev, seq_range, row_base = ctx.saved_tensors
    heads, head_dim, dropout_p, seed, precise = ctx.meta
    dqkv = torch.ops.grk.softmax_attention_backward(gout, qkv, out, lse, key_valid, heads, head_dim, dropout_p, seed,
                                                    seed_dev, precise, seq_range, row_base)
    return dqkv, None, None, None, None, None, None, None, None, None


torch.library.register_autograd('grk::softmax_attention', _softmax_backward, setup_context=_softmax_setup)


def _hstu_args(pb, rab32, key_valid, heads, head_dim, inv_n, precise, seq_range, timestamps=None, rab_t32=None,
               row_base=None):
    B, T = key_valid.shape
    D = heads * head_dim
    return K.attn_args(L.ATTN_HSTU, pb[:, 2 * D:3 * D], pb[:, 3 * D:], pb[:, D:2 * D], B, T, heads, head_dim,
                       key_valid=key_valid, scale=head_dim ** -0.5, rab=rab32, inv_n=inv_n, precise=precise,
                       out_dtype=torch.bfloat16, act='silu', seq_range=seq_range, timestamps=timestamps,
                       rab_t=rab_t32, row_base=row_base)


def _f32(t):
    return None if t is None else t.float().contiguous()


@torch.library.custom_op('grk::hstu_core', mutates_args=(), device_types='cuda')
def hstu_core(pre: Tensor, rab: Tensor, ln_w: Tensor, ln_b: Tensor, key_valid: Tensor, heads: int, head_dim: int,
              inv_n: float, eps: float, precise: int, dropout_p: float, seed: int, seed_dev: Optional[Tensor],
              seq_range: Optional[Tensor], timestamps: Optional[Tensor] = None,
              rab_t: Optional[Tensor] = None, row_base: Optional[Tensor] = None) -> Tuple[Tensor, Tensor, Tensor]:
    """y = dropout(LayerNorm(HSTU-attn(SiLU(q), SiLU(k), SiLU(v))) * SiLU(u)) on the
    [B*T, 4D] (u|v|q|k) pre-activation; bf16 math.  Returns (y bf16, o bf16,
    LayerNorm stats fp32 [B*T, 2]).  timestamps (int64 [B, T]) + rab_t ([H, nbt]):
    the time bias rab_t[h, time_bucket(t_q - t_k)]."""
    D = heads * head_dim
    pb = pre.to(torch.bfloat16).contiguous()
    args = _hstu_args(pb, rab.float().contiguous(), key_valid, heads, head_dim, inv_n, precise, seq_range,
                      timestamps, _f32(rab_t), row_base)
    o = torch.empty(pre.shape[0], D, dtype=torch.bfloat16, device=pre.device)
    K.attention_fwd(args, o)
    y, stats = K.norm_gate_fwd(o, pb[:, :D], ln_w.float().contiguous(), ln_b.float().contiguous(), eps, dropout_p,
                               _seed_arg(seed, seed_dev))
    return y, o, stats


@hstu_core.register_fake
def _(pre, rab, ln_w, ln_b, key_valid, heads, head_dim, inv_n, eps, precise, dropout_p, seed, seed_dev, seq_range,
      timestamps=None, rab_t=None, row_base=None):
    N, D = pre.shape[0], heads * head_dim
    return (pre.new_empty(N, D, dtype=torch.bfloat16), pre.new_empty(N, D, dtype=torch.bfloat16),
            pre.new_empty(N, 2, dtype=torch.float32))


@torch.library.custom_op('grk::hstu_core_backward', mutates_args=(), device_types='cuda')
def hstu_core_backward(gy: Tensor, pre: Tensor, o: Tensor, stats: Tensor, rab: Tensor, ln_w: Tensor, ln_b: Tensor,
                       key_valid: Tensor, heads: int, head_dim: int, inv_n: float, precise: int, dropout_p: float,
                       seed: int, seed_dev: Optional[Tensor], seq_range: Optional[Tensor],
                       timestamps: Optional[Tensor] = None,
                       rab_t: Optional[Tensor] = None,
                       row_base: Optional[Tensor] = None) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor]:
    """(dpre in pre's dtype, drab, dln_w, dln_b, drab_t in their parameters' dtypes;
    drab_t is empty without a time bias)."""
    D = heads * head_dim
    pb = pre.to(torch.bfloat16).contiguous()
    rab32 = rab.float().contiguous()
    g = gy.to(torch.bfloat16).contiguous()
    dpre = torch.empty(pre.shape[0], 4 * D, dtype=torch.bfloat16, device=pre.device)
    do, _, dw, db = K.norm_gate_bwd(g, o, pb[:, :D], ln_w.float().contiguous(), ln_b.float().contiguous(), stats,
                                    dropout_p, _seed_arg(seed, seed_dev), du=dpre[:, :D])
    drab = torch.empty_like(rab32)   # written by the backward (drab_set): no fill kernels
    rab_t32 = _f32(rab_t)
    drab_t = torch.empty_like(rab_t32) if rab_t is not None else None
    args = _hstu_args(pb, rab32, key_valid, heads, head_dim, inv_n, precise, seq_range, timestamps, rab_t32, row_base)
    K.attention_bwd(args, None, do, None, None, dpre[:, 2 * D:3 * D], dpre[:, 3 * D:], dpre[:, D:2 * D], drab,
                    drab_t=drab_t, drab_set=True)
    drab_t = drab_t.to(rab_t.dtype) if rab_t is not None else rab.new_empty(0)
    return dpre.to(pre.dtype), drab.to(rab.dtype), dw.to(ln_w.dtype), db.to(ln_b.dtype), drab_t


@hstu_core_backward.register_fake
def _(gy, pre, o, stats, rab, ln_w, ln_b, key_valid, heads, head_dim, inv_n, precise, dropout_p, seed, seed_dev,
      seq_range, timestamps=None, rab_t=None, row_base=None):
    return (torch.empty_like(pre), torch.empty_like(rab), torch.empty_like(ln_w), torch.empty_like(ln_b),
            torch.empty_like(rab_t) if rab_t is not None else rab.new_empty(0))


def _hstu_setup(ctx, inputs, output):
    (pre, rab, ln_w, ln_b, key_valid, heads, head_dim, inv_n, eps, precise, dropout_p, seed, seed_dev, seq_range,
     timestamps, rab_t, row_base) = inputs
    _, o, stats = output
    # o and stats are saved for backward, never differentiated: their None gradients stay
    # None (materialised, they were a bf16 [N, D] and an fp32 [N, 2] zero fill per layer)
    ctx.set_materialize_grads(False)
    ctx.save_for_backward(pre, o, stats, rab, ln_w, ln_b, key_valid, seed_dev, seq_range, timestamps, rab_t, row_base)
    ctx.meta = (heads, head_dim, inv_n, precise, dropout_p, seed)


def _hstu_backward(ctx, gy, go, gstats):
    if gy is None:   # y unused (grads are not materialised: _hstu_setup)
        return (None,) * 17
    pre, o, stats, rab, ln_w, ln_b, key_valid, seed_dev, seq_range, timestamps, rab_t, row_base = ctx.saved_tensors
    heads, head_dim, inv_n, precise, dropout_p, seed = ctx.meta
    dpre, drab, dw, db, drab_t = torch.ops.grk.hstu_core_backward(gy, pre, o, stats, rab, ln_w, ln_b, key_valid,
                                                                  heads, head_dim, inv_n, precise, dropout_p, seed,
                                                                  seed_dev, seq_range, timestamps, rab_t, row_base)
    return (dpre, drab, dw, db, None, None, None, None, None, None, None, None, None, None, None,
            drab_t if rab_t is not None else None, None)


torch.library.register_autograd('grk::hstu_core', _hstu_backward, setup_context=_hstu_setup)


# ---------------------------------------------------------------- logits ----
@torch.library.custom_op('grk::pair_logits', mutates_args=(), device_types='cuda')
def pair_logits(h: Tensor, e_pos: Tensor, e_neg: Tensor, next_token_type: Tensor) -> Tuple[Tensor, Tensor]:
    """(pos, neg) fp32 [N] = rowwise <h, e> * (next_token_type == 1); h, e [N, D]."""
    dt = torch.promote_types(torch.promote_types(h.dtype, e_pos.dtype), e_neg.dtype)
    h2, p2, n2 = (x.to(dt).contiguous() for x in (h, e_pos, e_neg))
    return K.pair_logits_fwd(h2, p2, n2, next_token_type)


@pair_logits.register_fake
def _(h, e_pos, e_neg, next_token_type):
    N = h.shape[0]
    return h.new_empty(N, dtype=torch.float32), h.new_empty(N, dtype=torch.float32)


@torch.library.custom_op('grk::pair_logits_backward', mutates_args=(), device_types='cuda')
def pair_logits_backward(gpos: Tensor, gneg: Tensor, h: Tensor, e_pos: Tensor, e_neg: Tensor,
                         next_token_type: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    dt = torch.promote_types(torch.promote_types(h.dtype, e_pos.dtype), e_neg.dtype)
    h2, p2, n2 = (x.to(dt).contiguous() for x in (h, e_pos, e_neg))
    dh, dp, dn = K.pair_logits_bwd(h2, p2, n2, gpos=gpos.float().contiguous(), gneg=gneg.float().contiguous(),
                                   next_token_type=next_token_type)
    return dh.to(h.dtype), dp.to(e_pos.dtype), dn.to(e_neg.dtype)


@pair_logits_backward.register_fake
def _(gpos, gneg, h, e_pos, e_neg, next_token_type):
    return torch.empty_like(h), torch.empty_like(e_pos), torch.empty_like(e_neg)


def _logits_setup(ctx, inputs, output):
    ctx.save_for_backward(*inputs)


def _logits_backward(ctx, gpos, gneg):
    h, ep, en, ntt = ctx.saved_tensors
    gpos = torch.zeros(h.shape[0], dtype=torch.float32, device=h.device) if gpos is None else gpos
    gneg = torch.zeros(h.shape[0], dtype=torch.float32, device=h.device) if gneg is None else gneg
    dh, dp, dn = torch.ops.grk.pair_logits_backward(gpos, gneg, h, ep, en, ntt)
    return dh, dp, dn, None


torch.library.register_autograd('grk::pair_logits', _logits_backward, setup_context=_logits_setup)
torch.library.register_autocast('grk::pair_logits', 'cuda', torch.float32)
