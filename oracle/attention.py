"""Masked softmax attention oracle (numpy).  TEST INFRASTRUCTURE ONLY.

Restates ``FlashMultiHeadAttention``'s core,
``F.scaled_dot_product_attention(Q, K, V, attn_mask=mask.unsqueeze(1))``
(``model/BaseLine/model.py:39-43``; math fallback ``:45-54``;
``model/BaseLineO1/model.py:73-92``) for the mask ``log2feats`` builds
(``model/BaseLine/model.py:331-335``): ``mask[b,i,j] = (j <= i) & key_valid[b,j]``
with ``key_valid = token_type != 0``.

Rows with no visible key (left padding) output 0 and get 0 gradient, which is
what torch 2.10's SDPA returns for a fully-masked boolean row.

Shapes: q, k, v ``[B, H, T, hd]``; key_valid ``[B, T]`` bool.  Computed in
float64 unless the inputs are float32 and ``exact32`` is requested.
"""
from __future__ import annotations

import numpy as np


def build_mask(key_valid: np.ndarray, causal: bool = True) -> np.ndarray:
    """``tril(T,T) & key_valid[:, None, :]`` -> [B, T, T] (model/BaseLine/model.py:332-335)."""
    key_valid = np.asarray(key_valid, dtype=bool)
    T = key_valid.shape[1]
    tri = np.tril(np.ones((T, T), dtype=bool)) if causal else np.ones((T, T), dtype=bool)
    return tri[None] & key_valid[:, None, :]


def forward(q, k, v, key_valid, scale=None, causal=True, keep=None, dropout_p=0.0):
    """Returns ``(out [B,H,T,hd], lse [B,H,T], probs [B,H,T,T])``.

    ``keep`` (optional bool ``[B,H,T,T]``) is a dropout keep-mask applied to
    the probabilities with ``1/(1-p)`` rescaling, as SDPA does in training.
    """
    q = np.asarray(q, np.float64); k = np.asarray(k, np.float64); v = np.asarray(v, np.float64)
    hd = q.shape[-1]
    scale = hd ** -0.5 if scale is None else scale
    mask = build_mask(key_valid, causal)[:, None]  # [B,1,T,T]
    s = np.einsum('bhid,bhjd->bhij', q, k) * scale
    s = np.where(mask, s, -np.inf)
    m = s.max(axis=-1, keepdims=True)
    any_visible = np.isfinite(m)
    m = np.where(any_visible, m, 0.0)
    e = np.where(mask, np.exp(s - m), 0.0)
    l = e.sum(axis=-1, keepdims=True)
    p = np.where(any_visible, e / np.where(l > 0, l, 1.0), 0.0)
    lse = np.where(any_visible[..., 0], (m + np.log(np.where(l > 0, l, 1.0)))[..., 0], -np.inf)
    pd = p
    if keep is not None:
        pd = p * keep / (1.0 - dropout_p)
    out = np.einsum('bhij,bhjd->bhid', pd, v)
    return out, lse, p


def backward(q, k, v, key_valid, dout, scale=None, causal=True, keep=None, dropout_p=0.0, out_stored=None):
    """Returns ``(dq, dk, dv)`` of ``forward`` for upstream ``dout``.

    ``out_stored``: the forward output as the caller kept it (e.g. rounded to
    bf16).  The flash-style backward forms delta = rowsum(dout * out) from the
    STORED output, so a kernel fed a bf16 output is checked against the same
    delta (its inputs identically rounded); default: the exact output."""
    q = np.asarray(q, np.float64); k = np.asarray(k, np.float64); v = np.asarray(v, np.float64)
    dout = np.asarray(dout, np.float64)
    hd = q.shape[-1]
    scale = hd ** -0.5 if scale is None else scale
    out, _, p = forward(q, k, v, key_valid, scale, causal, keep, dropout_p)
    rs = 1.0 / (1.0 - dropout_p)
    pd = p if keep is None else p * keep * rs
    dv = np.einsum('bhij,bhid->bhjd', pd, dout)
    dpd = np.einsum('bhid,bhjd->bhij', dout, v)
    dp = dpd if keep is None else dpd * keep * rs
    if out_stored is not None:
        out = np.asarray(out_stored, np.float64)
    delta = (dout * out).sum(-1, keepdims=True)  # == sum_j p_ij dp_ij
    ds = p * (dp - delta)
    dq = np.einsum('bhij,bhjd->bhid', ds, k) * scale
    dk = np.einsum('bhij,bhid->bhjd', ds, q) * scale
    return dq, dk, dv
