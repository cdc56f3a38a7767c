"""HSTU pointwise-aggregated attention oracle (numpy).  TEST INFRASTRUCTURE ONLY.

**Parity unpinned.**  The reference has no HSTU (its blocks are
softmax MHA only, ``model/BaseLine/model.py:10-62``).  This restates the HSTU
layer of Zhai et al., "Actions Speak Louder than Words" (ICML 2024), eq. (1)-(3),
as the north star (BASELINE.json) specifies it, with the reference's own
masking convention (``model/BaseLine/model.py:331-335``: causal AND
key-not-padding):

    S[i,j] = alpha * <q_i, k_j> + rab[h, min(i - j, NB - 1)]          (j <= i)
    A[i,j] = SiLU(S[i,j]) * inv_n * mask[i,j]
    O[i]   = sum_j A[i,j] v_j

``rab`` is a learned relative-position bias, one value per (head, distance
bucket).  The paper's time bias is optional (``ts``, ``rab_t``): S[i,j] +=
rab_t[h, time_bucket(t_i - t_j)] with half-octave buckets of the time gap
(``time_bucket`` below, the kernels' integer definition, include/grk.h); the
reference's dataset drops timestamps (``model/BaseLine/dataset.py:117``), so
this part has no reference anchor at all.  Pinned by its own fp64 closed form
here and by finite-difference gradient checks in
``tests/test_oracle_selfcheck.py``.
"""
from __future__ import annotations

import numpy as np

from .attention import build_mask


def silu(x):
    return x / (1.0 + np.exp(-x))


def dsilu(x):
    s = 1.0 / (1.0 + np.exp(-x))
    return s * (1.0 + x * (1.0 - s))


def _bias(rab, T):
    rab = np.asarray(rab, np.float64)
    nb = rab.shape[1]
    i = np.arange(T)[:, None]
    j = np.arange(T)[None, :]
    bucket = np.clip(i - j, 0, nb - 1)
    return rab[:, bucket], bucket  # [H,T,T], [T,T]


def time_bucket(d, nbt):
    """Half-octave bucket of integer time gaps d: x = |d| + 1, l = floor(log2 x),
    bucket = min(2 l + (bit l-1 of x if l > 0), nbt - 1)."""
    x = np.abs(np.asarray(d, np.int64)) + 1
    l = np.floor(np.log2(x.astype(np.float64))).astype(np.int64)
    l = np.where((np.int64(1) << (l + 1)) <= x, l + 1, l)          # guard float rounding at powers of two
    l = np.where((np.int64(1) << l) > x, l - 1, l)
    h1 = np.where(l > 0, (x >> np.maximum(l - 1, 0)) & 1, 0)
    return np.minimum(2 * l + h1, nbt - 1)


def _time_bias(ts, key_valid, rab_t):
    """rab_t[h, time_bucket(t_i - t_j)] as [B,H,T,T] and the buckets [B,T,T]; times are
    taken relative to each sequence's first valid event and clamped to +-(2^30 - 1), as
    the kernels stage them."""
    ts = np.asarray(ts, np.int64)
    valid = np.asarray(key_valid, bool)
    B, T = ts.shape
    first = np.where(valid.any(1), valid.argmax(1), T)
    base = np.where(first < T, ts[np.arange(B), np.minimum(first, T - 1)], 0)
    rel = np.clip(ts - base[:, None], -(2 ** 30 - 1), 2 ** 30 - 1)
    bt = time_bucket(rel[:, :, None] - rel[:, None, :], np.asarray(rab_t).shape[1])
    return np.asarray(rab_t, np.float64)[:, bt].transpose(1, 0, 2, 3), bt


def forward(q, k, v, key_valid, rab, alpha, inv_n, ts=None, rab_t=None):
    """Returns ``(out [B,H,T,hd], s [B,H,T,T] pre-activation, mask [B,1,T,T])``."""
    q = np.asarray(q, np.float64); k = np.asarray(k, np.float64); v = np.asarray(v, np.float64)
    T = q.shape[2]
    bias, _ = _bias(rab, T)
    mask = build_mask(key_valid, True)[:, None]
    s = alpha * np.einsum('bhid,bhjd->bhij', q, k) + bias[None]
    if rab_t is not None:
        s = s + _time_bias(ts, key_valid, rab_t)[0]
    a = np.where(mask, silu(s) * inv_n, 0.0)
    out = np.einsum('bhij,bhjd->bhid', a, v)
    return out, s, mask


def backward(q, k, v, key_valid, rab, alpha, inv_n, dout, ts=None, rab_t=None):
    """Returns ``(dq, dk, dv, drab [H, NB])``, plus ``drab_t [H, NBT]`` with a time bias."""
    q = np.asarray(q, np.float64); k = np.asarray(k, np.float64); v = np.asarray(v, np.float64)
    dout = np.asarray(dout, np.float64)
    T = q.shape[2]
    _, s, mask = forward(q, k, v, key_valid, rab, alpha, inv_n, ts, rab_t)
    a = np.where(mask, silu(s) * inv_n, 0.0)
    dv = np.einsum('bhij,bhid->bhjd', a, dout)
    da = np.einsum('bhid,bhjd->bhij', dout, v)
    ds = np.where(mask, da * dsilu(s) * inv_n, 0.0)
    dq = alpha * np.einsum('bhij,bhjd->bhid', ds, k)
    dk = alpha * np.einsum('bhij,bhid->bhjd', ds, q)
    nb = np.asarray(rab).shape[1]
    _, bucket = _bias(rab, T)
    drab = np.zeros((q.shape[1], nb), np.float64)
    dsh = ds.sum(axis=0)  # [H,T,T]
    for h in range(q.shape[1]):
        np.add.at(drab[h], bucket.reshape(-1), dsh[h].reshape(-1))
    if rab_t is None:
        return dq, dk, dv, drab
    _, bt = _time_bias(ts, key_valid, rab_t)
    drab_t = np.zeros((q.shape[1], np.asarray(rab_t).shape[1]), np.float64)
    for h in range(q.shape[1]):
        np.add.at(drab_t[h], bt.reshape(-1), ds[:, h].reshape(-1))
    return dq, dk, dv, drab, drab_t
