"""AdamW oracle (numpy, fp32 op-for-op).  TEST INFRASTRUCTURE ONLY.

Restates ``torch.optim.AdamW(model.parameters(), lr, betas=(0.9, 0.98),
weight_decay=wd)`` as the reference constructs it
(``model/BaseLine/main.py:131`` -- default ``weight_decay=0.01``;
``model/BaseLineO1/main.py:174`` -- ``weight_decay=args.l2_emb``), one step,
in the single-tensor update order torch uses:

    p  *= 1 - lr * wd
    m   = m + (1 - b1) * (g - m)               (lerp)
    v   = v * b2 + (1 - b2) * g * g
    p  -= (lr / (1 - b1**t)) * m / (sqrt(v) / sqrt(1 - b2**t) + eps)

``dense_rows`` is the dense-parity table update (every row moves; rows with
no gradient see g = 0).  ``lazy_rows`` is the documented row-sparse deviation
(DESIGN.md): only rows that received a gradient are touched.
Pinned by the model-step golden vectors (params after one step).
"""
from __future__ import annotations

import numpy as np

F = np.float32


def step(p, g, m, v, t, lr, b1=0.9, b2=0.98, eps=1e-8, wd=0.01):
    p = np.asarray(p, F).copy(); g = np.asarray(g, F)
    m = np.asarray(m, F).copy(); v = np.asarray(v, F).copy()
    p *= F(1.0 - lr * wd)
    m = m + F(1.0 - b1) * (g - m)
    v = v * F(b2) + F(1.0 - b2) * g * g
    bc1 = 1.0 - b1 ** t
    bc2s = np.sqrt(1.0 - b2 ** t)
    denom = np.sqrt(v) / F(bc2s) + F(eps)
    p = p - F(lr / bc1) * (m / denom)
    return p, m, v


def dense_rows(table, m, v, ids, grad_rows, t, lr, b1=0.9, b2=0.98, eps=1e-8, wd=0.01):
    """Dense-parity table AdamW fed a row-sparse gradient (ids, grad_rows)."""
    g = np.zeros_like(np.asarray(table, F))
    g[np.asarray(ids, np.int64)] = grad_rows
    return step(table, g, m, v, t, lr, b1, b2, eps, wd)


def lazy_rows(table, m, v, ids, grad_rows, t, lr, b1=0.9, b2=0.98, eps=1e-8, wd=0.01):
    """Row-sparse (lazy) AdamW: only ``ids`` rows are updated."""
    table = np.asarray(table, F).copy(); m = np.asarray(m, F).copy(); v = np.asarray(v, F).copy()
    ids = np.asarray(ids, np.int64)
    p2, m2, v2 = step(table[ids], grad_rows, m[ids], v[ids], t, lr, b1, b2, eps, wd)
    table[ids] = p2; m[ids] = m2; v[ids] = v2
    return table, m, v
