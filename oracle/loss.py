"""Logits + loss oracle (numpy).  TEST INFRASTRUCTURE ONLY.

* ``bce``: the reference's training loss.  Logits are row-wise dot products
  masked by ``next_token_type == 1`` (``model/BaseLine/model.py:374-382``;
  ``model/BaseLineO1/model.py:491-502``); the loss is
  ``BCEWithLogits(pos[idx], 1) + BCEWithLogits(neg[idx], 0)``, each a mean over
  the positions ``idx = np.where(next_token_type == 1)``
  (``model/BaseLine/main.py:177-182``; ``model/BaseLineO1/main.py:233-242``).
  Pinned by the model-step golden vectors.
* ``sampled_softmax``: **parity unpinned** north-star loss (not in the
  reference): in-batch softmax over every valid position's
  positive item, temperature ``tau``, with same-item collisions masked out.
"""
from __future__ import annotations

import numpy as np


def softplus(x):
    return np.logaddexp(0.0, x)


def sigmoid(x):
    return 0.5 * (1.0 + np.tanh(0.5 * x))


def bce(h, e_pos, e_neg, next_token_type):
    """Returns ``(loss, pos_logits, neg_logits, dh, de_pos, de_neg)`` (fp64).

    h, e_pos, e_neg: ``[N, D]``; next_token_type: ``[N]``.
    Gradients are of the scalar loss (upstream grad 1).
    """
    h = np.asarray(h, np.float64); ep = np.asarray(e_pos, np.float64); en = np.asarray(e_neg, np.float64)
    m = (np.asarray(next_token_type) == 1)
    mf = m.astype(np.float64)
    pos = (h * ep).sum(-1) * mf
    neg = (h * en).sum(-1) * mf
    cnt = max(int(m.sum()), 1)
    loss = softplus(-pos[m]).sum() / cnt + softplus(neg[m]).sum() / cnt
    gpos = np.where(m, (sigmoid(pos) - 1.0) / cnt, 0.0)
    gneg = np.where(m, sigmoid(neg) / cnt, 0.0)
    dh = gpos[:, None] * ep + gneg[:, None] * en
    dep = gpos[:, None] * h
    den = gneg[:, None] * h
    return loss, pos, neg, dh, dep, den


def sampled_softmax(h, e, item_ids, valid, tau, log_q=None):
    """In-batch sampled softmax.  Returns ``(loss, dh, de)`` (fp64).

    Row i (valid) scores every valid column j: ``z_ij = <h_i, e_j> / tau - log_q[j]``
    (``log_q`` optional: the logQ correction, Yi et al. RecSys 2019 -- the log
    sampling probability of column j's item; a constant, so the gradient
    formulas are unchanged);
    columns j != i with ``item_ids[j] == item_ids[i]`` are masked (the same
    item is not a negative of itself); the target is column i.
    ``loss = mean_i (logsumexp_j z_ij - z_ii)`` over valid rows.
    """
    h = np.asarray(h, np.float64); e = np.asarray(e, np.float64)
    ids = np.asarray(item_ids).reshape(-1)
    valid = np.asarray(valid, bool).reshape(-1)
    n = h.shape[0]
    z = h @ e.T / tau
    if log_q is not None:
        z = z - np.asarray(log_q, np.float64).reshape(1, -1)
    colmask = valid[None, :] & ~((ids[:, None] == ids[None, :]) & ~np.eye(n, dtype=bool))
    z = np.where(colmask, z, -np.inf)
    m = z.max(axis=1, keepdims=True)
    m = np.where(np.isfinite(m), m, 0.0)
    ez = np.where(colmask, np.exp(z - m), 0.0)
    lse = m[:, 0] + np.log(ez.sum(1))
    cnt = max(int(valid.sum()), 1)
    diag = np.diag(z)
    loss = np.where(valid, lse - diag, 0.0).sum() / cnt
    p = ez / ez.sum(1, keepdims=True)
    g = np.where(valid[:, None], p - np.eye(n), 0.0) / cnt / tau
    g = np.where(colmask, g, 0.0)
    dh = g @ e
    de = g.T @ h
    return loss, dh, de
