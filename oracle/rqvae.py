"""CPU oracle for the RQ-VAE semantic-ID tokenizer (config 4) -- TEST
INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
checker, never by the product path.

The reference has no tokenizer ("RQ-VAE semantic-ID tokenizer
(config 4) -- NO"); BASELINE.json configs[3] names it on top of
model/BaseLineO1.  Its semantic ids enter the O1 model as item_sparse features
(/root/reference/model/BaseLineO1/model.py:271-280 builds one embedding table per
item_sparse feature, :355 looks them up), computed from the items' multimodal
embeddings (mm_emb, BaseLineO1/dataset.py:535-567 loads them).  So this
restatement follows the published RQ-VAE (Lee et al., CVPR 2022, "Autoregressive
image generation using residual quantization"; TIGER, Rajput et al., NeurIPS
2023, for semantic ids): encoder MLP -> L-level residual quantiser -> decoder
MLP; loss = MSE(x_hat, x) + sum_l ||sg(r_l) - c_l||^2 + beta ||r_l - sg(c_l)||^2
(means over rows x dim).  **Parity unpinned** for the model as a whole (no
reference implementation or fixture exists); the code search itself is pinned
by construction: ``rq_assign`` defines the argmin exactly and the HIP kernel
(csrc/grk_rqvae.hip) must reproduce it bit for bit.
"""
from __future__ import annotations

import numpy as np


def rq_assign(z, codebooks):
    """Residual code search (grk_rq_assign's contract, include/grk.h).

    z float32 [n, d]; codebooks float32 [L, K, d].  Per level the distance to
    code k is sum_j (r[j] - C[k, j])^2 accumulated j ascending in float32 with
    every difference, square and sum rounded (numpy float32 ops round each
    step; no FMA); ties go to the lowest k.  Returns codes int32 [n, L], quant
    float32 [n, d] = C_0[c_0] + C_1[c_1] + ... (level order), dist float32
    [n, L] (the minimum distances), resid float32 [n, d] = r_L.
    """
    z = np.ascontiguousarray(z, dtype=np.float32)
    cb = np.ascontiguousarray(codebooks, dtype=np.float32)
    n, d = z.shape
    L, K, _ = cb.shape
    r = z.copy()
    codes = np.zeros((n, L), np.int32)
    dist = np.zeros((n, L), np.float32)
    quant = np.zeros((n, d), np.float32)
    rows = np.arange(n)
    for lvl in range(L):
        C = cb[lvl]
        acc = np.zeros((n, K), np.float32)
        for j in range(d):
            diff = r[:, j:j + 1] - C[None, :, j]          # float32, rounded
            acc = acc + diff * diff                       # square rounded, then sum rounded
        k = np.argmin(acc, axis=1)                        # first minimum = lowest k
        nan_rows = np.isnan(acc).all(axis=1)
        k[nan_rows] = 0
        codes[:, lvl] = k
        dist[:, lvl] = acc[rows, k]
        sel = C[k]
        r = r - sel
        quant = sel.copy() if lvl == 0 else quant + sel
    return codes, quant, dist, r


def rq_loss(z, codebooks, codes, beta):
    """Quantiser loss for given codes: sum over levels of
    mean((r_l - c_l)^2) * (1 + beta) (codebook + commitment terms share the
    value; they differ only in which side the gradient reaches) with
    r_{l+1} = r_l - c_l; float64."""
    z = np.asarray(z, np.float64)
    cb = np.asarray(codebooks, np.float64)
    r = z.copy()
    total = 0.0
    for lvl in range(cb.shape[0]):
        c = cb[lvl][codes[:, lvl]]
        total += (1.0 + beta) * np.mean((r - c) ** 2)
        r = r - c
    return total


def mlp(x, layers):
    """Linear -> ReLU ... -> Linear (no activation after the last), float64.
    ``layers`` = [(W [out, in], b [out]), ...] as torch.nn.Linear stores them."""
    h = np.asarray(x, np.float64)
    for i, (w, b) in enumerate(layers):
        h = h @ np.asarray(w, np.float64).T + np.asarray(b, np.float64)
        if i + 1 < len(layers):
            h = np.maximum(h, 0.0)
    return h


def rqvae_forward(x, enc_layers, codebooks, dec_layers, beta, codes=None):
    """Whole RQ-VAE forward in float64 given (or searching) the codes:
    returns (loss, recon, rq_loss, codes, x_hat)."""
    z = mlp(x, enc_layers)
    if codes is None:
        codes = rq_assign(z.astype(np.float32), codebooks)[0]
    cb = np.asarray(codebooks, np.float64)
    q = np.zeros_like(z)
    for lvl in range(cb.shape[0]):
        q = q + cb[lvl][codes[:, lvl]]
    x_hat = mlp(q, dec_layers)              # straight-through: decoder sees the quantised latent
    recon = np.mean((x_hat - np.asarray(x, np.float64)) ** 2)
    rql = rq_loss(z, codebooks, codes, beta)
    return recon + rql, recon, rql, codes, x_hat


def semantic_feature_ids(codes, codebook_size):
    """Semantic ids as 1-based item_sparse feature values (0 = padding, as the
    reference's feature tables reserve row 0: BaseLineO1/model.py:271-280 sizes
    each table feat_statistics[k] + 1)."""
    return np.asarray(codes, np.int64) + 1


def dedup_level(codes):
    """TIGER's collision level (restated with a dict walk in item order): the
    extra code of item i = how many earlier items share its code tuple."""
    codes = np.asarray(codes, np.int64)
    seen = {}
    extra = np.zeros(len(codes), np.int64)
    for i, row in enumerate(map(tuple, codes)):
        extra[i] = seen.get(row, 0)
        seen[row] = extra[i] + 1
    return np.concatenate([codes, extra[:, None]], 1)


def kmeans_init(z, codebook_size, iters, seed=0):
    """Lloyd k-means on float32 rows (codebook initialisation, level by level
    on the residuals).  Assignment uses ``rq_assign`` with one level; the
    update is the float64 mean of the assigned rows; empty clusters keep their
    centre.  Initial centres: rows chosen by a seeded permutation."""
    z = np.asarray(z, np.float32)
    rng = np.random.default_rng(seed)
    cent = z[rng.permutation(z.shape[0])[:codebook_size]].copy()
    for _ in range(iters):
        k = rq_assign(z, cent[None])[0][:, 0]
        sums = np.zeros((codebook_size, z.shape[1]), np.float64)
        np.add.at(sums, k, z.astype(np.float64))
        cnt = np.bincount(k, minlength=codebook_size)
        nz = cnt > 0
        cent[nz] = (sums[nz] / cnt[nz, None]).astype(np.float32)
    return cent
