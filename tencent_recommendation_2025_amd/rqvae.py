"""RQ-VAE semantic-ID tokenizer for config 4 (BASELINE.json configs[3]:
"model/BaseLineO1 + RQ-VAE semantic-ID tokenizer, d=512").

The reference has no tokenizer.  What it defines is where the
semantic ids go: each one is an extra ``item_sparse`` feature of the O1 model
(``BaseLineO1/model.py:271-280`` builds a table per item_sparse feature sized
``feat_statistics[k] + 1``, ``:355`` looks them up with the other item
features), computed from the items' multimodal embeddings (``mm_emb``, loaded by
``BaseLineO1/dataset.py:535-567``).  The tokenizer follows the published RQ-VAE
(Lee et al. 2022; TIGER, Rajput et al. 2023): encoder MLP -> ``levels``-level
residual quantiser over ``codebook_size`` codes -> decoder MLP, trained on
MSE(x_hat, x) + sum_l ||sg(r_l) - c_l||^2 + beta ||r_l - sg(c_l)||^2 with the
straight-through estimator.

MI355X path:
* the code search (argmin over every code of every level, the O(n*L*K*d)
  part) is ``grk_rq_assign`` (csrc/grk_rqvae.hip): exact fp32 VALU distances
  in a fixed order, bit-identical to ``oracle/rqvae.py``;
* the selected codewords come back through ``_CodebookRows``, whose backward
  is the deterministic scatter-add of the embedding backward
  (``grk_embedding_backward``, bit-exact sequential fp32 per code), so a
  training step is run-to-run reproducible;
* encoder / decoder are plain ``nn.Linear`` (hipBLASLt GEMMs through torch).
There is no CPU path for the kernels: they raise without the HIP library
(`dedup_level` and the id-table helpers are integer torch glue, any device).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib as L
from . import kernels as K


def rq_assign(z, codebooks, want_quant=True, want_dist=False, want_resid=False):
    """grk_rq_assign: codes int32 [n, levels] (+ quant [n, d], dist [n, levels],
    resid [n, d] fp32 when asked).  z fp32 [n, d], codebooks fp32 [levels, K, d]."""
    K._require_cuda(z, codebooks)
    if z.dtype != torch.float32 or codebooks.dtype != torch.float32:
        raise L.GrkError('rq_assign takes fp32 latents and codebooks')
    if z.dim() != 2 or codebooks.dim() != 3 or codebooks.shape[2] != z.shape[1]:
        raise L.GrkError('z [n, d] and codebooks [levels, codes, d] must share d')
    if z.stride(1) != 1 or z.stride(0) % 4 or z.data_ptr() % 16:
        z = z.contiguous()
    codebooks = codebooks.contiguous()
    n, d = z.shape
    lv, kc, _ = codebooks.shape
    dev = z.device
    codes = torch.empty(n, lv, dtype=torch.int32, device=dev)
    quant = torch.empty(n, d, dtype=torch.float32, device=dev) if want_quant else None
    dist = torch.empty(n, lv, dtype=torch.float32, device=dev) if want_dist else None
    resid = torch.empty(n, d, dtype=torch.float32, device=dev) if want_resid else None
    rc = L.lib().grk_rq_assign(z.data_ptr(), z.stride(0), codebooks.data_ptr(), n, d, kc, lv, codes.data_ptr(),
                               K._ptr(quant), K._ptr(dist), K._ptr(resid), L.stream_ptr(dev))
    L.check(rc, 'grk_rq_assign')
    return codes, quant, dist, resid


class _CodebookRows(torch.autograd.Function):
    """rows[n, l] = codebooks[l, codes[n, l]]; backward = deterministic
    scatter-add of the row gradients into the codebooks (grk_embedding_backward
    over the flattened [levels * K, d] table, no padding row)."""

    @staticmethod
    def forward(ctx, codebooks, codes):
        lv, kc, d = codebooks.shape
        flat = (codes.long() + torch.arange(lv, device=codes.device) * kc).reshape(-1)
        ctx.save_for_backward(flat)
        ctx.shape = (lv, kc, d)
        return codebooks.reshape(lv * kc, d).index_select(0, flat).view(codes.shape[0], lv, d)

    @staticmethod
    def backward(ctx, grad):
        (flat,) = ctx.saved_tensors
        lv, kc, d = ctx.shape
        g = grad.reshape(-1, d).float().contiguous()
        res = K.embedding_backward([K.GradSource(idx=flat, grad=g, grad_col=0)], lv * kc, d, padding_idx=None)
        return res.dense.view(lv, kc, d), None


def _mlp(dims):
    layers = []
    for i in range(len(dims) - 1):
        layers.append(torch.nn.Linear(dims[i], dims[i + 1]))
        if i + 2 < len(dims):
            layers.append(torch.nn.ReLU())
    return torch.nn.Sequential(*layers)


class RQVAE(torch.nn.Module):
    """Encoder MLP -> residual quantiser -> decoder MLP.

    ``forward(x)`` returns ``(x_hat, codes, losses)`` with ``losses`` a dict of
    ``loss`` (the training objective), ``recon`` and ``rq``.  ``tokenize(x)``
    returns the codes only (inference, no decoder)."""

    def __init__(self, in_dim, hidden=(512, 256), latent_dim=64, levels=3, codebook_size=256, beta=0.25):
        super().__init__()
        if latent_dim not in (16, 32, 64, 128):
            raise ValueError('latent_dim must be 16, 32, 64 or 128 (grk_rq_assign)')
        self.in_dim, self.latent_dim = in_dim, latent_dim
        self.levels, self.codebook_size, self.beta = levels, codebook_size, beta
        self.encoder = _mlp([in_dim, *hidden, latent_dim])
        self.decoder = _mlp([latent_dim, *reversed(hidden), in_dim])
        self.codebooks = torch.nn.Parameter(torch.randn(levels, codebook_size, latent_dim) * (latent_dim ** -0.5))

    def encode(self, x):
        return self.encoder(x.float())

    def quantize(self, z):
        """codes [n, L], codeword rows [n, L, d] (differentiable w.r.t. the
        codebooks), and the residuals r_l [n, L, d] (r_0 = z) the loss uses."""
        codes = rq_assign(z.detach(), self.codebooks.detach(), want_quant=False)[0]
        rows = _CodebookRows.apply(self.codebooks, codes)
        prev = torch.cumsum(rows.detach(), 1) - rows.detach()
        resid = z.unsqueeze(1) - prev
        return codes, rows, resid

    def forward(self, x):
        x = x.float()
        z = self.encode(x)
        codes, rows, resid = self.quantize(z)
        quant = rows.detach().sum(1)
        zq = z + (quant - z).detach()                       # straight-through
        x_hat = self.decoder(zq)
        recon = F.mse_loss(x_hat, x)
        codebook = ((resid.detach() - rows) ** 2).mean(dim=(0, 2)).sum()
        commit = ((resid - rows.detach()) ** 2).mean(dim=(0, 2)).sum()
        rq = codebook + self.beta * commit
        return x_hat, codes, {'loss': recon + rq, 'recon': recon, 'rq': rq}

    @torch.no_grad()
    def init_codebooks(self, x, iters=10, seed=0):
        """k-means initialisation, level by level on the residuals of a sample
        (rows of x); assignment by grk_rq_assign, centres = exact means via a
        one-hot GEMM in fp64 (deterministic)."""
        z = self.encode(x).float()
        g = torch.Generator(device='cpu').manual_seed(seed)
        r = z
        for lvl in range(self.levels):
            n = r.shape[0]
            if n < self.codebook_size:
                raise ValueError('k-means init needs at least codebook_size rows')
            cent = r[torch.randperm(n, generator=g)[:self.codebook_size].to(r.device)].clone()
            for _ in range(iters):
                k = rq_assign(r, cent[None], want_quant=False)[0][:, 0].long()
                onehot = F.one_hot(k, self.codebook_size).double()
                sums = onehot.T @ r.double()
                cnt = onehot.sum(0)
                nz = cnt > 0
                cent[nz] = (sums[nz] / cnt[nz, None]).float()
            self.codebooks[lvl].copy_(cent)
            k = rq_assign(r, cent[None], want_quant=False)[0][:, 0].long()
            r = r - cent[k]

    @torch.no_grad()
    def tokenize(self, x, batch=65536):
        """Semantic ids of every row of x: int32 [n, levels] codes."""
        out = []
        for i in range(0, x.shape[0], batch):
            z = self.encode(x[i:i + batch])
            out.append(rq_assign(z, self.codebooks, want_quant=False)[0])
        return torch.cat(out) if out else torch.empty(0, self.levels, dtype=torch.int32, device=x.device)


def dedup_level(codes):
    """TIGER's collision level: an extra code per item that makes every
    item's code tuple unique -- the item's rank (in item order) among the
    items sharing its tuple.  codes int [n, L] -> int64 [n, L + 1]; the extra
    level's cardinality is the largest collision group (``int(out[:, -1].max()) + 1``).
    Integer work on n x L codes: a stable sort of the packed tuples and a
    rank-in-run (torch ops on the codes' device, deterministic)."""
    n, lv = codes.shape
    c = codes.long()
    if n == 0:
        return torch.empty(0, lv + 1, dtype=torch.int64, device=codes.device)
    # dense tuple ids: lexicographic rank of each row's tuple (no overflow for any K, L)
    _, tid = torch.unique(c, dim=0, return_inverse=True)
    order = torch.sort(tid, stable=True).indices          # items grouped by tuple, item order inside
    st = tid[order]
    pos = torch.arange(n, device=codes.device)
    head = torch.ones(n, dtype=torch.bool, device=codes.device)
    head[1:] = st[1:] != st[:-1]
    first = torch.cummax(torch.where(head, pos, torch.zeros_like(pos)), 0).values
    rank = torch.empty(n, dtype=torch.int64, device=codes.device)
    rank[order] = pos - first
    return torch.cat([c, rank[:, None]], 1)


def semantic_id_table(codes, num_items):
    """Per-item semantic-id feature rows for the O1 model: int64
    [num_items + 1, levels], row i = codes of item i + 1 (feature values are
    1-based: row 0 of each item_sparse table is padding), row 0 = 0.
    ``codes`` [num_items, levels] holds items 1..num_items in order."""
    lv = codes.shape[1]
    t = torch.zeros(num_items + 1, lv, dtype=torch.int64, device=codes.device)
    t[1:] = codes.long() + 1
    return t


def semantic_id_schema(levels, codebook_size=None, prefix='sid', codes=None):
    """Feature names and statistics the semantic ids add to the O1 model's
    ``item_sparse`` features (the model sizes each table feat_statistics[k] + 1,
    BaseLineO1/model.py:271-280).

    ``codes`` (int [n, levels], 0-based -- e.g. ``dedup_level`` output, whose
    collision level can exceed the codebook size): per-level cardinalities
    ``codes[:, l].max() + 1``, so every 1-based id of semantic_id_table(codes)
    has its table row.  Without codes every level gets ``codebook_size``."""
    if codes is not None:
        c = torch.as_tensor(codes)
        levels = c.shape[1]
        card = [int(c[:, lvl].max()) + 1 if c.shape[0] else 1 for lvl in range(levels)]
        if codebook_size is not None:
            card = [max(k, int(codebook_size)) for k in card]
    elif codebook_size is None:
        raise ValueError('semantic_id_schema needs codebook_size or codes')
    else:
        card = [int(codebook_size)] * levels
    names = [f'{prefix}{lvl}' for lvl in range(levels)]
    return names, dict(zip(names, card))
