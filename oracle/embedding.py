"""Embedding-table oracle (numpy).  TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py.

Restates the arithmetic of the reference's table lookups:

* plain gather   -- ``self.item_emb(...)`` / ``self.user_emb(...)`` /
  ``self.sparse_emb[k](t)`` / ``self.pos_emb(poss)``
  (``model/BaseLine/model.py:242-247,275,328``;
  ``model/BaseLineO1/model.py:345-350,380,439``);
* bag-sum        -- ``self.sparse_emb[k](t).sum(2)`` for array features
  (``model/BaseLine/model.py:277``; ``model/BaseLineO1/model.py:383``):
  left-to-right sequential accumulation over the array slots;
* dense backward -- autograd's ``embedding_dense_backward`` of the calls above
  with ``padding_idx=0`` (``model/BaseLine/model.py:115-117,159-165``):
  per table row, sequential fp32 accumulation in occurrence order
  (flattened index order), padding row excluded.

All three are pinned against torch-CPU outputs of the reference's own
modules in ``tests/golden/emb_ops.npz``.
"""
from __future__ import annotations

import numpy as np

_BF16_MASK = np.uint32(0xFFFF0000)


def to_bf16_f32(x: np.ndarray) -> np.ndarray:
    """Round fp32 -> bf16 (round-to-nearest-even) and return it as fp32."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    u = x.view(np.uint32).astype(np.uint64)
    rounded = ((u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000).astype(np.uint32)
    out = rounded.view(np.float32).copy()
    nan = np.isnan(x)
    out[nan] = np.float32(np.nan)
    return out


def gather(table: np.ndarray, idx: np.ndarray) -> np.ndarray:
    """``table[idx]`` -- bit-exact row copy (model/BaseLine/model.py:242-247)."""
    return table[np.asarray(idx, dtype=np.int64)]


def bag_sum(table: np.ndarray, idx: np.ndarray, out_bf16: bool = False) -> np.ndarray:
    """Sum over the last index axis, slot 0 first (model/BaseLine/model.py:277).

    Accumulates in fp32, left to right; ``out_bf16`` rounds the fp32 sum once
    to bf16 (what the bf16-table kernel does).
    """
    idx = np.asarray(idx, dtype=np.int64)
    rows = table[idx].astype(np.float32)  # [..., A, D]
    acc = rows[..., 0, :].copy()
    for a in range(1, rows.shape[-2]):
        acc = acc + rows[..., a, :]
    return to_bf16_f32(acc) if out_bf16 else acc


def dense_backward(grad: np.ndarray, idx: np.ndarray, num_rows: int,
                   padding_idx: int | None = 0) -> np.ndarray:
    """Dense table gradient of a lookup (autograd of model/BaseLine/model.py:242-277).

    ``grad`` has shape ``idx.shape + (D,)``.  Rows are accumulated in fp32 in
    flattened occurrence order; ``np.add.at`` is unbuffered and applies the
    updates strictly in index order, which is exactly that order.
    """
    idx = np.asarray(idx, dtype=np.int64).reshape(-1)
    g = np.asarray(grad, dtype=np.float32).reshape(idx.shape[0], -1)
    out = np.zeros((num_rows, g.shape[1]), dtype=np.float32)
    keep = idx != padding_idx if padding_idx is not None else np.ones_like(idx, bool)
    np.add.at(out, idx[keep], g[keep])
    return out


def chunked_backward(grad: np.ndarray, idx: np.ndarray, num_rows: int, padding_idx: int | None = 0,
                     chunk: int = 256) -> np.ndarray:
    """The fixed chunk order of grk_embedding_backward(GRK_BWD_CHUNKED) -- no
    reference counterpart (used only for intermediates such as the fused
    trainer's projected feature rows, whose reference gradient is dE = sum dY W).

    Occurrences are stably sorted by row (padding dropped) and cut into
    ``chunk``-entry chunks; each (row, chunk) piece is summed in occurrence
    order from zero, and a row's pieces are added in chunk order.
    """
    idx = np.asarray(idx, dtype=np.int64).reshape(-1)
    g = np.asarray(grad, dtype=np.float32).reshape(idx.shape[0], -1)
    keep = idx != padding_idx if padding_idx is not None else np.ones_like(idx, bool)
    idx, g = idx[keep], g[keep]
    order = np.argsort(idx, kind='stable')
    keys, rows = idx[order], g[order]
    n = len(keys)
    out = np.zeros((num_rows, g.shape[1]), dtype=np.float32)
    if n == 0:
        return out
    piece_key = keys * ((n + chunk - 1) // chunk) + np.arange(n) // chunk
    heads = np.concatenate([[True], piece_key[1:] != piece_key[:-1]])
    pid = np.cumsum(heads) - 1
    pieces = np.zeros((int(pid[-1]) + 1, g.shape[1]), dtype=np.float32)
    np.add.at(pieces, pid, rows)
    np.add.at(out, keys[heads], pieces)
    return out


def multi_source_backward(sources, num_rows: int, padding_idx: int | None = 0) -> np.ndarray:
    """Sum of several lookups of ONE table (item table: seq, pos, neg calls).

    ``sources`` is a list of ``(grad, idx)``.  Occurrence order runs over the
    sources in list order, then flattened index order.  The reference's
    autograd sums the per-call dense grads instead, so against the full
    model this matches to rounding only (SURVEY.md §7 hard part 4).
    """
    idx = np.concatenate([np.asarray(i, dtype=np.int64).reshape(-1) for _, i in sources])
    g = np.concatenate([np.asarray(gr, dtype=np.float32).reshape(np.asarray(i).size, -1)
                        for gr, i in sources])
    return dense_backward(g, idx, num_rows, padding_idx)


def unique_rows(idx: np.ndarray, padding_idx: int | None = 0):
    """Sorted unique non-padding ids of a lookup (row-sparse gradient layout)."""
    idx = np.asarray(idx, dtype=np.int64).reshape(-1)
    if padding_idx is not None:
        idx = idx[idx != padding_idx]
    return np.unique(idx)
