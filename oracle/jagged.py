"""CPU oracle of the jagged (valid-token) batch layout -- TEST INFRASTRUCTURE ONLY
(imported by tests/ and never by the product path).

Restates grk_jagged_layout / grk_gather_rows (tencent_recommendation_2025_amd/
csrc/grk_jagged.hip) in numpy.  The reference has no such layout: it runs every
token-wise op over the left-padded [B, T] batch (model/BaseLine/model.py:
331-350, 379-384).  What pins it to the reference is the padded step itself:
the tests check that the jagged step computes the same logits, loss and
gradients as the padded one (the rows it drops are the padding rows before
each sequence's first valid token: no key of any query, logits masked).
"""
import numpy as np


def layout(key_valid, capacity):
    """(ranges int32 [B, 3] cols 0-1, row_base int64 [B], row_map int32 [capacity], n)
    of a [B, T] key-validity array: span of b = [start_b, T), start_b = first valid
    position (T if none); spans packed in b order.  A capacity below the span rows
    drops the trailing spans that do not fit (grk_jagged_layout, err bit 2)."""
    kv = np.asarray(key_valid) != 0
    B, T = kv.shape
    start = np.where(kv.any(1), kv.argmax(1), T)
    contig = np.array([kv[b, start[b]:].all() for b in range(B)], np.int32)
    span = T - start
    incl = np.cumsum(span)
    # spans ending past the capacity are dropped (start T, row_base -T; err bit 2)
    drop = incl > capacity
    start = np.where(drop, T, start)
    contig = np.where(drop, 1, contig).astype(np.int32)
    span = np.where(drop, 0, span)
    base = np.concatenate([[0], np.cumsum(span)[:-1]]).astype(np.int64)
    n = int(span.sum())
    row_map = np.full(capacity, -1, np.int32)
    for b in range(B):
        for t in range(start[b], T):
            row_map[base[b] + t - start[b]] = b * T + t
    row_base = np.where(drop, -T, base - start).astype(np.int64)
    return np.stack([start, contig], 1).astype(np.int32), row_base, row_map, n


def gather_rows(src, row_map):
    """dst[r] = src.reshape(B*T, ...)[row_map[r]], zeros where row_map[r] < 0."""
    s = np.asarray(src)
    flat = s.reshape(-1, *s.shape[2:]) if s.ndim >= 2 else s
    out = np.zeros((len(row_map),) + flat.shape[1:], flat.dtype)
    ok = row_map >= 0
    out[ok] = flat[row_map[ok]]
    return out
