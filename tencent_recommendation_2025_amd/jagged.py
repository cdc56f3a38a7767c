"""Jagged (valid-token) training batches.

The reference left-pads every sequence to T = maxlen + 1 and runs each
token-wise op -- lookups, itemdnn / userdnn, the attention blocks, LayerNorms,
logits -- over all B*T rows (model/BaseLine/model.py:331-350, 379-384).  A row
before its sequence's first valid token is dead: it is no key of any query
(the key-padding half of log2feats' mask), its logits are masked
(next_token_type != 1), so it adds nothing to the loss and every gradient it
would carry is an exact zero.  At BASELINE config 2 (lengths U{32..201}) those
rows are ~47 % of the batch.

``layout(batch, capacity)`` packs each sequence's span [start_b, T) back to
back (grk_jagged_layout) and ``compact(batch, jag)`` copies every per-token
tensor of the batch (ids, token types, feature ids, mm rows, positions) into
that order in one launch (grk_gather_rows).  The fused trainer then runs the
whole token-wise step on ``capacity`` rows (a multiple of ``quantum`` >= the
batch's span rows; the rows past them are dead padding: zero ids, no loss
term).  The attention kernels address token (b, t) as row ``row_base[b] + t``;
key validity, timestamps and the softmax statistics stay [B, T].

The host needs the span-row count to pick the capacity (GEMM shapes and the
captured HIP graph depend on it): ``span_rows(token_type)`` reads it from a CPU
batch for free, and from a device batch with one host sync (the bench computes
it once per pooled batch).
"""
from __future__ import annotations

import torch

from . import kernels as K


class Jagged:
    """Layout of one batch: B, T, capacity and the device index tensors."""
    __slots__ = ('B', 'T', 'capacity', 'key_valid', 'seq_range', 'row_base', 'row_map', 'n', 'err')

    def __init__(self, B, T, capacity, key_valid, seq_range, row_base, row_map, n, err):
        self.B, self.T, self.capacity = B, T, capacity
        self.key_valid, self.seq_range, self.row_base, self.row_map, self.n, self.err = \
            key_valid, seq_range, row_base, row_map, n, err


def span_rows(token_type):
    """Host count of the span rows sum_b (T - first valid position of b) of a [B, T]
    token_type / key-valid tensor (a host sync when it lives on the device)."""
    kv = (token_type != 0)
    T = kv.shape[1]
    first = torch.where(kv.any(1), kv.to(torch.int8).argmax(1), torch.full_like(kv[:, 0], T, dtype=torch.int64))
    return int((T - first).sum().item())


JAGGED_ERRORS = {1: 'a labelled token (next_token_type == 1) lies before its sequence\'s first valid token '
                    'or in a dropped span',
                 2: 'the batch holds more span rows than the jagged capacity (rows under-stated): '
                    'trailing sequences were dropped'}


def check_error(err):
    """Raise ValueError when a layout error flag (int32 [1], host sync) is set."""
    v = int(err.item())
    if v:
        raise ValueError('jagged layout: ' + '; '.join(m for bit, m in JAGGED_ERRORS.items() if v & bit))


def capacity_for(n, quantum=1024, limit=None):
    """Rows of the jagged step for n span rows: n rounded up to a multiple of quantum
    (a few distinct shapes = a few GEMM plans and captured graphs), at most ``limit``."""
    cap = max(quantum, -(-int(n) // quantum) * quantum)
    return min(cap, limit) if limit is not None else cap


def layout(token_type, capacity, next_token_type=None, err=None):
    """The jagged layout of a batch with token_type [B, T] (0 = padding) in `capacity` rows.

    ``err`` (optional int32 [1] device tensor, OR-ed into, never cleared; a fresh
    zero flag otherwise): bit 1 -- a labelled token (next_token_type == 1) outside
    the kept spans; bit 2 -- the spans hold more than ``capacity`` rows, so the
    trailing spans were dropped (never addressed past the capacity)."""
    kv = (token_type != 0).contiguous().view(torch.uint8)   # bool bytes are 0 / 1: no cast kernel
    B, T = kv.shape
    if err is None:
        err = torch.zeros(1, dtype=torch.int32, device=kv.device)
    ranges, row_base, row_map, n = K.jagged_layout(kv, capacity, next_token_type, err)
    return Jagged(B, T, int(capacity), kv, ranges, row_base, row_map, n, err)


def _as_rows(t, N):
    """A [B, T, ...] tensor viewed as [B*T, ...] contiguous rows."""
    t = t if t.is_contiguous() else t.contiguous()
    return t.reshape(N, *t.shape[2:])


_POSITIONS = {}


def _positions(T, device):
    """Cached int64 [1, T] = 1 .. T on the device."""
    key = (int(T), str(device))
    t = _POSITIONS.get(key)
    if t is None:
        t = _POSITIONS[key] = torch.arange(1, T + 1, dtype=torch.int64).unsqueeze(0).to(device)
    return t


def compact(batch, jag, with_positions=True):
    """The batch's per-token tensors in the jagged row order, as [1, capacity, ...]
    tensors (one grk_gather_rows launch for all of them): (seq, pos, neg, tt, ntt, nat,
    seq_feat, pos_feat, neg_feat) and, with_positions, the position-embedding index
    (t + 1 where seq != 0, model/BaseLine/model.py:326-328) as an 11th field.  A
    10th field (event times) stays [B, T]: the attention kernels read it per (b, t).
    pos / neg ids and each pos / neg feature of one shape land in the two halves of
    one buffer (model.feat2emb_pair stacks them without a copy)."""
    B, T, cap = jag.B, jag.T, jag.capacity
    N = B * T
    pairs, out = [], []

    def source(t):
        src = _as_rows(t, N)
        if src.dtype == torch.bool or src.element_size() * (src[0].numel() if src.dim() > 1 else 1) % 4:
            src = src.to(torch.int32)
        return src

    def take(t, dst=None):
        if t is None:
            return None
        src = source(t)
        if dst is None:
            dst = torch.empty((cap,) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
        pairs.append((src, dst))
        return dst.unsqueeze(0)

    def take_pair(a, b):
        """Two tensors of one shape and dtype into the halves of ONE [2 cap, ...] buffer:
        the model's pos / neg stacking (feat2emb_pair) is then a view, not a copy."""
        if a is None or b is None:
            return take(a), take(b)
        sa, sb = source(a), source(b)
        if sa.dtype != sb.dtype or sa.shape[1:] != sb.shape[1:]:
            return take(a), take(b)
        buf = torch.empty((2 * cap,) + tuple(sa.shape[1:]), dtype=sa.dtype, device=sa.device)
        pairs.append((sa, buf[:cap]))
        pairs.append((sb, buf[cap:]))
        return buf[:cap].unsqueeze(0), buf[cap:].unsqueeze(0)

    seq_o = take(batch[0])
    pos_o, neg_o = take_pair(batch[1], batch[2])
    out += [seq_o, pos_o, neg_o] + [take(x) for x in batch[3:6]]
    sf, pf, nf = batch[6:9]
    out.append(None if sf is None else {k: take(v) for k, v in sf.items()})
    if pf is not None and nf is not None:
        po, no = {}, {}
        for k, v in pf.items():
            if k in nf:
                po[k], no[k] = take_pair(v, nf[k])
            else:
                po[k] = take(v)
        for k, v in nf.items():
            if k not in no:
                no[k] = take(v)
        out += [po, no]
    else:
        out += [None if f is None else {k: take(v) for k, v in f.items()} for f in (pf, nf)]
    out.append(batch[9] if len(batch) > 9 else None)
    if with_positions:
        seq = batch[0]
        pidx = torch.where(seq != 0, _positions(T, seq.device), 0)
        out.append(take(pidx))
    K.gather_rows(pairs, jag.row_map)
    return tuple(out)
