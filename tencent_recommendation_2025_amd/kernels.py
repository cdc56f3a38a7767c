"""Thin torch-facing wrappers over the libgrk.so C ABI (include/grk.h).

Each function validates shapes on the host, passes raw device pointers and
torch's current HIP stream, and raises ``GrkError`` on any failure.  There is
no CPU / eager fallback: these functions require CUDA(HIP) tensors and the
built library.
"""
from __future__ import annotations

import ctypes as C
import math
import os
from dataclasses import dataclass

import torch

from . import _lib as L


def _ptr(t):
    return None if t is None else t.data_ptr()


def _require_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise L.GrkError('grk kernels need device (HIP) tensors; there is no CPU path')


@dataclass
class Lookup:
    """One table lookup feeding a fused gather (see grk_feature / grk_lookup).

    ``idx`` is ``[..., bag]`` when ``bag > 1`` (array feature) else ``[...]``;
    tokens are the leading dims flattened (``n = b*T + t``).
    """
    table: torch.Tensor
    idx: torch.Tensor
    out_col: int
    mode: int = L.IDX_PLAIN
    bag: int = 1
    skip_row0: bool = False   # row 0 is a zero padding row: bag slots on it are not read

    def idx_ld(self):
        return self.bag


def _idx_contig(idx, bag):
    idx = idx if idx.is_contiguous() else idx.contiguous()
    n = idx.numel() // bag
    return idx, n


def embedding_gather(lookups, out, num_tokens, token_type=None, seq_len=0, err_flag=None):
    """out[n, col:col+D] = sum_a table[row(n, a)]  for every lookup (grk_embedding_gather)."""
    if not lookups:
        return out
    if len(lookups) > L.MAX_FEATURES:
        raise L.GrkError(f'at most {L.MAX_FEATURES} features per gather call')
    dim = lookups[0].table.shape[1]
    dt = lookups[0].table.dtype
    it = lookups[0].idx.dtype
    _require_cuda(out, token_type, err_flag, *[lk.table for lk in lookups])
    if out.dtype != dt or out.dim() != 2 or out.stride(1) != 1:
        raise L.GrkError('out must be a row-major [N, ld] tensor of the table dtype')
    feats = (L.GrkFeature * len(lookups))()
    keep = []
    for i, lk in enumerate(lookups):
        if lk.table.shape[1] != dim or lk.table.dtype != dt or lk.idx.dtype != it:
            raise L.GrkError('all lookups of one call share dim, table dtype and index dtype')
        if not lk.table.is_contiguous():
            raise L.GrkError('tables must be contiguous')
        idx, n = _idx_contig(lk.idx, lk.bag)
        if n != num_tokens:
            raise L.GrkError(f'lookup {i}: {n} tokens, expected {num_tokens}')
        keep.append(idx)
        feats[i] = L.GrkFeature(lk.table.data_ptr(), idx.data_ptr(), lk.table.shape[0], lk.bag, lk.bag,
                                lk.out_col, lk.mode, L.FEAT_SKIP_ROW0 if lk.skip_row0 else 0)
    if token_type is not None:
        token_type = token_type.to(torch.int32).contiguous()
        keep.append(token_type)
    rc = L.lib().grk_embedding_gather(feats, len(lookups), dim, L.dtype_code(dt), L.itype_code(it), num_tokens,
                                      _ptr(token_type), seq_len, out.data_ptr(), out.stride(0), _ptr(err_flag),
                                      L.stream_ptr(out.device))
    L.check(rc, 'grk_embedding_gather')
    return out


@dataclass
class GradSource:
    """One lookup's upstream gradient for a table (grk_lookup).

    ``row_offset``/``table_rows`` place the lookup's table inside a table
    group (several tables in one flat buffer); -1 rows = the whole group."""
    idx: torch.Tensor
    grad: torch.Tensor      # [N, ld]
    grad_col: int
    mode: int = L.IDX_PLAIN
    bag: int = 1
    row_offset: int = 0
    table_rows: int = -1


class BackwardResult:
    __slots__ = ('dense', 'ids', 'rows', 'count', 'capacity')

    def __init__(self, dense, ids, rows, count, capacity):
        self.dense, self.ids, self.rows, self.count, self.capacity = dense, ids, rows, count, capacity


BACKWARD_TRACE = None  # bench.py: a list records the embedding_backward calls of one eager step


def embedding_backward(sources, num_rows, dim, padding_idx=0, token_type=None, seq_len=0, dense=True,
                       sparse=False, row_slot=None, err_flag=None, chunked=False, dense_dtype=torch.float32):
    """Deterministic scatter-add table gradient (grk_embedding_backward).

    Returns a ``BackwardResult`` with ``dense`` ([num_rows, dim] fp32) when
    ``dense`` and ``ids``/``rows``/``count`` (row-sparse form, capacity =
    number of occurrences) when ``sparse``.  ``chunked``: rows spanning several
    chunks of the sorted occurrences are added chunk-sum by chunk-sum
    (GRK_BWD_CHUNKED; fixed order, not the occurrence order).  ``dense_dtype``
    bfloat16 (chunked, bf16 gradients, dim 512): the dense rows rounded to bf16
    once in the kernel (GRK_BWD_DENSE_BF16).
    """
    if BACKWARD_TRACE is not None:
        BACKWARD_TRACE.append(dict(sources=list(sources), num_rows=num_rows, dim=dim, padding_idx=padding_idx,
                                   token_type=token_type, seq_len=seq_len, dense=dense, sparse=sparse,
                                   row_slot=None if row_slot is None else row_slot.clone(), chunked=chunked,
                                   dense_dtype=dense_dtype))
    dev = sources[0].grad.device
    gdt = sources[0].grad.dtype
    it = sources[0].idx.dtype
    _require_cuda(*[s.grad for s in sources], token_type, row_slot, err_flag)
    lk = (L.GrkLookup * len(sources))()
    keep = []
    total = 0
    for i, s in enumerate(sources):
        if s.grad.dtype != gdt or s.idx.dtype != it:
            raise L.GrkError('all sources of one table share grad dtype and index dtype')
        if s.grad.stride(-1) != 1 or s.grad.dim() != 2:
            raise L.GrkError('grad must be a row-major [N, ld] tensor')
        idx, n = _idx_contig(s.idx, s.bag)
        if n != s.grad.shape[0]:
            raise L.GrkError(f'source {i}: {n} index tokens vs {s.grad.shape[0]} grad rows')
        if s.grad_col + dim > s.grad.shape[1]:
            raise L.GrkError(f'source {i}: grad_col out of range')
        keep.append(idx)
        rows = num_rows - s.row_offset if s.table_rows < 0 else s.table_rows
        lk[i] = L.GrkLookup(idx.data_ptr() if n else None, s.grad.data_ptr() if n else None, n, s.bag,
                            s.grad.stride(0), s.row_offset, rows, s.bag, s.grad_col, s.mode, 0)
        total += n * s.bag
    if token_type is not None:
        token_type = token_type.to(torch.int32).contiguous()
        keep.append(token_type)
    ws_bytes = L.lib().grk_embedding_backward_workspace(total, num_rows, dim)
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    if dense_dtype not in (torch.float32, torch.bfloat16):
        raise L.GrkError(f'dense gradient dtype {dense_dtype} is neither fp32 nor bf16')
    bf16_out = dense and dense_dtype == torch.bfloat16
    if bf16_out and not (chunked and gdt == torch.bfloat16 and dim == 512):
        raise L.GrkError('a bf16 dense gradient needs chunked=True with bf16 gradients of 512 columns')
    dense_out = torch.empty((num_rows, dim), dtype=torch.bfloat16 if bf16_out else torch.float32,
                            device=dev) if dense else None
    cap = max(total, 1)
    ids = torch.empty(cap, dtype=torch.int64, device=dev) if sparse else None
    rows = torch.empty((cap, dim), dtype=torch.float32, device=dev) if sparse else None
    count = torch.empty(1, dtype=torch.int32, device=dev)
    rc = L.lib().grk_embedding_backward(lk, len(sources), dim, L.dtype_code(gdt), L.itype_code(it),
                                        _ptr(token_type), seq_len, num_rows, -1 if padding_idx is None else padding_idx,
                                        _ptr(dense_out), _ptr(ids), _ptr(rows), count.data_ptr(), _ptr(row_slot),
                                        (L.BWD_CHUNKED if chunked else L.BWD_ORDERED) | (L.BWD_DENSE_BF16 if bf16_out else 0),
                                        ws.data_ptr(), ws.numel(),
                                        _ptr(err_flag), L.stream_ptr(dev))
    L.check(rc, 'grk_embedding_backward')
    return BackwardResult(dense_out, ids, rows, count, cap)


def chunked_size():
    """Chunk length of the GRK_BWD_CHUNKED order (a build constant of the
    library: oracle/embedding.chunked_backward restates the order with it)."""
    return int(L.lib().grk_embedding_chunked_size())


def sort_pairs(keys, vals, end_bit=32):
    """grk_sort_pairs: (keys, vals) stably sorted by the low ``end_bit`` bits of
    the keys (uint32 keys as int32, uint64 values as int64 tensors)."""
    _require_cuda(keys, vals)
    if keys.dtype != torch.int32 or vals.dtype != torch.int64 or keys.dim() != 1 or vals.shape != keys.shape:
        raise L.GrkError('sort_pairs takes int32 keys and int64 values of the same length')
    keys, vals = keys.contiguous(), vals.contiguous()
    n = keys.numel()
    ko, vo = torch.empty_like(keys), torch.empty_like(vals)
    kt, vt = torch.empty_like(keys), torch.empty_like(vals)
    wsb = L.lib().grk_sort_pairs_workspace(n)
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=keys.device)
    L.check(L.lib().grk_sort_pairs(_ptr(keys), _ptr(vals), _ptr(ko), _ptr(vo), _ptr(kt), _ptr(vt), n, int(end_bit),
                                   ws.data_ptr(), ws.numel(), L.stream_ptr(keys.device)), 'grk_sort_pairs')
    return ko, vo


def adamw_hparams(lr, beta1, beta2, eps, weight_decay, step):
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    return L.GrkAdamwHparams(lr, beta1, beta2, eps, weight_decay, lr / bc1, math.sqrt(bc2), 0.0)


class DeviceClock:
    """The optimizer step in device memory plus a ring of per-step hyper-parameters.

    Passed where a ``GrkAdamwHparams`` (hp) or an int step (t) is expected, the
    table kernels read the step from ``t`` at execution time and the
    hyper-parameters from ``ring[t % ring_len]`` (the ``*_dev`` entry points):
    a launch captured once in a HIP graph then does the right step on every
    replay.  ``advance()`` (t += 1) is itself a device op, captured with the
    step.  The owner keeps the ring filled for the steps ahead."""

    def __init__(self, ring_len, device):
        nf = C.sizeof(L.GrkAdamwHparams) // 4
        self.ring_len = int(ring_len)
        self.ring = torch.zeros(self.ring_len, nf, dtype=torch.float32, device=device)
        self.t = torch.zeros(1, dtype=torch.int32, device=device)

    def advance(self):
        self.t.add_(1)


def table_adamw(param, exp_avg, exp_avg_sq, hp, ids=None, rows=None, count=None, capacity=0, row_slot=None,
                lazy=False):
    """AdamW update of one table from a row-sparse gradient (grk_table_adamw / _dev when hp is a DeviceClock)."""
    _require_cuda(param, exp_avg, exp_avg_sq, ids, rows, count, row_slot)
    if exp_avg.dtype != torch.float32 or exp_avg_sq.dtype != torch.float32:
        raise L.GrkError('optimizer moments must be float32')
    if not (param.is_contiguous() and exp_avg.is_contiguous() and exp_avg_sq.is_contiguous()):
        raise L.GrkError('param and moments must be contiguous')
    args = (param.data_ptr(), L.dtype_code(param.dtype), exp_avg.data_ptr(), exp_avg_sq.data_ptr(), param.shape[0],
            param.shape[1], _ptr(ids), _ptr(rows), _ptr(count), capacity, _ptr(row_slot))
    mode = L.ADAM_LAZY if lazy else L.ADAM_DENSE
    if isinstance(hp, DeviceClock):
        rc = L.lib().grk_table_adamw_dev(*args, hp.ring.data_ptr(), hp.ring_len, hp.t.data_ptr(), mode,
                                         L.stream_ptr(param.device))
    else:
        rc = L.lib().grk_table_adamw(*args, hp, mode, L.stream_ptr(param.device))
    L.check(rc, 'grk_table_adamw')


MAX_GRAD_RANGES = 64   # kMaxGradRanges (csrc/grk_optim.hip)


def table_adamw_ranges(param, exp_avg, exp_avg_sq, clock, ranges, shadow=None):
    """Dense-parity AdamW of a whole table from dense gradient blocks in ONE launch
    (grk_table_adamw_ranges_dev): ranges = [(row_offset, grad [rows, >= D] bf16/fp32)],
    other rows g = 0.  shadow (bf16, param's shape, fp32 param only): also receives
    the updated parameters rounded to bf16."""
    launch_prepared(prepare_table_adamw_ranges(param, exp_avg, exp_avg_sq, clock, ranges, shadow))


def prepare_table_adamw_ranges(param, exp_avg, exp_avg_sq, clock, ranges, shadow=None):
    """The checked arguments of one table_adamw_ranges launch (a PreparedCall):
    launch_prepared() runs it on the current stream.  A caller whose tensors keep
    their storage from step to step (optim.DenseFlat) builds it once -- the ctypes
    range array is most of the host cost of a launch with dozens of ranges."""
    _require_cuda(param, exp_avg, exp_avg_sq, *[g for _, g in ranges])
    if shadow is not None and (shadow.dtype != torch.bfloat16 or shadow.shape != param.shape
                               or not shadow.is_contiguous() or param.dtype != torch.float32):
        raise L.GrkError('shadow: a contiguous bf16 tensor of an fp32 param\'s shape')
    rows, D = param.shape
    if len(ranges) > MAX_GRAD_RANGES:
        raise L.GrkError(f'at most {MAX_GRAD_RANGES} gradient ranges per launch, got {len(ranges)}')
    if not (param.is_contiguous() and exp_avg.is_contiguous() and exp_avg_sq.is_contiguous()):
        raise L.GrkError('param and moments must be contiguous')
    rs = sorted(ranges, key=lambda r: r[0])
    arr = (L.GrkGradRange * max(1, len(rs)))()
    for i, (off, g) in enumerate(rs):
        if g.dim() != 2 or g.stride(1) != 1 or g.shape[1] < D:
            raise L.GrkError(f'range {i}: grad must be a row-major [n, >= {D}] matrix')
        if g.dtype == torch.float32 and (g.data_ptr() % 16 or g.stride(0) % 4):
            # k_adamw_ranges reads fp32 gradient rows as 16-byte vectors
            raise L.GrkError(f'range {i}: fp32 grad rows must be 16-byte aligned')
        arr[i] = L.GrkGradRange(int(off), int(off) + g.shape[0], g.data_ptr(), g.stride(0), L.dtype_code(g.dtype), 0)
    args = (param.data_ptr(), L.dtype_code(param.dtype), exp_avg.data_ptr(), exp_avg_sq.data_ptr(), rows, D, arr,
            len(rs), clock.ring.data_ptr(), clock.ring_len, clock.t.data_ptr(),
            None if shadow is None else shadow.data_ptr())
    # the gradients are not kept: a caller reusing the call checks that its gradients
    # still live at these addresses (optim.DenseFlat's key), and holding them would keep
    # a whole extra set of dense gradients alive between eager steps
    return PreparedCall('grk_table_adamw_ranges_dev', args, param.device,
                        (param, exp_avg, exp_avg_sq, clock.ring, clock.t, shadow))


@dataclass
class PreparedCall:
    """A grk entry point and its arguments but the stream (appended at launch);
    ``keep`` holds the long-lived tensors the pointers refer to."""
    name: str
    args: tuple
    device: torch.device
    keep: tuple


def launch_prepared(call):
    rc = getattr(L.lib(), call.name)(*call.args, L.stream_ptr(call.device))
    L.check(rc, call.name)


def table_l2_norm(param, l2, norm=None, coef=None):
    """(norm fp32 [1], l2 / norm fp32 [1]) of a whole table (grk_table_l2_norm):
    the l2_emb term's value and gradient scale, on the device."""
    _require_cuda(param, norm, coef)
    if not param.is_contiguous() or param.data_ptr() % 16:
        raise L.GrkError('param must be contiguous and 16-byte aligned')
    dev = param.device
    norm = torch.empty(1, dtype=torch.float32, device=dev) if norm is None else norm
    coef = torch.empty(1, dtype=torch.float32, device=dev) if coef is None else coef
    ws = torch.empty(L.lib().grk_table_l2_norm_workspace(), dtype=torch.uint8, device=dev)
    rc = L.lib().grk_table_l2_norm(param.data_ptr(), L.dtype_code(param.dtype), param.shape[0], param.shape[1],
                                   float(l2), norm.data_ptr(), coef.data_ptr(), ws.data_ptr(), ws.numel(),
                                   L.stream_ptr(dev))
    L.check(rc, 'grk_table_l2_norm')
    return norm, coef


def table_adamw_l2(param, exp_avg, exp_avg_sq, clock, l2_coef, ids=None, rows=None, count=None, capacity=0,
                   row_slot=None):
    """Dense-mode table AdamW with every row's gradient + l2_coef * p (grk_table_adamw_l2_dev)."""
    _require_cuda(param, exp_avg, exp_avg_sq, ids, rows, count, row_slot, l2_coef)
    if not (param.is_contiguous() and exp_avg.is_contiguous() and exp_avg_sq.is_contiguous()):
        raise L.GrkError('param and moments must be contiguous')
    rc = L.lib().grk_table_adamw_l2_dev(param.data_ptr(), L.dtype_code(param.dtype), exp_avg.data_ptr(),
                                        exp_avg_sq.data_ptr(), param.shape[0], param.shape[1], _ptr(ids), _ptr(rows),
                                        _ptr(count), capacity, _ptr(row_slot), clock.ring.data_ptr(), clock.ring_len,
                                        clock.t.data_ptr(), l2_coef.data_ptr(), L.stream_ptr(param.device))
    L.check(rc, 'grk_table_adamw_l2_dev')


# ------------------------------------------------------------------ attention
def _col_view_ok(t, name, dtypes=(torch.bfloat16,)):
    if t.dim() != 2 or t.stride(1) != 1 or t.dtype not in dtypes:
        raise L.GrkError(f'{name} must be a {"/".join(str(d)[6:] for d in dtypes)} [B*T, >=H*hd] row-major view')
    if t.stride(0) % 8 or t.data_ptr() % 16:
        raise L.GrkError(f'{name}: row stride must be a multiple of 8 and the view 16-byte aligned')


def table_adamw_dense(param, exp_avg, exp_avg_sq, hp, grad):
    """AdamW of every row of `param` (a [rows, D] table or row range of one) from a dense
    gradient (fp32 or bf16, [rows, >= D] row-major) -- grk_table_adamw_dense."""
    _require_cuda(param, exp_avg, exp_avg_sq, grad)
    rows, D = param.shape
    for t, n in ((param, 'param'), (exp_avg, 'exp_avg'), (exp_avg_sq, 'exp_avg_sq')):
        if t.shape != (rows, D) or not t.is_contiguous():
            raise L.GrkError(f'{n} must be a contiguous [{rows}, {D}] tensor')
    if grad.dim() != 2 or grad.shape[0] != rows or grad.shape[1] < D or grad.stride(1) != 1:
        raise L.GrkError(f'grad must be a row-major [{rows}, >= {D}] tensor')
    args = (param.data_ptr(), L.dtype_code(param.dtype), exp_avg.data_ptr(), exp_avg_sq.data_ptr(), rows, D,
            grad.data_ptr(), L.dtype_code(grad.dtype), grad.stride(0))
    if isinstance(hp, DeviceClock):
        rc = L.lib().grk_table_adamw_dense_dev(*args, hp.ring.data_ptr(), hp.ring_len, hp.t.data_ptr(),
                                               L.stream_ptr(param.device))
    else:
        rc = L.lib().grk_table_adamw_dense(*args, hp, L.stream_ptr(param.device))
    L.check(rc, 'grk_table_adamw_dense')


def table_adamw_catchup(param, exp_avg, exp_avg_sq, last, hp_ring, t, ids=None):
    """Replay the skipped g = 0 steps (last[row], t] of rows `ids` (all rows if None) --
    grk_table_adamw_catchup.  hp_ring: uint8/float tensor holding grk_adamw_hparams[ring_len];
    t: an int, or a DeviceClock (its step and ring; hp_ring is then ignored)."""
    if isinstance(t, DeviceClock):
        hp_ring = t.ring
    _require_cuda(param, exp_avg, exp_avg_sq, last, hp_ring, ids)
    rows, D = param.shape
    if last.dtype != torch.int32 or last.shape != (rows,):
        raise L.GrkError('last must be an int32 [rows] tensor')
    ring_len = hp_ring.numel() * hp_ring.element_size() // C.sizeof(L.GrkAdamwHparams)
    n = 0
    if ids is not None:
        if ids.dtype != torch.int64 or not ids.is_contiguous():
            raise L.GrkError('ids must be a contiguous int64 tensor')
        n = ids.numel()
    args = (param.data_ptr(), L.dtype_code(param.dtype), exp_avg.data_ptr(), exp_avg_sq.data_ptr(), rows, D,
            last.data_ptr(), _ptr(ids), n, hp_ring.data_ptr(), ring_len)
    if isinstance(t, DeviceClock):
        rc = L.lib().grk_table_adamw_catchup_dev(*args, t.t.data_ptr(), L.stream_ptr(param.device))
    else:
        rc = L.lib().grk_table_adamw_catchup(*args, int(t), L.stream_ptr(param.device))
    L.check(rc, 'grk_table_adamw_catchup')


def table_adamw_catchup_slice(param, exp_avg, exp_avg_sq, last, clock, num_slices):
    """Rolling flush (grk_table_adamw_catchup_slice_dev): bring slice (clock.t mod
    num_slices) of the rows up to the clock's step -- one launch per step, its slice
    read on the device, so a captured step replays the right slice every time."""
    _require_cuda(param, exp_avg, exp_avg_sq, last)
    rows, D = param.shape
    if last.dtype != torch.int32 or last.shape != (rows,):
        raise L.GrkError('last must be an int32 [rows] tensor')
    rc = L.lib().grk_table_adamw_catchup_slice_dev(param.data_ptr(), L.dtype_code(param.dtype), exp_avg.data_ptr(),
                                                   exp_avg_sq.data_ptr(), rows, D, last.data_ptr(), clock.ring.data_ptr(),
                                                   clock.ring_len, clock.t.data_ptr(), int(num_slices),
                                                   L.stream_ptr(param.device))
    L.check(rc, 'grk_table_adamw_catchup_slice')


def stamp_rows(last, ids, count, capacity, t):
    """last[ids[:count]] = t (grk_stamp_rows; t may be a DeviceClock)."""
    _require_cuda(last, ids, count)
    if isinstance(t, DeviceClock):
        rc = L.lib().grk_stamp_rows_dev(last.data_ptr(), ids.data_ptr(), count.data_ptr(), int(capacity),
                                        t.t.data_ptr(), L.stream_ptr(last.device))
    else:
        rc = L.lib().grk_stamp_rows(last.data_ptr(), ids.data_ptr(), count.data_ptr(), int(capacity), int(t),
                                    L.stream_ptr(last.device))
    L.check(rc, 'grk_stamp_rows')


def _seed_parts(seed):
    """(host seed, device seed tensor or None) of a dropout seed given as an int or an int64 [1] device tensor."""
    if isinstance(seed, torch.Tensor):
        if seed.dtype != torch.int64 or seed.numel() != 1 or not seed.is_cuda:
            raise L.GrkError('a device dropout seed must be an int64 [1] tensor on the GPU')
        return 0, seed
    return int(seed) & (2 ** 64 - 1), None


def attn_args(kind, q, k, v, B, T, H, hd, key_valid=None, scale=None, rab=None, inv_n=1.0, dropout_p=0.0, seed=0,
              precise=True, out_dtype=torch.bfloat16, act=None, seq_range=None, timestamps=None, rab_t=None,
              row_base=None):
    """Build grk_attn_args for bf16 [B*T, ld] column views q/k/v (head h at cols h*hd).

    act="silu": q/k/v are pre-activations; SiLU is applied on load and the
    backward's dq/dk/dv are gradients w.r.t. the pre-activations.
    seq_range: optional int32 [B, 3] from seq_ranges(key_valid) (computed once per step).
    seed: an int, or a device int64 [1] tensor the kernels read when they run
    (drawn on the device each step, so a graph-replayed step gets a fresh mask).
    precise: 0 / False (P and dS rounded to bf16), 1 / True (P, dS as bf16 hi + lo),
    2 (fp32 fidelity: Q/K/V and dO split into hi + lo as well; q/k/v may then be
    fp32 / fp16 / bf16 and are read exactly -- fidelity_supported(T, hd)).
    timestamps (int64 [B, T]) + rab_t (fp32 [H, nbt], nbt <= 64): the HSTU time
    bias rab_t[h, time_bucket(t_q - t_k)] (include/grk.h, grk_attn_args).
    row_base (int64 [B + 1], with seq_range -- jagged_layout): the jagged layout --
    q/k/v (and every output / gradient) hold only each sequence's span [start_b, T),
    token (b, t) at row row_base[b] + t; row_base[B] = n, the span rows: output rows
    [n, q.shape[0]) are zeroed.  key_valid / timestamps stay [B, T].
    float8_e4m3fn q/k/v (precise 0 / 1, act None; head_dim 64 / 128): the fp8
    attention of config C5 -- QK^T on the fp8 MFMA, the rest on bf16 MFMA over
    the exactly widened values."""
    precise = int(precise)
    if precise not in (0, 1, 2):
        raise L.GrkError('precise must be 0, 1 or 2')
    f8 = q.dtype == torch.float8_e4m3fn
    if precise == 2:
        dts = (torch.bfloat16, torch.float32, torch.float16)
    else:
        dts = (torch.float8_e4m3fn,) if f8 else (torch.bfloat16,)
    for t, n in ((q, 'q'), (k, 'k'), (v, 'v')):
        _col_view_ok(t, n, dts)
        if (row_base is None and t.shape[0] != B * T) or t.shape[1] < H * hd:
            raise L.GrkError(f'{n}: shape {tuple(t.shape)} does not fit B*T={B * T}, H*hd={H * hd}')
    if row_base is not None:
        if seq_range is None or row_base.dtype != torch.int64 or row_base.shape != (B + 1,) \
                or not row_base.is_contiguous():
            raise L.GrkError('row_base must be a contiguous int64 [B + 1] tensor, with seq_range (jagged_layout)')
    if not q.dtype == k.dtype == v.dtype:
        raise L.GrkError('q, k and v must share a dtype')
    if f8 and act is not None:
        raise L.GrkError('fp8 q/k/v hold activations: act must be None')
    if key_valid is not None:
        if key_valid.dtype != torch.uint8 or key_valid.shape != (B, T) or not key_valid.is_contiguous():
            raise L.GrkError('key_valid must be a contiguous uint8 [B, T] tensor')
    nb = 0
    if seq_range is not None and (seq_range.dtype != torch.int32 or seq_range.shape != (B, 3)
                                  or not seq_range.is_contiguous()):
        raise L.GrkError('seq_range must be a contiguous int32 [B, 3] tensor (kernels.seq_ranges)')
    if kind == L.ATTN_HSTU:
        if rab is None or rab.dtype != torch.float32 or rab.dim() != 2 or rab.shape[0] != H or not rab.is_contiguous():
            raise L.GrkError('hstu needs a contiguous fp32 rab [H, num_buckets]')
        nb = rab.shape[1]
    nbt = 0
    if timestamps is not None or rab_t is not None:
        if kind != L.ATTN_HSTU or timestamps is None or rab_t is None:
            raise L.GrkError('the time bias is an HSTU feature and needs both timestamps and rab_t')
        if timestamps.dtype != torch.int64 or timestamps.shape != (B, T) or not timestamps.is_contiguous():
            raise L.GrkError('timestamps must be a contiguous int64 [B, T] tensor')
        if rab_t.dtype != torch.float32 or rab_t.dim() != 2 or rab_t.shape[0] != H or not rab_t.is_contiguous():
            raise L.GrkError('rab_t must be a contiguous fp32 [H, num_time_buckets] tensor')
        nbt = rab_t.shape[1]
    if scale is None:
        scale = hd ** -0.5
    seed, seed_dev = _seed_parts(seed)
    args = L.GrkAttnArgs(kind, B, H, T, hd, nb, q.data_ptr(), k.data_ptr(), v.data_ptr(), q.stride(0), k.stride(0),
                         v.stride(0), _ptr(key_valid), _ptr(rab), float(scale), float(inv_n), float(dropout_p),
                         precise, seed, L.dtype_code(out_dtype),
                         {None: L.ACT_NONE, 'silu': L.ACT_SILU}[act], _ptr(seq_range), _ptr(seed_dev),
                         L.GRK_FP8_E4M3 if f8 else L.dtype_code(q.dtype), _ptr(timestamps), _ptr(rab_t), nbt, None,
                         None, _ptr(row_base), None if row_base is None else row_base.data_ptr() + 8 * B,
                         q.shape[0] if row_base is not None else 0)
    args._keep = (q, k, v, key_valid, rab, seq_range, seed_dev, timestamps, rab_t, row_base)  # raw pointers: keep alive
    return args


def fidelity_supported(seq_len, head_dim):
    """Whether the fp32-fidelity attention (precise=2) runs for this shape (whole-sequence kernels' LDS)."""
    return bool(L.lib().grk_attention_fidelity_supported(int(seq_len), int(head_dim)))


def seq_ranges(key_valid):
    """int32 [B, 3]: (first valid key, contiguous flag) per sequence and, in column 2,
    the sequences longest first (grk_seq_ranges)."""
    _require_cuda(key_valid)
    if key_valid.dtype != torch.uint8 or key_valid.dim() != 2 or not key_valid.is_contiguous():
        raise L.GrkError('key_valid must be a contiguous uint8 [B, T] tensor')
    B, T = key_valid.shape
    out = torch.empty(B, 3, dtype=torch.int32, device=key_valid.device)
    rc = L.lib().grk_seq_ranges(key_valid.data_ptr() if B else None, B, T, out.data_ptr() if B else None,
                                L.stream_ptr(key_valid.device))
    L.check(rc, 'grk_seq_ranges')
    return out


def jagged_layout(key_valid, capacity, next_token_type=None, err_flag=None):
    """The jagged (valid-token) layout of a left-padded batch (grk_jagged_layout):
    (seq_range int32 [B, 3], row_base int64 [B + 1], row_map int32 [capacity], n int64 [1]
    = a view of row_base[B]) -- device tensors, no host sync.  Row r of the layout
    holds token row_map[r] (= b * T + t, t in the span [start_b, T)), -1 past the n
    span rows; token (b, t) is row row_base[b] + t."""
    _require_cuda(key_valid, next_token_type, err_flag)
    if key_valid.dtype != torch.uint8 or key_valid.dim() != 2 or not key_valid.is_contiguous():
        raise L.GrkError('key_valid must be a contiguous uint8 [B, T] tensor')
    B, T = key_valid.shape
    dev = key_valid.device
    ranges = torch.empty(B, 3, dtype=torch.int32, device=dev)
    row_base = torch.empty(B + 1, dtype=torch.int64, device=dev)
    row_map = torch.empty(int(capacity), dtype=torch.int32, device=dev)
    n = row_base[B:]
    ntt = None if next_token_type is None else next_token_type.to(torch.int32).contiguous()
    rc = L.lib().grk_jagged_layout(key_valid.data_ptr(), B, T, int(capacity), _ptr(ntt), ranges.data_ptr(),
                                   row_base.data_ptr(), row_map.data_ptr(), n.data_ptr(), _ptr(err_flag),
                                   L.stream_ptr(dev))
    L.check(rc, 'grk_jagged_layout')
    return ranges, row_base, row_map, n


MAX_COLUMN_BLOCKS = 16   # kMaxColumnBlocks (csrc/grk_index.hip)


def write_columns(out, blocks):
    """out[:, col:col + w] = x for every (col, x) in blocks (grk_write_columns, one launch):
    x fp32 / bf16 [rows, w] with unit column stride, or [1, w] broadcast to every row;
    out bf16 / fp32 [rows, ld] row-major.  Blocks in column order, disjoint."""
    if not blocks:
        return out
    if len(blocks) > MAX_COLUMN_BLOCKS:
        raise L.GrkError(f'at most {MAX_COLUMN_BLOCKS} column blocks per launch')
    _require_cuda(out, *[x for _, x in blocks])
    if out.dim() != 2 or out.stride(1) != 1 or out.dtype not in (torch.float32, torch.bfloat16):
        raise L.GrkError('out must be a row-major [rows, ld] fp32 / bf16 tensor')
    rows = out.shape[0]
    arr = (L.GrkColumnBlock * len(blocks))()
    keep = []
    for k, (col, x) in enumerate(sorted(blocks, key=lambda b: b[0])):
        x = x.detach()
        if x.dtype not in (torch.float32, torch.bfloat16):
            x = x.float()
        if x.dim() != 2 or x.stride(1) != 1:
            x = x.reshape(x.shape[0], -1).contiguous()
        if x.shape[0] not in (1, rows):
            raise L.GrkError(f'column block {k}: {x.shape[0]} rows, expected 1 or {rows}')
        keep.append(x)
        ld = 0 if x.shape[0] == 1 and rows != 1 else x.stride(0)
        arr[k] = L.GrkColumnBlock(x.data_ptr(), ld, x.shape[1], int(col), L.dtype_code(x.dtype), 0)
    L.check(L.lib().grk_write_columns(arr, len(blocks), rows, out.data_ptr(), out.stride(0), L.dtype_code(out.dtype),
                                      L.stream_ptr(out.device)), 'grk_write_columns')
    return out


def proj_index(blocks, rows, out=None):
    """int64 [rows, sum of widths]: column block k = blocks[k] = (src [rows, w] int, offset)
    with every non-zero value shifted by offset, 0 kept (grk_proj_index, one launch):
    the projected tables' bag index of the fused model (model._proj_index)."""
    if not blocks:
        raise L.GrkError('proj_index needs at least one block')
    _require_cuda(*[b for b, _ in blocks], out)
    itype = blocks[0][0].dtype
    if itype not in (torch.int32, torch.int64) or any(b.dtype != itype for b, _ in blocks):
        raise L.GrkError('proj_index blocks must share one int32 / int64 dtype')
    arr = (L.GrkIndexBlock * len(blocks))()
    col = 0
    for k, (b, off) in enumerate(blocks):
        b2 = b.reshape(rows, -1)
        if b2.stride(-1) != 1:
            raise L.GrkError(f'proj_index block {k}: rows must be contiguous')
        arr[k] = L.GrkIndexBlock(b2.data_ptr(), b2.stride(0), b2.shape[1], col, int(off))
        col += b2.shape[1]
    if out is None:
        out = torch.empty(rows, col, dtype=torch.int64, device=blocks[0][0].device)
    if out.dtype != torch.int64 or out.dim() != 2 or out.shape[0] != rows or out.shape[1] < col or out.stride(1) != 1:
        raise L.GrkError('proj_index out must be an int64 [rows, >= columns] row-major tensor')
    L.check(L.lib().grk_proj_index(arr, len(blocks), 1 if itype == torch.int64 else 0, rows, out.data_ptr(),
                                   out.stride(0), L.stream_ptr(out.device)), 'grk_proj_index')
    return out


def batch_row_ids(seq, pos, neg, token_type, with_user=True):
    """(item ids int64 [3n] = item tokens' ids | pos | neg, user ids int64 [n] or None), -1 for
    padding (grk_batch_row_ids, one launch): the table rows a batch reads."""
    _require_cuda(seq, pos, neg, token_type)
    ts = [t.contiguous() for t in (seq, pos, neg, token_type)]
    dt = ts[0].dtype
    if dt not in (torch.int32, torch.int64):
        raise L.GrkError('batch_row_ids: int32 / int64 ids')
    ts = [t if t.dtype == dt else t.to(dt) for t in ts]
    n = ts[0].numel()
    if any(t.numel() != n for t in ts):
        raise L.GrkError('batch_row_ids: seq, pos, neg and token_type must have one shape')
    item = torch.empty(3 * n, dtype=torch.int64, device=seq.device)
    user = torch.empty(n, dtype=torch.int64, device=seq.device) if with_user else None
    L.check(L.lib().grk_batch_row_ids(*[t.data_ptr() for t in ts], 1 if dt == torch.int64 else 0, n,
                                      item.data_ptr(), _ptr(user), L.stream_ptr(seq.device)), 'grk_batch_row_ids')
    return item, user


MAX_ROW_COPIES = 64   # kMaxRowCopies (csrc/grk_jagged.hip)


def gather_rows(pairs, row_map):
    """dst[r] = src[row_map[r]] (zeros where row_map[r] < 0) for every (src, dst) pair
    in ONE launch (grk_gather_rows): src [N, ...] and dst [rows, ...] of one dtype with
    contiguous rows of the same width (any trailing shape)."""
    if not pairs:
        return
    rows = row_map.numel()
    _require_cuda(row_map, *[t for pr in pairs for t in pr])
    if row_map.dtype != torch.int32 or not row_map.is_contiguous():
        raise L.GrkError('row_map must be a contiguous int32 tensor')
    for i in range(0, len(pairs), MAX_ROW_COPIES):
        chunk = pairs[i:i + MAX_ROW_COPIES]
        cps = (L.GrkRowCopy * len(chunk))()
        for j, (src, dst) in enumerate(chunk):
            if src.dtype != dst.dtype or dst.shape[0] != rows or src.shape[1:] != dst.shape[1:]:
                raise L.GrkError(f'gather_rows pair {i + j}: src {tuple(src.shape)} {src.dtype} vs dst '
                                 f'{tuple(dst.shape)} {dst.dtype} ({rows} rows)')
            if not (src.is_contiguous() and dst.is_contiguous()):
                raise L.GrkError(f'gather_rows pair {i + j}: tensors must be contiguous')
            rb = src[0].numel() * src.element_size() if src.dim() > 1 else src.element_size()
            if rb % 4:
                raise L.GrkError(f'gather_rows pair {i + j}: a row of {rb} bytes (multiple of 4 required)')
            cps[j] = L.GrkRowCopy(src.data_ptr(), dst.data_ptr(), rb, rb, rb)
        L.check(L.lib().grk_gather_rows(cps, len(chunk), row_map.data_ptr(), rows, L.stream_ptr(row_map.device)),
                'grk_gather_rows')


_ROUTE_WS = {}


def route(ids, world, rows_per_owner, global_rows):
    """Routing plan of one row-sharded table's ids (grk_route, five launches, no sort):
    {'send_ids': int64 [n] (distinct ids, owner-major (owner = id % world), ascending
    within an owner, in the first n_uniq slots), 'inverse': int64 [n] (each id's slot,
    -1 for ids outside the table), 'send_counts': int64 [world], 'n_uniq': int64 [1],
    'bad': int64 [1] (ids outside [0, global_rows))} -- sharding.ShardExchange.route's
    plan; the caller's all-to-all of the counts completes it."""
    _require_cuda(ids)
    ids = ids.reshape(-1)
    if ids.dtype != torch.int64:
        ids = ids.long()
    ids = ids.contiguous()
    dev, n = ids.device, ids.numel()
    key = (dev, int(world), int(rows_per_owner))
    ws = _ROUTE_WS.get(key)
    if ws is None:
        ws = _ROUTE_WS[key] = torch.empty(max(L.lib().grk_route_workspace(world, rows_per_owner), 1),
                                          dtype=torch.uint8, device=dev)
    out = dict(send_ids=torch.empty(n, dtype=torch.int64, device=dev),
               inverse=torch.empty(n, dtype=torch.int64, device=dev),
               send_counts=torch.empty(world, dtype=torch.int64, device=dev),
               n_uniq=torch.empty(1, dtype=torch.int64, device=dev),
               bad=torch.empty(1, dtype=torch.int64, device=dev))
    L.check(L.lib().grk_route(_ptr(ids), n, int(world), int(rows_per_owner), int(global_rows), _ptr(out['send_ids']),
                              _ptr(out['inverse']), _ptr(out['send_counts']), _ptr(out['n_uniq']), _ptr(out['bad']),
                              ws.data_ptr(), ws.numel(), L.stream_ptr(dev)), 'grk_route')
    return out


MAX_PACK_RANGES = 64   # kPackMax (csrc/grk_shard.hip)


def flat_pack(dst, parts):
    """dst (fp32, contiguous) [off:off + n] = src (bf16 / fp32, any shape, contiguous) or
    zeros for src None, for every (src, off, n) in parts -- grk_flat_pack, one launch
    per 64 parts (an all-reduce bucket's gradients into its flat buffer)."""
    _require_cuda(dst)
    if dst.dtype != torch.float32 or not dst.is_contiguous():
        raise L.GrkError('flat_pack: dst must be a contiguous fp32 tensor')
    keep = []
    for i in range(0, len(parts), MAX_PACK_RANGES):
        chunk = parts[i:i + MAX_PACK_RANGES]
        arr = (L.GrkPackRange * len(chunk))()
        for j, (src, off, n) in enumerate(chunk):
            if off < 0 or off + n > dst.numel():
                raise L.GrkError(f'flat_pack part {i + j}: [{off}, {off + n}) outside dst ({dst.numel()})')
            if src is None:
                arr[j] = L.GrkPackRange(None, n, off, L.GRK_F32, 0)
                continue
            if src.dtype not in (torch.float32, torch.bfloat16):
                src = src.float()
            src = src.contiguous()
            if src.numel() != n:
                raise L.GrkError(f'flat_pack part {i + j}: {src.numel()} elements, expected {n}')
            keep.append(src)
            arr[j] = L.GrkPackRange(src.data_ptr(), n, off, L.dtype_code(src.dtype), 0)
        L.check(L.lib().grk_flat_pack(arr, len(chunk), dst.data_ptr(), L.stream_ptr(dst.device)), 'grk_flat_pack')
    return dst


def jagged_remap(roles, row_map):
    """[out int64 [rows] per role] with out[r] = inv[row_map[r]] and, for a dead row
    (row_map < 0), inv at the role's first padding position (grk_jagged_remap, one
    launch): roles = [(inv int64 [n], ids int64 [n], tt int64 [n] or None, tt_want)],
    a role's id at i being ids[i], or 0 where tt[i] != tt_want."""
    if not roles:
        return []
    if len(roles) > 8:
        raise L.GrkError('jagged_remap: at most 8 roles per launch')
    _require_cuda(row_map)
    if row_map.dtype != torch.int32 or not row_map.is_contiguous():
        raise L.GrkError('row_map must be a contiguous int32 tensor')
    rows = row_map.numel()
    arr = (L.GrkRemapRole * len(roles))()
    outs, keep = [], []
    for k, (inv, ids, tt, want) in enumerate(roles):
        inv = inv.reshape(-1).contiguous()
        ids = ids.reshape(-1).long().contiguous()
        if inv.dtype != torch.int64 or ids.numel() != inv.numel() or inv.numel() == 0:
            raise L.GrkError(f'jagged_remap role {k}: int64 inv and ids of one non-zero length')
        if tt is not None:
            tt = tt.reshape(-1).long().contiguous()
            if tt.numel() != ids.numel():
                raise L.GrkError(f'jagged_remap role {k}: tt of {tt.numel()} elements, expected {ids.numel()}')
        out = torch.empty(rows, dtype=torch.int64, device=row_map.device)
        keep += [inv, ids, tt]
        outs.append(out)
        arr[k] = L.GrkRemapRole(inv.data_ptr(), out.data_ptr(), ids.data_ptr(), _ptr(tt), int(want), inv.numel())
    L.check(L.lib().grk_jagged_remap(arr, len(roles), row_map.data_ptr(), rows, L.stream_ptr(row_map.device)),
            'grk_jagged_remap')
    return outs


def attention_fwd(args, out, lse=None):
    """grk_attention_fwd: out [B*T, >=H*hd] (args.out_dtype); lse fp32 [B, H, T] (softmax)."""
    _require_cuda(out, lse)
    if out.stride(1) != 1 or out.stride(0) % 8:
        raise L.GrkError('out must be row-major with a row stride multiple of 8')
    rc = L.lib().grk_attention_fwd(C.byref(args), out.data_ptr(), out.stride(0), _ptr(lse), L.stream_ptr(out.device))
    L.check(rc, 'grk_attention_fwd')


_CLEAN_WS = {}


def _clean_ws(n, device):
    """An int64 [n] scratch that grk leaves zero after every GRK_ATTN_BWD_WS_CLEAN call,
    one per (device, stream, size): zeroed once here, never again per call."""
    key = (str(device), L.stream_ptr(device), int(n))
    t = _CLEAN_WS.get(key)
    if t is None:
        t = _CLEAN_WS[key] = torch.zeros(int(n), dtype=torch.int64, device=device)
    return t


def attention_bwd(args, out, dout, lse, delta, dq, dk, dv, drab=None, parts=L.ATTN_BWD_DQ | L.ATTN_BWD_DKDV,
                  drab_t=None, drab_set=False):
    """grk_attention_bwd(_parts): writes dq/dk/dv (args.out_dtype) and accumulates drab
    (and, with a time bias, drab_t) deterministically.  ``parts`` selects the dq half
    (L.ATTN_BWD_DQ: delta, dq, drab, drab_t) and/or the dk/dv half (L.ATTN_BWD_DKDV);
    tensors of a half not run may be None.  drab_set: drab / drab_t are written, not
    accumulated (no zero fill needed), through this stream's clean fixed-point scratch
    (GRK_ATTN_BWD_WS_CLEAN: no reset launch; the whole-sequence dq kernel's last
    workgroup finalizes them, no finalize launch)."""
    _require_cuda(dout, dq, dk, dv, drab, drab_t)
    clean = bool(drab_set) and drab is not None and bool(parts & L.ATTN_BWD_DQ)
    wst = None
    args.drab_t, args.drab_t_ws = None, None
    if drab_t is not None:
        if args.num_time_buckets == 0 or drab_t.dtype != torch.float32 or not drab_t.is_contiguous() \
                or drab_t.numel() != args.heads * args.num_time_buckets:
            raise L.GrkError('drab_t must be a contiguous fp32 [H, num_time_buckets] tensor of a time-bias call')
        wst = _clean_ws(drab_t.numel(), drab_t.device) if clean else \
            torch.empty(drab_t.numel(), dtype=torch.int64, device=drab_t.device)
        args.drab_t, args.drab_t_ws = drab_t.data_ptr(), wst.data_ptr()
    for t, n in ((dout, 'dout'), (dq, 'dq'), (dk, 'dk'), (dv, 'dv')):
        if t is not None and (t.stride(1) != 1 or t.stride(0) % 8):
            raise L.GrkError(f'{n} must be row-major with a row stride multiple of 8')
    if clean:   # the bins + one counter slot
        ws = _clean_ws(drab.numel() + 1, drab.device)
        parts |= L.ATTN_BWD_WS_CLEAN | L.ATTN_BWD_DRAB_SET
    else:
        ws = None if drab is None or not parts & L.ATTN_BWD_DQ else torch.empty(drab.numel(), dtype=torch.int64,
                                                                                device=drab.device)

    def p_ld(t):
        return (None, 0) if t is None else (t.data_ptr(), t.stride(0))

    (q_p, q_ld), (k_p, k_ld), (v_p, v_ld) = p_ld(dq), p_ld(dk), p_ld(dv)
    rc = L.lib().grk_attention_bwd_parts(C.byref(args), _ptr(out), 0 if out is None else out.stride(0),
                                         dout.data_ptr(), dout.stride(0), L.dtype_code(dout.dtype), _ptr(lse),
                                         _ptr(delta), q_p, q_ld, k_p, k_ld, v_p, v_ld, _ptr(drab), _ptr(ws), parts,
                                         L.stream_ptr(dout.device))
    args.drab_t, args.drab_t_ws = None, None
    L.check(rc, 'grk_attention_bwd')


# ------------------------------------------------------------------ GEMM
def gemm(a, b, trans_a=False, trans_b=False, out=None, out_dtype=torch.bfloat16, alpha=1.0, beta=0.0, bias=None,
         addend=None, relu=False):
    """grk_gemm (hipBLASLt): out[m, n] = alpha op(a) @ op(b) + beta C (+ bias[n]),
    then max(., 0) with relu (grk_gemm_ex's epilogue).

    a, b bf16 row-major 2-D (op = transpose when trans_*); out bf16 or fp32.
    C = ``addend`` (out's dtype and row stride) when given, else ``out``
    itself (accumulate; an allocated out needs beta == 0 or an addend)."""
    _require_cuda(a, b, out, bias)
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16:
        raise L.GrkError('gemm operands must be bf16')
    if a.dim() != 2 or b.dim() != 2 or a.stride(1) != 1 or b.stride(1) != 1:
        raise L.GrkError('gemm operands must be row-major 2-D matrices')
    m, k = (a.shape[1], a.shape[0]) if trans_a else (a.shape[0], a.shape[1])
    kb, n = (b.shape[1], b.shape[0]) if trans_b else (b.shape[0], b.shape[1])
    if kb != k:
        raise L.GrkError(f'gemm inner dimensions differ: {k} vs {kb}')
    if out is None:
        if beta != 0.0 and addend is None:
            raise L.GrkError('beta != 0 needs an output to accumulate into or an addend')
        out = torch.empty(m, n, dtype=addend.dtype if addend is not None else out_dtype, device=a.device)
    elif tuple(out.shape) != (m, n) or out.stride(1) != 1 or out.dtype not in (torch.bfloat16, torch.float32):
        raise L.GrkError(f'gemm output must be a row-major bf16/fp32 [{m}, {n}] matrix')
    if addend is not None and (tuple(addend.shape) != (m, n) or addend.dtype != out.dtype
                               or addend.stride(1) != 1 or addend.stride(0) != out.stride(0)):
        raise L.GrkError("addend must match the output's shape, dtype and row stride")
    if bias is not None and (bias.numel() != n or not bias.is_contiguous()):
        raise L.GrkError(f'bias must be a contiguous vector of {n}')
    rc = L.lib().grk_gemm_ex(int(trans_a), int(trans_b), m, n, k, a.data_ptr(), max(a.stride(0), 1), b.data_ptr(),
                             max(b.stride(0), 1), L.dtype_code(a.dtype), out.data_ptr(), max(out.stride(0), 1),
                             L.dtype_code(out.dtype), _ptr(addend), float(alpha), float(beta), _ptr(bias),
                             L.dtype_code(bias.dtype) if bias is not None else 0,
                             L.GRK_GEMM_EP_RELU if relu else L.GRK_GEMM_EP_NONE, L.stream_ptr(a.device))
    L.check(rc, 'grk_gemm_ex')
    return out


def gemm_mfma(a, b, trans_b=False, out=None, out_dtype=torch.bfloat16, bias=None, c_in=None, relu=False):
    """grk_gemm_mfma directly (grk's MFMA GEMM, whatever grk_gemm would route the shape to):
    out[m, n] = act(a @ op(b) + bias + c_in); a [m, k] bf16 row-major, b [n, k] (trans_b) or
    [k, n] bf16, c_in None or out-shaped (may be out itself)."""
    _require_cuda(a, b, out, bias, c_in)
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16 or a.stride(1) != 1 or b.stride(1) != 1:
        raise L.GrkError('gemm_mfma operands must be bf16 row-major')
    m, k = a.shape
    n = b.shape[0] if trans_b else b.shape[1]
    if (b.shape[1] if trans_b else b.shape[0]) != k:
        raise L.GrkError('gemm_mfma inner dimensions differ')
    if out is None:
        out = torch.empty(m, n, dtype=out_dtype, device=a.device)
    if c_in is not None and (c_in.shape != out.shape or c_in.stride() != out.stride() or c_in.dtype != out.dtype):
        raise L.GrkError("c_in must match the output's shape, strides and dtype")
    rc = L.lib().grk_gemm_mfma(0 if trans_b else 1, m, n, k, a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0),
                               out.data_ptr(), out.stride(0), L.dtype_code(out.dtype), _ptr(c_in), _ptr(bias),
                               L.dtype_code(bias.dtype) if bias is not None else 0,
                               L.GRK_GEMM_EP_RELU if relu else L.GRK_GEMM_EP_NONE, L.stream_ptr(a.device))
    L.check(rc, 'grk_gemm_mfma')
    return out


WGRAD_TRACE = None   # bench.py: a list records the (K, M, N, out_dtype, want_db) of every grk_wgrad call


def wgrad(dy, x, out_dtype=torch.float32, want_db=False):
    """grk_wgrad: (dW = dy^T x [M, N] in out_dtype, db = column sums of dy [M] fp32 or None)
    for dy [K, M] and x [K, N] bf16 row-major (the weight / bias gradients of x @ W^T + b)."""
    _require_cuda(dy, x)
    if WGRAD_TRACE is not None:
        WGRAD_TRACE.append((dy.shape[0], dy.shape[1], x.shape[1], out_dtype, want_db))
    if dy.dtype != torch.bfloat16 or x.dtype != torch.bfloat16 or dy.dim() != 2 or x.dim() != 2:
        raise L.GrkError('wgrad operands must be bf16 2-D matrices')
    if dy.stride(1) != 1 or x.stride(1) != 1 or dy.shape[0] != x.shape[0]:
        raise L.GrkError('wgrad operands must be row-major with the same number of rows')
    k, m = dy.shape
    n = x.shape[1]
    dev = dy.device
    ws = torch.empty(max(L.lib().grk_wgrad_workspace(k, m, n), 16), dtype=torch.uint8, device=dev)
    dw = torch.empty(m, n, dtype=out_dtype, device=dev)
    db = torch.empty(m, dtype=torch.float32, device=dev) if want_db else None
    rc = L.lib().grk_wgrad(dy.data_ptr(), max(dy.stride(0), m), x.data_ptr(), max(x.stride(0), n), k, m, n,
                           dw.data_ptr(), n, L.dtype_code(out_dtype), _ptr(db), ws.data_ptr(), ws.numel(),
                           L.stream_ptr(dev))
    L.check(rc, 'grk_wgrad')
    return dw, db


def _gemm_group_array(groups):
    arr = (L.GrkGemmGroup * len(groups))()
    for i, (a, b, c, rows, b_rows) in enumerate(groups):
        for t, nm in ((a, 'A'), (b, 'B'), (c, 'C')):
            if t.dim() != 2 or t.stride(1) != 1:
                raise L.GrkError(f'group {i}: {nm} must be a 2-D view with unit column stride')
        if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16:
            raise L.GrkError(f'group {i}: A and B must be bf16')
        arr[i] = L.GrkGemmGroup(a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), c.data_ptr(), c.stride(0),
                                int(rows), int(b_rows))
    return arr


def grouped_gemm(groups, n, k, b_layout):
    """grk_grouped_gemm: for each (A [rows, >= k] bf16, B bf16, C [rows, >= n] fp32 / bf16)
    C = A . B^T (b_layout 0, B [n, k]) or A . B (b_layout 1, B [k, n]); views with unit
    column strides (row strides taken from the views).  One launch for every group."""
    if not groups:
        return
    _require_cuda(*[t for g in groups for t in g])
    cdt = {g[2].dtype for g in groups}
    if len(cdt) != 1 or next(iter(cdt)) not in (torch.float32, torch.bfloat16):
        raise L.GrkError('every C must be fp32, or every C bf16')
    for i, (a, b, c) in enumerate(groups):
        kb, nb = (b.shape[1], b.shape[0]) if b_layout == 0 else (b.shape[0], b.shape[1])
        if a.shape[1] < k or kb < k or nb < n or c.shape[1] < n or c.shape[0] != a.shape[0]:
            raise L.GrkError(f'group {i}: shapes do not match n = {n}, k = {k}')
    arr = _gemm_group_array([(a, b, c, a.shape[0], 0) for a, b, c in groups])
    rc = L.lib().grk_grouped_gemm(arr, len(groups), int(b_layout), int(n), int(k),
                                  L.dtype_code(next(iter(cdt))), L.stream_ptr(groups[0][0].device))
    L.check(rc, 'grk_grouped_gemm')


def grouped_wgrad(groups, m, n):
    """grk_grouped_wgrad: for each (A [rows, >= m] bf16, B [>= b_rows, >= n] bf16, C [m, >= n]
    fp32, rows, b_rows) C = A[:rows]^T . B[:rows] with B's rows past b_rows read as its row
    b_rows - 1 (A must be zero there); rows a multiple of 32.  One launch (+ one
    reduction of the split-K slices)."""
    if not groups:
        return
    _require_cuda(*[t for g in groups for t in g[:3]])
    for i, (a, b, c, rows, b_rows) in enumerate(groups):
        if c.dtype != torch.float32 or a.shape[0] < rows or b.shape[0] < b_rows or c.shape[0] != m:
            raise L.GrkError(f'group {i}: C must be fp32 [m, n], A hold rows, B hold b_rows rows')
    arr = _gemm_group_array(groups)
    dev = groups[0][0].device
    nbytes = L.lib().grk_grouped_wgrad_workspace(arr, len(groups), int(m), int(n))
    if nbytes == 0:
        raise L.GrkError('grouped_wgrad: rows must be positive multiples of 32')
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    rc = L.lib().grk_grouped_wgrad(arr, len(groups), int(m), int(n), ws.data_ptr(), ws.numel(), L.stream_ptr(dev))
    L.check(rc, 'grk_grouped_wgrad')


def wgrad_ok(dy, x):
    """Shapes / strides / alignment grk_wgrad takes (else the hipBLASLt GEMM path)."""
    return (dy.dim() == 2 and x.dim() == 2 and dy.shape[1] % 8 == 0 and x.shape[1] % 8 == 0
            and dy.stride(1) == 1 and x.stride(1) == 1 and max(dy.stride(0), dy.shape[1]) % 8 == 0
            and max(x.stride(0), x.shape[1]) % 8 == 0 and dy.data_ptr() % 16 == 0 and x.data_ptr() % 16 == 0)


def mips_topk(queries, items, k, item_ids=None):
    """grk_mips_topk: exact inner-product top-k of every query row over all item rows
    (scores fp32 [Q, k] descending, ids int64 [Q, k]: item_ids[i] (uint64 retrieval
    ids, as an int64 tensor) or the item row index; -1 / -inf past the item count)."""
    _require_cuda(queries, items, item_ids)
    if queries.dtype != items.dtype or queries.dtype not in (torch.float32, torch.bfloat16):
        raise L.GrkError('queries and items must both be fp32 or both bf16')
    if queries.dim() != 2 or items.dim() != 2 or queries.shape[1] != items.shape[1]:
        raise L.GrkError('queries [Q, D] and items [N, D] must share D')
    queries, items = queries.contiguous(), items.contiguous()
    q, d = queries.shape
    n = items.shape[0]
    if item_ids is not None:
        if item_ids.dtype not in (torch.int64, torch.uint64) or item_ids.numel() != n:
            raise L.GrkError('item_ids must be a 64-bit integer tensor with one id per item row')
        item_ids = item_ids.contiguous()
    dev = queries.device
    ws = torch.empty(max(L.lib().grk_mips_topk_workspace(q, n), 16), dtype=torch.uint8, device=dev)
    scores = torch.empty(q, k, dtype=torch.float32, device=dev)
    ids = torch.empty(q, k, dtype=torch.int64, device=dev)
    rc = L.lib().grk_mips_topk(queries.data_ptr(), d, items.data_ptr(), d, L.dtype_code(queries.dtype), q, n, d,
                               int(k), _ptr(item_ids), scores.data_ptr(), ids.data_ptr(), ws.data_ptr(), ws.numel(),
                               L.stream_ptr(dev))
    L.check(rc, 'grk_mips_topk')
    return scores, ids


def gemm_tuning(candidates):
    """grk_gemm_tuning: hipBLASLt candidates timed per new GEMM shape (1 = heuristic pick, no timing)."""
    L.check(L.lib().grk_gemm_tuning(int(candidates)), 'grk_gemm_tuning')


# ------------------------------------------------------------- HSTU gate
def _bf16_rows(t, name, dim):
    if t.dtype != torch.bfloat16 or t.dim() != 2 or t.stride(1) != 1 or t.stride(0) % 8 or t.shape[1] < dim:
        raise L.GrkError(f'{name} must be a bf16 row-major [N, >={dim}] matrix with row stride % 8 == 0')
    if t.data_ptr() % 16:
        raise L.GrkError(f'{name} must be 16-byte aligned')
    return t.data_ptr(), t.stride(0)


def _mat_rows(t, name, dim, dtypes=(torch.bfloat16,)):
    if t.dtype not in dtypes or t.dim() != 2 or t.stride(1) != 1 or t.stride(0) % 8 or t.shape[1] < dim:
        raise L.GrkError(f'{name} must be a row-major [N, >={dim}] matrix of {dtypes} with row stride % 8 == 0')
    return t.data_ptr(), t.stride(0)


def add_norm_fwd(s, y, gamma, beta, eps, x_dtype=torch.bfloat16):
    """grk_add_norm_fwd: s_new = bf16(s + y) (y may be None), x = LayerNorm(s_new) in x_dtype.

    Returns (s_new or None, x, stats fp32 [N, 2])."""
    _require_cuda(s, y, gamma, beta)
    N, D = s.shape[0], gamma.shape[0]
    dev = s.device
    x = torch.empty(N, D, dtype=x_dtype, device=dev)
    stats = torch.empty(N, 2, dtype=torch.float32, device=dev)
    s_new = torch.empty(N, D, dtype=torch.bfloat16, device=dev) if y is not None else None
    (sp, sl), (xp, xl) = _mat_rows(s, 's', D), _mat_rows(x, 'x', D, (torch.bfloat16, torch.float32))
    yp, yl = _mat_rows(y, 'y', D) if y is not None else (None, 0)
    op, ol = _mat_rows(s_new, 's_new', D) if s_new is not None else (None, 0)
    rc = L.lib().grk_add_norm_fwd(sp, sl, yp, yl, gamma.data_ptr(), beta.data_ptr(), float(eps), N, D, op, ol, xp,
                                  xl, L.dtype_code(x_dtype), stats.data_ptr(), L.stream_ptr(dev))
    L.check(rc, 'grk_add_norm_fwd')
    return s_new, x, stats


def add_norm_bwd(gx, gs, s_new, gamma, stats):
    """Gradients of add_norm_fwd: (ds bf16 [N, D] -- for both s and y --, dgamma, dbeta fp32)."""
    _require_cuda(gx, gs, s_new, gamma, stats)
    N, D = s_new.shape[0], gamma.shape[0]
    dev = s_new.device
    ds = torch.empty(N, D, dtype=torch.bfloat16, device=dev)
    dgamma = torch.empty(D, dtype=torch.float32, device=dev)
    dbeta = torch.empty(D, dtype=torch.float32, device=dev)
    ws = torch.empty(max(L.lib().grk_add_norm_bwd_workspace(N, D), 4), dtype=torch.uint8, device=dev)
    (gxp, gxl), (sp, sl), (dp, dl) = (_mat_rows(gx, 'gx', D, (torch.bfloat16, torch.float32)), _mat_rows(s_new, 's_new', D),
                                      _mat_rows(ds, 'ds', D))
    gsp, gsl = _mat_rows(gs, 'gs', D) if gs is not None else (None, 0)
    rc = L.lib().grk_add_norm_bwd(gxp, gxl, L.dtype_code(gx.dtype), gsp, gsl, sp, sl, gamma.data_ptr(),
                                  stats.data_ptr(), N, D, dp, dl, dgamma.data_ptr(), dbeta.data_ptr(), ws.data_ptr(),
                                  ws.numel(), L.stream_ptr(dev))
    L.check(rc, 'grk_add_norm_bwd')
    return ds, dgamma, dbeta


def silu_fp8(pre, out=None):
    """e4m3(SiLU(pre)) of bf16 [N, C] (column view allowed): grk_silu_fp8 (fp32 SiLU,
    round to nearest even, clamped to +-448) -> float8_e4m3fn [N, C]."""
    _require_cuda(pre, out)
    if pre.dtype != torch.bfloat16 or pre.dim() != 2 or pre.stride(1) != 1:
        raise L.GrkError('silu_fp8 takes a row-major bf16 [N, C] (column view)')
    N, C = pre.shape
    if out is None:
        out = torch.empty(N, C, dtype=torch.float8_e4m3fn, device=pre.device)
    L.check(L.lib().grk_silu_fp8(pre.data_ptr(), pre.stride(0), N, C, out.data_ptr(), out.stride(0),
                                 L.stream_ptr(pre.device)), 'grk_silu_fp8')
    return out


def dsilu_mul_(g, pre):
    """g *= dSiLU(pre) in place (bf16 [N, C] column views): grk_dsilu_mul."""
    _require_cuda(g, pre)
    if g.dtype != torch.bfloat16 or pre.dtype != torch.bfloat16 or g.shape != pre.shape or g.stride(1) != 1 \
            or pre.stride(1) != 1:
        raise L.GrkError('dsilu_mul_ takes two row-major bf16 [N, C] views of one shape')
    N, C = g.shape
    L.check(L.lib().grk_dsilu_mul(g.data_ptr(), g.stride(0), pre.data_ptr(), pre.stride(0), N, C,
                                  L.stream_ptr(g.device)), 'grk_dsilu_mul')
    return g


def norm_gate_fwd(o, u, gamma, beta, eps, dropout_p=0.0, seed=0, y=None):
    """y = dropout(LayerNorm(o) * SiLU(u)) (grk_norm_gate_fwd).  Returns (y bf16 [N, D], stats fp32 [N, 2]).
    seed: int or device int64 [1] tensor (read at kernel time)."""
    _require_cuda(o, u, gamma, beta)
    N, D = o.shape[0], gamma.shape[0]
    dev = o.device
    if y is None:
        y = torch.empty(N, D, dtype=torch.bfloat16, device=dev)
    stats = torch.empty(N, 2, dtype=torch.float32, device=dev)
    (op, ol), (up, ul), (yp, yl) = _bf16_rows(o, 'o', D), _bf16_rows(u, 'u', D), _bf16_rows(y, 'y', D)
    hs, ds = _seed_parts(seed)
    rc = L.lib().grk_norm_gate_fwd(op, ol, up, ul, gamma.data_ptr(), beta.data_ptr(), float(eps), N, D,
                                   float(dropout_p), hs, _ptr(ds), yp, yl, stats.data_ptr(), L.stream_ptr(dev))
    L.check(rc, 'grk_norm_gate_fwd')
    return y, stats


def norm_gate_bwd(gy, o, u, gamma, beta, stats, dropout_p=0.0, seed=0, dout=None, du=None):
    """Gradients of norm_gate_fwd: (dout bf16 [N, D], du bf16 [N, D] w.r.t. pre-activation u, dgamma, dbeta fp32)."""
    _require_cuda(gy, o, u, gamma, beta, stats)
    N, D = o.shape[0], gamma.shape[0]
    dev = o.device
    if dout is None:
        dout = torch.empty(N, D, dtype=torch.bfloat16, device=dev)
    if du is None:
        du = torch.empty(N, D, dtype=torch.bfloat16, device=dev)
    dgamma = torch.empty(D, dtype=torch.float32, device=dev)
    dbeta = torch.empty(D, dtype=torch.float32, device=dev)
    ws = torch.empty(max(L.lib().grk_norm_gate_bwd_workspace(N, D), 4), dtype=torch.uint8, device=dev)
    ptrs = [_bf16_rows(t, n, D) for t, n in ((gy, 'gy'), (o, 'o'), (u, 'u'), (dout, 'dout'), (du, 'du'))]
    (gp, gl), (op, ol), (up, ul), (dp, dl), (dup, dul) = ptrs
    hs, ds = _seed_parts(seed)
    rc = L.lib().grk_norm_gate_bwd(gp, gl, op, ol, up, ul, gamma.data_ptr(), beta.data_ptr(), stats.data_ptr(), N, D,
                                   float(dropout_p), hs, _ptr(ds), dp, dl, dup, dul, dgamma.data_ptr(),
                                   dbeta.data_ptr(), ws.data_ptr(), ws.numel(), L.stream_ptr(dev))
    L.check(rc, 'grk_norm_gate_bwd')
    return dout, du, dgamma, dbeta


def emb_combine_fwd(a, b, pos, scale, relu=True, dropout_p=0.0, seed=0):
    """y = dropout((act(a) + act(b)) * scale + pos) (grk_emb_combine_fwd): bf16 [N, D]
    rows in, a contiguous bf16 [N, D] out.  b / pos may be None."""
    _require_cuda(a, b, pos)
    N, D = a.shape
    y = torch.empty(N, D, dtype=torch.bfloat16, device=a.device)
    (ap, al), (bp, bl), (pp, pl), (yp, yl) = [_bf16_rows(t, n, D) if t is not None else (None, 0)
                                              for t, n in ((a, 'a'), (b, 'b'), (pos, 'pos'), (y, 'y'))]
    hs, ds = _seed_parts(seed)
    L.check(L.lib().grk_emb_combine_fwd(ap, al, bp, bl, pp, pl, float(scale), int(bool(relu)), N, D,
                                        float(dropout_p), hs, _ptr(ds), yp, yl, L.stream_ptr(a.device)),
            'grk_emb_combine_fwd')
    return y


def emb_combine_bwd(gy, a, b, scale, relu=True, dropout_p=0.0, seed=0, want=(True, True, True), has_b=None):
    """Gradients of emb_combine_fwd w.r.t. (a, b, pos) (grk_emb_combine_bwd); None where
    not wanted (or the forward had no b).  a / b: the forward's operands, needed with
    relu only (their signs mask the gradient); has_b: whether the forward had a b
    (default: b is not None)."""
    _require_cuda(gy, a, b)
    N, D = gy.shape
    dev = gy.device
    has_b = b is not None if has_b is None else bool(has_b)
    outs = [torch.empty(N, D, dtype=torch.bfloat16, device=dev) if w and (i != 1 or has_b) else None
            for i, w in enumerate(want)]
    rows = [_bf16_rows(t, n, D) if t is not None else (None, 0)
            for t, n in ((gy, 'gy'), (a, 'a'), (b, 'b'), (outs[0], 'ga'), (outs[1], 'gb'), (outs[2], 'gpos'))]
    (gp, gl), (ap, al), (bp, bl), (p0, l0), (p1, l1), (p2, l2) = rows
    hs, ds = _seed_parts(seed)
    L.check(L.lib().grk_emb_combine_bwd(gp, gl, ap, al, bp, bl, float(scale), int(bool(relu)), N, D,
                                        float(dropout_p), hs, _ptr(ds), p0, l0, p1, l1, p2, l2, L.stream_ptr(dev)),
            'grk_emb_combine_bwd')
    return tuple(outs)


# -------------------------------------------------------------- pair logits
def _rows(t, name):
    if t is None:
        return None, 0
    if t.dim() != 2 or t.stride(1) != 1:
        raise L.GrkError(f'{name} must be a row-major [N, >=D] matrix')
    return t.data_ptr(), t.stride(0)


def _pair_dtype(h, e_pos, e_neg):
    if e_pos.dtype != e_neg.dtype:
        raise L.GrkError('e_pos and e_neg must share a dtype')
    if h.dtype == torch.float32 and e_pos.dtype == torch.bfloat16:
        return L.GRK_F32_BF16
    if h.dtype != e_pos.dtype:
        raise L.GrkError('pair logits take h and e of one dtype, or fp32 h with bf16 e')
    return L.dtype_code(h.dtype)


def pair_logits_fwd(h, e_pos, e_neg, next_token_type=None, with_loss=False):
    """Returns (pos_logits, neg_logits[, loss, count]) -- grk_pair_logits_fwd.
    h and e share a dtype, or h is fp32 and e bf16 (read as they are)."""
    _require_cuda(h, e_pos, e_neg, next_token_type)
    dt = _pair_dtype(h, e_pos, e_neg)
    N, D = h.shape
    dev = h.device
    pos = torch.empty(N, dtype=torch.float32, device=dev)
    neg = torch.empty(N, dtype=torch.float32, device=dev)
    loss = count = part = None
    if with_loss:
        part = torch.empty(max(L.lib().grk_pair_logits_partials(N), 1), dtype=torch.float32, device=dev)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        count = torch.empty(1, dtype=torch.int32, device=dev)
    ntt = None if next_token_type is None else next_token_type.to(torch.int32).contiguous()
    (hp, hl), (pp, pl), (np_, nl) = _rows(h, 'h'), _rows(e_pos, 'e_pos'), _rows(e_neg, 'e_neg')
    rc = L.lib().grk_pair_logits_fwd(hp, hl, pp, pl, np_, nl, _ptr(ntt), N, D, dt,
                                     pos.data_ptr(), neg.data_ptr(), _ptr(part), _ptr(loss), _ptr(count),
                                     L.stream_ptr(dev))
    L.check(rc, 'grk_pair_logits_fwd')
    return (pos, neg, loss, count) if with_loss else (pos, neg)


def pair_logits_bwd(h, e_pos, e_neg, gpos=None, gneg=None, pos_logits=None, neg_logits=None, next_token_type=None,
                    count=None, grad_loss=None, need=(True, True, True), stacked=False):
    """Returns (dh, de_pos, de_neg) -- grk_pair_logits_bwd (None where not needed);
    each gradient in its input's dtype.  stacked: de_pos and de_neg as the two halves
    of one buffer (not for custom-op returns, which may not alias each other)."""
    _require_cuda(h, e_pos, e_neg, gpos, gneg, pos_logits, neg_logits, count, grad_loss)
    dt = _pair_dtype(h, e_pos, e_neg)
    N, D = h.shape
    outs = [torch.empty(N, D, dtype=x.dtype, device=h.device) if n else None for n, x in zip(need, (h, e_pos, e_neg))]
    if stacked and need[1] and need[2] and e_pos.dtype == e_neg.dtype:
        # de_pos and de_neg in the halves of one buffer: the model's pos / neg split of one
        # stacked feat2emb (functional.split_pair) takes them back without a cat
        pair = torch.empty(2 * N, D, dtype=e_pos.dtype, device=h.device)
        outs[1], outs[2] = pair[:N], pair[N:]
    ntt = None if next_token_type is None else next_token_type.to(torch.int32).contiguous()
    gpos = None if gpos is None else gpos.float().contiguous()
    gneg = None if gneg is None else gneg.float().contiguous()
    gl = None if grad_loss is None else grad_loss.float().reshape(1).contiguous()
    (hp, hl), (pp, pl), (np_, nl) = _rows(h, 'h'), _rows(e_pos, 'e_pos'), _rows(e_neg, 'e_neg')
    (a, al), (b, bl), (c, cl) = _rows(outs[0], 'dh'), _rows(outs[1], 'de_pos'), _rows(outs[2], 'de_neg')
    rc = L.lib().grk_pair_logits_bwd(hp, hl, pp, pl, np_, nl, N, D, dt, _ptr(gpos), _ptr(gneg),
                                     _ptr(pos_logits), _ptr(neg_logits), _ptr(ntt), _ptr(count), _ptr(gl), a, al, b,
                                     bl, c, cl, L.stream_ptr(h.device))
    L.check(rc, 'grk_pair_logits_bwd')
    return tuple(outs)


# --------------------------------------------------------- sampled softmax
def _logq(log_q, M):
    if log_q is None:
        return None
    if log_q.dtype != torch.float32 or log_q.numel() != M or not log_q.is_contiguous():
        raise L.GrkError(f'log_q must be a contiguous fp32 tensor of {M} positions')
    return log_q


def sampled_softmax_fwd(h, e, item_ids, valid, tau, log_q=None):
    """(loss, lse2, count) of the in-batch sampled softmax (grk_sampled_softmax_fwd);
    log_q (fp32 [M], natural log): the logQ correction subtracted from column j's logits."""
    _require_cuda(h, e, item_ids, valid, log_q)
    M, D = h.shape
    dev = h.device
    (hp, hl), (ep, el) = _rows(h, 'h'), _rows(e, 'e')
    ws = torch.empty(max(L.lib().grk_sampled_softmax_workspace(M, D), 4), dtype=torch.uint8, device=dev)
    lse2 = torch.empty(M, dtype=torch.float32, device=dev)
    loss = torch.empty((), dtype=torch.float32, device=dev)
    count = torch.empty(1, dtype=torch.int32, device=dev)
    rc = L.lib().grk_sampled_softmax_fwd(hp, hl, ep, el, item_ids.data_ptr(), valid.data_ptr(), M, D, float(tau),
                                         _ptr(_logq(log_q, M)), lse2.data_ptr(), loss.data_ptr(), count.data_ptr(),
                                         ws.data_ptr(), ws.numel(), L.stream_ptr(dev))
    L.check(rc, 'grk_sampled_softmax_fwd')
    return loss, lse2, count


def sampled_softmax_bwd(h, e, item_ids, valid, tau, lse2, grad_loss=None, log_q=None):
    """(dh, de) fp32 [M, D] of the in-batch sampled softmax, fused (grk_sampled_softmax_bwd)."""
    _require_cuda(h, e, item_ids, valid, lse2, grad_loss, log_q)
    M, D = h.shape
    dev = h.device
    dh = torch.empty(M, D, dtype=torch.float32, device=dev)
    de = torch.empty(M, D, dtype=torch.float32, device=dev)
    gl = None if grad_loss is None else grad_loss.float().reshape(1).contiguous()
    ws = torch.empty(max(L.lib().grk_sampled_softmax_workspace(M, D), 4), dtype=torch.uint8, device=dev)
    (hp, hl), (ep, el) = _rows(h, 'h'), _rows(e, 'e')
    rc = L.lib().grk_sampled_softmax_bwd(hp, hl, ep, el, item_ids.data_ptr(), valid.data_ptr(), M, D, float(tau),
                                         _ptr(_logq(log_q, M)), lse2.data_ptr(), _ptr(gl), dh.data_ptr(), D,
                                         de.data_ptr(), D, ws.data_ptr(), ws.numel(), L.stream_ptr(dev))
    L.check(rc, 'grk_sampled_softmax_bwd')
    return dh, de


def sample_negatives(pos, next_token_type, excl, num_items, seed, max_tries=1000, item_feat=None, err_flag=None,
                     item_ok=None):
    """grk_sample_negatives: neg int32 [B, T] -- for positions with next_token_type == 1
    and pos != 0, a uniform id in [1, num_items] outside excl[b] (int32 [B, L], 0 =
    unused slot) and, with item_ok (bool/uint8 [num_items + 1]), with item_ok[id] set
    (an id with a feature row), else 0 -- and, with item_feat (int32 [num_items + 1,
    F]), the negatives' feature rows int32 [B, T, F].  err_flag (int32 [1]) gets bit 2
    when a position exhausted max_tries."""
    _require_cuda(pos, next_token_type, excl, item_feat, err_flag, item_ok)
    if item_ok is not None:
        if item_ok.dim() != 1 or item_ok.shape[0] != num_items + 1:
            raise L.GrkError('item_ok must be [num_items + 1]')
        item_ok = item_ok.to(torch.uint8).contiguous()
    if pos.dim() != 2 or next_token_type.shape != pos.shape or excl.dim() != 2 or excl.shape[0] != pos.shape[0]:
        raise L.GrkError('pos / next_token_type [B, T] and excl [B, L] expected')
    i32 = lambda t: t if t.dtype == torch.int32 and t.is_contiguous() else t.to(torch.int32).contiguous()
    pos, ntt, excl = i32(pos), i32(next_token_type), i32(excl)
    B, T = pos.shape
    neg = torch.empty(B, T, dtype=torch.int32, device=pos.device)
    feat = nf = None
    if item_feat is not None:
        if item_feat.dim() != 2 or item_feat.shape[0] != num_items + 1:
            raise L.GrkError('item_feat must be [num_items + 1, F]')
        item_feat = i32(item_feat)
        nf = item_feat.shape[1]
        feat = torch.empty(B, T, nf, dtype=torch.int32, device=pos.device)
    rc = L.lib().grk_sample_negatives(pos.data_ptr(), ntt.data_ptr(), B, T, excl.data_ptr(), excl.shape[1],
                                      int(num_items), int(seed) & ((1 << 64) - 1), int(max_tries),
                                      _ptr(item_feat), nf or 0, _ptr(item_ok), neg.data_ptr(), _ptr(feat),
                                      _ptr(err_flag), L.stream_ptr(pos.device))
    L.check(rc, 'grk_sample_negatives')
    return neg, feat
