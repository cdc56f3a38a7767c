"""Autograd functions over the libgrk.so kernels.

These are the device ops under the reference's nn.Module surface
(tencent_recommendation_2025_amd/model.py).  Every forward/backward runs a
hand-written HIP kernel from libgrk.so; dense GEMMs, LayerNorm and the
elementwise glue stay torch ops (hipBLASLt / MIOpen).  No CPU fallback: the
kernels require device tensors.
"""
from __future__ import annotations

import os
import weakref

import torch
import torch.nn.functional as F

from . import _lib as L
from . import kernels as K
from . import ops  # noqa: F401  (registers the grk:: custom ops)

_disable = torch._dynamo.disable  # ctypes calls: explicit graph breaks under torch.compile

# bf16 shadows of fp32 dense weights (optim.DenseFlat registers them): the bf16 copy
# its AdamW launch writes with every update, read by the GEMMs here instead of a
# per-step cast of each weight.  id(Parameter) -> (weakref to it, weakref to its
# DenseFlat): keyed by identity (a tensor's == is elementwise, so it cannot key a
# mapping).  Both references are weak -- the DenseFlat holds its Parameters, so a
# strong one here would keep every optimizer's parameters, moments and shadow alive
# for the life of the process -- and a DenseFlat that dies takes its
# entries with it (weakref.finalize).
_SHADOWS = {}


def _drop_shadows(keys, flat_ref):
    for k in keys:
        hit = _SHADOWS.get(k)
        if hit is not None and hit[1] is flat_ref:
            del _SHADOWS[k]


def register_shadows(params, flat):
    """Register ``flat`` (an optim.DenseFlat) as the bf16 shadow owner of ``params``."""
    fref = weakref.ref(flat)
    keys = []
    for p in params:
        _SHADOWS[id(p)] = (weakref.ref(p), fref)
        keys.append(id(p))
    weakref.finalize(flat, _drop_shadows, keys, fref)


def bf16_shadow(weight):
    """weight's bf16 shadow (a view of its DenseFlat's shadow buffer, equal to
    weight.to(bf16) bit for bit), or None when the weight has none."""
    hit = _SHADOWS.get(id(weight))
    if hit is None or hit[0]() is not weight:
        return None
    flat = hit[1]()
    return None if flat is None else flat.shadow_of(weight)

# Debug hook (bench.py): when a list, every fused gather appends its launch arguments.
GATHER_TRACE = None


# --------------------------------------------------------------- lookups ----
class TableRef:
    """Where a lookup's rows live: a plain table weight (drop-in: dense
    autograd gradient) or a row range of a TableGroup (fused optimizer:
    row-sparse gradient collected by the group's sink).  ``chunked``: the
    weight is an intermediate whose row gradients may be summed in the
    chunked fixed order (K.embedding_backward); honoured when every
    drop-in table of a fused lookup allows it.  ``merge``: a DenseMerge
    shared by the fused lookups of one forward that read this weight."""
    __slots__ = ('weight', 'group', 'row_offset', 'chunked', 'merge', 'zero_row0')

    def __init__(self, weight, group=None, row_offset=0, chunked=False, merge=None, zero_row0=False):
        self.weight, self.group, self.row_offset, self.chunked = weight, group, row_offset, chunked
        self.merge = merge
        self.zero_row0 = zero_row0   # row 0 is a zero padding row (the gather skips bag slots on it)


class DenseMerge:
    """Dense row gradients of intermediate tables read by several fused lookups
    of one forward -- the projected feature tables P, read by the seq-side
    feat2emb and by feat2emb_pair: instead of one grk_embedding_backward per
    lookup (each a sort, a zero-filled dense output and a cast) plus autograd's
    add of the two results, every lookup's backward deposits its gradient
    sources here and the LAST one to run reduces them all in one chunked call.
    Every lookup takes all the merged weights as inputs (so whichever runs last
    can return their gradients); the earlier ones return None for them.  The
    sources are added in deposit order (the backward's fixed call order):
    deterministic.  Opt-in (model args.merge_proj_backward)."""

    def __init__(self):
        self.weights = []
        self.pending = 0
        self.sources = []

    def add(self, w):
        if all(x is not w for x in self.weights):
            self.weights.append(w)

    def deposit(self, live):
        for s, g, c in live:
            if s.mode != L.IDX_PLAIN:
                raise RuntimeError('merged dense lookups must be plain (no token-type mask)')
            self.sources.append((s, g, c))

    def resolve(self):
        """{id(weight): gradient or None} after one consumer's backward."""
        self.pending -= 1
        if self.pending > 0:
            return {id(w): None for w in self.weights}
        offs, total = {}, 0
        for w in self.weights:
            offs[id(w)] = total
            total += w.shape[0]
        out = {id(w): None for w in self.weights}
        if self.sources:
            D = self.weights[0].shape[1]
            src = [K.GradSource(sp.idx, g, c, sp.mode, sp.bag, offs[id(sp.ref.weight)], sp.ref.weight.shape[0])
                   for sp, g, c in self.sources]
            chunked = all(sp.ref.chunked for sp, _, _ in self.sources)
            # bf16 tables (the fused trainer's projections): the kernel rounds each dense row to
            # bf16 itself (GRK_BWD_DENSE_BF16) -- no fp32 buffer and no cast kernel
            bf16 = (chunked and D == 512 and all(w.dtype == torch.bfloat16 for w in self.weights)
                    and all(g.dtype == torch.bfloat16 for _, g, _ in self.sources))
            res = K.embedding_backward(src, total, D, padding_idx=0, dense=True, chunked=chunked,
                                       dense_dtype=torch.bfloat16 if bf16 else torch.float32)
            out = {id(w): res.dense[offs[id(w)]:offs[id(w)] + w.shape[0]].to(w.dtype) for w in self.weights}
        self.sources = []
        return out


class LookupSpec:
    __slots__ = ('ref', 'idx', 'out_col', 'mode', 'bag')

    def __init__(self, ref, idx, out_col, mode=L.IDX_PLAIN, bag=1):
        self.ref, self.idx, self.out_col, self.mode, self.bag = ref, idx, out_col, mode, bag


class _FeatureLookupFn(torch.autograd.Function):
    """One fused gather into a [num_tokens, out_ld] buffer, returned as column
    blocks (``splits``) so each consumer (itemdnn / userdnn / position add)
    back-propagates into its own block: no full-width gradient buffer is ever
    materialised or accumulated."""

    @staticmethod
    def forward(ctx, specs, token_type, seq_len, num_tokens, out_ld, extras, splits, *weights):
        dt = specs[0].ref.weight.dtype
        dev = specs[0].ref.weight.device
        out = torch.empty(num_tokens, out_ld, dtype=dt, device=dev)
        lookups = [K.Lookup(s.ref.weight, s.idx, s.out_col, s.mode, s.bag, getattr(s.ref, 'zero_row0', False))
                   for s in specs]
        for i in range(0, len(lookups), L.MAX_FEATURES):
            K.embedding_gather(lookups[i:i + L.MAX_FEATURES], out, num_tokens, token_type, seq_len)
        if GATHER_TRACE is not None:
            GATHER_TRACE.append((lookups, out, num_tokens, token_type, seq_len))
        write_extras(out, extras)
        ctx.specs, ctx.token_type, ctx.seq_len, ctx.splits = specs, token_type, seq_len, splits
        ctx.n_weights = len(weights)
        ctx.weight_ids = [id(w) for w in weights]
        ctx.merges = _merges_of(specs)
        return tuple(out[:, a:b] for a, b in splits)

    @staticmethod
    def backward(ctx, *gsplits):
        specs, splits = ctx.specs, ctx.splits
        D = specs[0].ref.weight.shape[1]

        def locate(col, width):
            """(grad block, column inside it) holding output columns [col, col+width); None if no gradient."""
            for (a, b), g in zip(splits, gsplits):
                if a <= col and col + width <= b:
                    if g is None:
                        return None, 0
                    return (g if g.stride(-1) == 1 else g.contiguous()), col - a
            raise RuntimeError(f'output columns [{col}, {col + width}) are not inside one split')

        live = []
        for s in specs:
            g, c = locate(s.out_col, D)
            if g is not None:
                live.append((s, g, c))
        grads = []
        # drop-in: one deterministic reduction over every distinct table of the call
        dense = [(s, g, c) for s, g, c in live if s.ref.group is None]
        if ctx.n_weights and ctx.merges:
            grads = _merged_grads(ctx, dense)
        elif ctx.n_weights:
            tables, offs, total = {}, {}, 0
            for s in specs:
                w = s.ref.weight
                if s.ref.group is None and id(w) not in tables:
                    tables[id(w)] = w
                    offs[id(w)] = total
                    total += w.shape[0]
            if dense:
                src = [K.GradSource(s.idx, g, c, s.mode, s.bag, offs[id(s.ref.weight)], s.ref.weight.shape[0])
                       for s, g, c in dense]
                res = K.embedding_backward(src, total, D, padding_idx=0, token_type=ctx.token_type,
                                           seq_len=ctx.seq_len, dense=True,
                                           chunked=all(s.ref.chunked for s, _, _ in dense))
                by_id = {k: res.dense[offs[k]:offs[k] + w.shape[0]].to(w.dtype) for k, w in tables.items()}
            else:
                by_id = {k: None for k in tables}
            grads = [by_id[wid] for wid in ctx.weight_ids]
        for s, g, c in live:
            if s.ref.group is not None:
                s.ref.group.collect(K.GradSource(s.idx, g, c, s.mode, s.bag, s.ref.row_offset,
                                                 s.ref.weight.shape[0]), ctx.token_type, ctx.seq_len)
        # extras are dense inputs (features, constants): no gradient is propagated to them
        return (None, None, None, None, None, None, None, *grads)


def _merges_of(specs):
    out = []
    for s in specs:
        m = s.ref.merge
        if s.ref.group is None and m is not None and all(x is not m for x in out):
            out.append(m)
    return out


def _merged_grads(ctx, dense):
    """Gradients of the call's drop-in weights when some are DenseMerge members:
    the members' sources go to their merge (resolved by its last consumer), the
    other drop-in tables are reduced here as usual."""
    D = ctx.specs[0].ref.weight.shape[1]
    by_id = {}
    for m in ctx.merges:
        m.deposit([(s, g, c) for s, g, c in dense if s.ref.merge is m])
    plain = [(s, g, c) for s, g, c in dense if s.ref.merge is None]
    tables, offs, total = {}, {}, 0
    for s in ctx.specs:
        w = s.ref.weight
        if s.ref.group is None and s.ref.merge is None and id(w) not in tables:
            tables[id(w)] = w
            offs[id(w)] = total
            total += w.shape[0]
    if plain:
        src = [K.GradSource(s.idx, g, c, s.mode, s.bag, offs[id(s.ref.weight)], s.ref.weight.shape[0])
               for s, g, c in plain]
        res = K.embedding_backward(src, total, D, padding_idx=0, token_type=ctx.token_type, seq_len=ctx.seq_len,
                                   dense=True, chunked=all(s.ref.chunked for s, _, _ in plain))
        by_id.update({k: res.dense[offs[k]:offs[k] + w.shape[0]].to(w.dtype) for k, w in tables.items()})
    else:
        by_id.update({k: None for k in tables})
    for m in ctx.merges:
        by_id.update(m.resolve())
    return [by_id.get(wid) for wid in ctx.weight_ids]


def feature_lookup(specs, num_tokens, out_ld, token_type=None, seq_len=0, extras=(), splits=None):
    """Fused multi-table gather (+ bag sums) into one [num_tokens, out_ld] buffer.

    ``extras``: (column, [num_tokens, w] or broadcast [1, w] tensor) blocks copied
    into the buffer (dense features, constants; treated as non-differentiable).  Returns the
    buffer's column blocks ``splits`` (list of (start, end); default: the whole
    buffer, returned as a single tensor).  Drop-in tables get dense gradients
    through autograd; grouped tables push row-sparse gradient sources into
    their group's sink."""
    if token_type is not None:
        token_type = token_type.to(torch.int32).contiguous()
    single = splits is None
    splits = tuple((0, out_ld) if single else ((int(a), int(b)) for a, b in splits))
    extras = tuple((int(c), x) for c, x in extras)
    if all(s.ref.group is None for s in specs):
        outs = _lookup_op(specs, token_type, seq_len, num_tokens, out_ld, extras, splits)
    else:
        outs = _lookup_groups(specs, token_type, seq_len, num_tokens, out_ld, extras, splits)
    return outs[0] if single else outs


def _lookup_op(specs, token_type, seq_len, num_tokens, out_ld, extras, splits):
    """Drop-in tables (plain weights, dense gradients): custom op grk::feature_lookup."""
    tables, where, table_of = [], {}, []
    for s in specs:
        w = s.ref.weight
        if id(w) not in where:
            where[id(w)] = len(tables)
            tables.append(w)
        table_of.append(where[id(w)])
    out = torch.ops.grk.feature_lookup(tables, [s.idx for s in specs], table_of, [int(s.out_col) for s in specs],
                                       [int(s.mode) for s in specs], [int(s.bag) for s in specs], token_type,
                                       int(seq_len), int(num_tokens), int(out_ld))
    write_extras(out, extras)
    return tuple(out[:, a:b] for a, b in splits)


def write_extras(out, extras):
    """Dense blocks into the gather buffer: (column, [num_tokens, w] tensor, or a [1, w]
    row broadcast over every token -- e.g. the dnn operand's constant [1, 0, ...] bias /
    padding columns).  On the GPU one grk_write_columns launch for every block (was one
    copy kernel per block), the dtype converted inside it (the same rounding as a .to()
    before the copy).  Dense inputs: no gradient propagates."""
    if not extras:
        return
    if out.is_cuda and len(extras) <= K.MAX_COLUMN_BLOCKS and out.dtype in (torch.float32, torch.bfloat16) \
            and not torch.compiler.is_compiling():   # traced (drop-in under torch.compile): the copies
        K.write_columns(out, extras)
        return
    for col, x in extras:
        out[:, col:col + x.shape[1]].copy_(x.detach())


@_disable
def _lookup_groups(specs, token_type, seq_len, num_tokens, out_ld, extras, splits):
    """Table-group lookups (fused optimizer: row-sparse gradients into the groups' sinks)."""
    weights, seen = [], set()
    for s in specs:
        if s.ref.group is None and id(s.ref.weight) not in seen and s.ref.weight.requires_grad:
            seen.add(id(s.ref.weight))
            weights.append(s.ref.weight)
    merges = _merges_of(specs) if torch.is_grad_enabled() else []
    for m in merges:   # every merged weight is an input of every consumer (the last one returns the gradients)
        m.pending += 1
        for w in m.weights:
            if id(w) not in seen and w.requires_grad:
                seen.add(id(w))
                weights.append(w)
    return _FeatureLookupFn.apply(specs, token_type, seq_len, num_tokens, out_ld, extras, splits, *weights)


# Side-stream branches of the step (the deferred tables' rolling flush slice,
# optim.begin_step): run_on_side forks them from the current stream, join_side_work
# puts the current stream behind them.  Weight gradients on a side stream were tried
# and removed (round 6): the captured C5 step then differed from the eager one
# (DESIGN.md §3f).
_SIDE_PENDING = {}


def join_side_work(index=None):
    """The current stream waits for the pending side-stream work (every private
    stream, or only private stream ``index``)."""
    if not _SIDE_PENDING:
        return
    for key, side in list(_SIDE_PENDING.items()):
        if index is None or key[1] == index:
            torch.cuda.current_stream(key[0]).wait_stream(side)
            del _SIDE_PENDING[key]


def run_on_side(fn, device, index):
    """fn() on private stream ``index`` of ``device``, forked from the current stream;
    joined by the next join_side_work().  fn's tensors must be kept alive by the
    caller (or record_stream'd) until then."""
    from .streams import private_stream
    dev = torch.device(device)
    cur = torch.cuda.current_stream(dev)
    side = private_stream(dev, index)
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        fn()
    _SIDE_PENDING[(dev.index if dev.index is not None else torch.cuda.current_device(), index)] = side


class _LinearFn(torch.autograd.Function):
    """y = x W^T + b (+ addend) (then ReLU) on grk_gemm (hipBLASLt with stream-K
    eligible).  bf16 operands (the autocast dtype of the reference's training),
    fp32 accumulation; the weight gradient is written by the GEMM in the weight's
    own dtype (fp32 master weights: no bf16 round trip and no cast kernel).

    relu: the dnn layers' ReLU in the GEMM's store (grk_gemm_ex epilogue); the
    backward masks the gradient by the saved output (threshold_backward).
    in_place: a bf16 row-major addend whose only use is this sum (the projected
    rows' bag sum, a column block of the gather buffer) is accumulated into where
    it lies -- the output is that view -- instead of being copied to a contiguous
    C first."""

    @staticmethod
    def forward(ctx, x, weight, bias, addend, relu, in_place):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        if x2.dtype != torch.bfloat16:
            x2 = x2.to(torch.bfloat16)
        if x2.stride(-1) != 1 or (x2.shape[0] > 1 and x2.stride(0) < x2.shape[1]):
            x2 = x2.contiguous()
        wb = weight if weight.dtype == torch.bfloat16 and weight.is_contiguous() else bf16_shadow(weight)
        if wb is None:
            wb = weight.detach().to(torch.bfloat16).contiguous()
        b = None if bias is None else bias.detach().contiguous()
        out = None
        if addend is not None:
            addend = addend.reshape(-1, wb.shape[0])
            if in_place and addend.dtype == torch.bfloat16 and addend.stride(1) == 1 and addend.stride(0) % 8 == 0 \
                    and addend.data_ptr() % 16 == 0:
                out, addend = addend, None
            elif addend.dtype != torch.bfloat16 or addend.stride(1) != 1 or addend.stride(0) != wb.shape[0]:
                addend = addend.to(torch.bfloat16).contiguous()
        y = K.gemm(x2, wb, trans_b=True, bias=b, addend=addend, out=out,
                   beta=0.0 if addend is None and out is None else 1.0, relu=relu)
        ctx.save_for_backward(x2, wb, y if relu else None)
        ctx.meta = (shp, weight.dtype, None if bias is None else bias.dtype, ctx.needs_input_grad[3])
        return y.view(*shp[:-1], wb.shape[0])

    @staticmethod
    def backward(ctx, gy):
        x2, wb, y = ctx.saved_tensors
        shp, wdt, bdt, want_addend = ctx.meta
        g2 = gy.reshape(-1, gy.shape[-1])
        if y is not None:            # ReLU in the forward's store: the gradient through its mask
            g2 = torch.ops.aten.threshold_backward(g2, y, 0)
        if g2.dtype != torch.bfloat16:
            g2 = g2.to(torch.bfloat16)
        if not g2.is_contiguous():
            g2 = g2.contiguous()
        dx = K.gemm(g2, wb).view(shp) if ctx.needs_input_grad[0] else None
        dw_dt = torch.float32 if wdt == torch.float32 else torch.bfloat16
        dw = db = None
        if ctx.needs_input_grad[1] and K.wgrad_ok(g2, x2):
            # split-K MFMA weight gradient, bias gradient from the same pass over gy
            dw, db = K.wgrad(g2, x2, out_dtype=dw_dt, want_db=ctx.needs_input_grad[2])
            db = db.to(bdt) if db is not None else None
        elif ctx.needs_input_grad[1]:
            dw = K.gemm(g2, x2, trans_a=True, out_dtype=dw_dt)
        if ctx.needs_input_grad[2] and db is None:
            db = g2.sum(0, dtype=torch.float32).to(bdt)
        ga = None
        if want_addend:
            ga = g2.view(gy.shape) if y is not None else gy
        return dx, dw, db, ga, None, None


@_disable
def linear(x, weight, bias=None, addend=None, relu=False, in_place=False):
    """torch.nn.functional.linear (+ addend, as torch.addmm; then ReLU with relu) on
    grk_gemm: bf16 operands, fp32 accumulation, bf16 output.  in_place: accumulate
    into the addend where it lies (see _LinearFn; the addend's values are consumed)."""
    return _LinearFn.apply(x, weight, bias, addend, bool(relu), bool(in_place))


_ZERO_BLOCKS = {}


def _zero_block(rows, cols, dtype, device):
    """A cached all-zero [rows, cols] tensor (read only): no fill kernel per use."""
    key = (int(rows), int(cols), dtype, str(device))
    t = _ZERO_BLOCKS.get(key)
    if t is None:
        t = _ZERO_BLOCKS[key] = torch.zeros(rows, cols, dtype=dtype, device=device)
    return t


class _DnnWeightFn(torch.autograd.Function):
    """The composed
    itemdnn / userdnn weight of the projection restatement
    (model._dnn_weight): [d, width] = [blocks... | W_k [W_t | b_t] (mm features,
    the emb_transform folded in) | b + sum_k W_k b_t | 0], cast once to `dtype`.

    Forward: one cat + one mm per mm feature, one cat of every column block and
    one cast; backward: one cast of the gradient, then views, plus one cat and
    two mm per mm feature -- where autograd of the eager composition (cats,
    pads, slices, their zero-filled backwards, autocast casts) ran ~25 kernels
    for C2's two dnn weights.  fp32 arithmetic throughout (the eager form ran
    the W_k [W_t | b_t] product under bf16 autocast).  A one-launch HIP form of
    this node was measured slower and removed."""

    @staticmethod
    def forward(ctx, nblocks, nmm, width, dtype, *ts):
        blocks, bias = ts[:nblocks], ts[nblocks]
        mms = [ts[nblocks + 1 + 3 * i: nblocks + 4 + 3 * i] for i in range(nmm)]
        d = bias.shape[0]
        cols = [b.detach() for b in blocks]
        bcol = bias.detach()[:, None]
        ets = []
        with torch.autocast(bias.device.type, enabled=False):
            for Wk, Wt, bt in mms:
                et = torch.cat([Wt.detach(), bt.detach()[:, None]], 1)
                Mk = Wk.detach() @ et
                cols.append(Mk[:, :-1])
                bcol = bcol + Mk[:, -1:]
                ets.append(et)
            cols.append(bcol)
            used = sum(c.shape[1] for c in cols)
            if width > used:
                cols.append(_zero_block(d, width - used, bias.dtype, bias.device))
            Wc = torch.cat(cols, 1)
        out = Wc.to(dtype) if dtype != Wc.dtype else Wc
        ctx.save_for_backward(*[m[0] for m in mms], *ets)
        ctx.meta = (nblocks, nmm, [b.shape[1] for b in blocks], [m[1].shape[1] for m in mms],
                    [b.dtype for b in blocks], bias.dtype)
        return out

    @staticmethod
    def backward(ctx, g):
        nblocks, nmm, bw, mmw, bdt, biasdt = ctx.meta
        saved = ctx.saved_tensors
        Wks, ets = saved[:nmm], saved[nmm:]
        g32 = g.float()
        grads, c = [], 0
        for w, dt in zip(bw, bdt):
            grads.append(g32[:, c:c + w].to(dt))
            c += w
        mm_cols = []
        for w in mmw:
            mm_cols.append((c, c + w))
            c += w
        gb = g32[:, c]
        mm_grads = []
        with torch.autocast(g.device.type, enabled=False):
            for (c0, c1), Wk, et in zip(mm_cols, Wks, ets):
                dM = torch.cat([g32[:, c0:c1], g32[:, c:c + 1]], 1)
                dWk = dM @ et.t()
                det = Wk.t() @ dM
                mm_grads += [dWk, det[:, :-1], det[:, -1]]
        return (None, None, None, None, *grads, gb.to(biasdt), *mm_grads)


@_disable
def dnn_weight(blocks, bias, mms, width, dtype):
    """model._dnn_weight as one autograd node (_DnnWeightFn): blocks = the weight's
    column blocks taken as they are, mms = [(W_k, emb_transform weight, bias)]."""
    flat = [t for m in mms for t in m]
    return _DnnWeightFn.apply(len(blocks), len(mms), int(width), dtype, *blocks, bias, *flat)


class _SplitPairFn(torch.autograd.Function):
    """x[:n], x[n:] whose backward takes the two gradients back as ONE view when
    they are the halves of one buffer (kernels.pair_logits_bwd writes them so),
    where autograd's split backward always copies them into a new tensor (cat)."""

    @staticmethod
    def forward(ctx, x, n):
        ctx.n, ctx.shape = n, x.shape
        return x[:n], x[n:]

    @staticmethod
    def backward(ctx, ga, gb):
        n, shape = ctx.n, ctx.shape
        if ga is None and gb is None:
            return None, None
        if ga is None:
            ga = gb.new_zeros((n,) + tuple(shape[1:]))
        if gb is None:
            gb = ga.new_zeros((shape[0] - n,) + tuple(shape[1:]))
        v = _adjacent_rows(ga, gb)
        return (v if v is not None else torch.cat([ga, gb], 0)), None


def _adjacent_rows(a, b):
    """torch.cat([a, b], 0) as a view when b starts where a ends in one storage, else None."""
    if a.dtype != b.dtype or a.shape[1:] != b.shape[1:] or not (a.is_contiguous() and b.is_contiguous()) \
            or a.device != b.device or a.untyped_storage().data_ptr() != b.untyped_storage().data_ptr() \
            or b.data_ptr() != a.data_ptr() + a.numel() * a.element_size():
        return None
    return a.as_strided((a.shape[0] + b.shape[0],) + tuple(a.shape[1:]), a.stride(), a.storage_offset())


@_disable
def split_pair(x, n):
    """(x[:n], x[n:]) along dim 0; the backward joins adjacent gradient halves without a copy."""
    return _SplitPairFn.apply(x, int(n))


class _EmbCombineFn(torch.autograd.Function):
    """seqs = dropout((act(a) + act(b)) * scale + pos) on grk_emb_combine (one pass
    each way); a / b the itemdnn / userdnn outputs before their ReLU when relu."""

    @staticmethod
    def forward(ctx, a, b, pos, scale, relu, dropout_p, seed):
        D = a.shape[-1]

        def rows(t):
            if t is None:
                return None
            t = t.reshape(-1, D)
            return t if t.dtype == torch.bfloat16 and t.stride(-1) == 1 and t.stride(0) % 8 == 0 \
                and t.data_ptr() % 16 == 0 else t.to(torch.bfloat16).contiguous()

        a2, b2, p2 = rows(a), rows(b), rows(pos)
        y = K.emb_combine_fwd(a2, b2, p2, scale, relu, dropout_p, seed)
        ctx.save_for_backward(a2 if relu else None, b2 if relu else None,
                              seed if isinstance(seed, torch.Tensor) else None)
        ctx.meta = (a.shape, scale, relu, dropout_p, None if isinstance(seed, torch.Tensor) else seed,
                    a.dtype, None if b is None else b.dtype, None if pos is None else pos.dtype)
        return y.view(a.shape)

    @staticmethod
    def backward(ctx, gy):
        a2, b2, seed_t = ctx.saved_tensors
        shp, scale, relu, p, seed_i, adt, bdt, pdt = ctx.meta
        g2 = gy.reshape(-1, shp[-1])
        if g2.dtype != torch.bfloat16 or g2.stride(-1) != 1 or g2.stride(0) % 8 or g2.data_ptr() % 16:
            g2 = g2.to(torch.bfloat16).contiguous()
        want = (ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.needs_input_grad[2])
        ga, gb, gp = K.emb_combine_bwd(g2, a2, b2, scale, relu, p, seed_t if seed_t is not None else seed_i, want,
                                       has_b=bdt is not None)
        ga = ga.view(shp).to(adt) if ga is not None else None
        gb = gb.view(shp).to(bdt) if gb is not None else None
        gp = gp.view(shp).to(pdt) if gp is not None else None
        return ga, gb, gp, None, None, None, None


@_disable
def emb_combine(a, b, pos, scale, relu=True, dropout_p=0.0, seed=0):
    """The first block's input: dropout((act(a) + act(b)) * scale + pos) (bf16 out).
    b / pos may be None; seed an int or a device int64 [1] tensor (model.dropout_seed)."""
    return _EmbCombineFn.apply(a, b, pos, float(scale), bool(relu), float(dropout_p), seed)


class _AddNormFn(torch.autograd.Function):
    """HSTU residual stream step on grk_add_norm: s_new = bf16(s + y),
    x = LayerNorm(s_new) (x_dtype).  Returns (s_new, x), or x alone when y is
    None (the first block: LayerNorm of s)."""

    @staticmethod
    def forward(ctx, s, y, weight, bias, eps, x_dtype):
        shp = s.shape
        D = shp[-1]

        def rows(t):
            t = t.reshape(-1, D)
            return t if t.dtype == torch.bfloat16 and t.stride(-1) == 1 and t.stride(0) % 8 == 0 \
                else t.to(torch.bfloat16).contiguous()

        s2 = rows(s)
        y2 = rows(y) if y is not None else None
        g32 = weight.detach().float().contiguous()
        b32 = bias.detach().float().contiguous()
        s_new, x, stats = K.add_norm_fwd(s2, y2, g32, b32, eps, x_dtype)
        saved = s_new if s_new is not None else s2
        ctx.save_for_backward(saved, stats, g32)
        ctx.meta = (shp, y is not None, weight.dtype, bias.dtype, s.dtype, None if y is None else y.dtype)
        if y is None:
            return x.view(shp)
        return s_new.view(shp), x.view(shp)

    @staticmethod
    def backward(ctx, *grads):
        saved, stats, g32 = ctx.saved_tensors
        shp, has_y, wdt, bdt, sdt, ydt = ctx.meta
        D = shp[-1]
        gs, gx = (grads if has_y else (None, grads[0]))
        gx = gx.reshape(-1, D)
        if gx.stride(-1) != 1 or gx.stride(0) % 8:
            gx = gx.contiguous()
        if gs is not None:
            gs = gs.reshape(-1, D)
            if gs.dtype != torch.bfloat16 or gs.stride(-1) != 1 or gs.stride(0) % 8:
                gs = gs.to(torch.bfloat16).contiguous()
        ds, dg, db = K.add_norm_bwd(gx, gs, saved, g32, stats)
        ds = ds.view(shp)
        return (ds.to(sdt), ds.to(ydt) if has_y else None, dg.to(wdt), db.to(bdt), None, None)


@_disable
def add_norm(s, y, weight, bias, eps, x_dtype=torch.bfloat16):
    """(s + y, LayerNorm(s + y)) with a bf16 residual stream (grk_add_norm); y None -> LayerNorm(s) only."""
    return _AddNormFn.apply(s, y, weight, bias, float(eps), x_dtype)


class _GroupStackFn(torch.autograd.Function):
    """Equally-sized tables of a TableGroup as one [G, rows, D] tensor for use
    in differentiable torch ops (a view of the group buffer when the tables
    are adjacent); the backward hands the dense gradient to the group (fused
    optimizer) instead of autograd (the group's weight views do not require
    grad)."""

    @staticmethod
    def forward(ctx, anchor, group, offsets, rows):
        ctx.group, ctx.offsets, ctx.rows = group, offsets, rows
        o0 = offsets[0]
        ctx.contiguous = all(o == o0 + j * rows for j, o in enumerate(offsets))
        if ctx.contiguous:
            return group.flat[o0:o0 + len(offsets) * rows].view(len(offsets), rows, -1)
        return torch.stack([group.flat[o:o + rows] for o in offsets])

    @staticmethod
    def backward(ctx, g):
        if ctx.contiguous:
            ctx.group.collect_dense(ctx.offsets[0], g.reshape(-1, g.shape[-1]))
        else:
            for j, o in enumerate(ctx.offsets):
                ctx.group.collect_dense(o, g[j])
        return None, None, None, None


_ANCHOR = torch.zeros((), requires_grad=True)  # makes _GroupStackFn's output part of the graph


class _WeightBlocksFn(torch.autograd.Function):
    """Column blocks of an itemdnn / userdnn weight ``W [d_out, nb * d]`` for the
    projection restatement (model._projection / model._dnn_weight): ``singles``
    are single blocks as views of W (W_0, direct-feature and mm blocks of the
    composed dnn weight), ``stacks`` are [len(js), d_out, d] stacks of blocks
    cast to the tables' dtype (the projections P_f = E_f W_f^T, one per
    equal-row-count table group).

    The backward writes every block's gradient into ONE buffer of W's shape --
    zeros only for blocks no output reached.  Autograd of the slice / index
    ops it replaces zero-fills a full-size tensor per slice and per group,
    index_puts into it, adds those full-size tensors and casts the bf16 sum
    back to fp32 (~18 launches and ~300 MB per step for C2's itemdnn).  Every
    block gets its gradient from exactly one output, so the values are the
    same bits (a sum with zeros is exact; bf16 -> fp32 is exact)."""

    @staticmethod
    def forward(ctx, W, d, singles, stacks):
        ctx.set_materialize_grads(False)
        ctx.d, ctx.singles, ctx.stacks = d, singles, stacks
        ctx.shape, ctx.dtype, ctx.device = W.shape, W.dtype, W.device
        Wv = W.detach().view(W.shape[0], -1, d)
        outs = [Wv[:, j, :] for j in singles]
        cast = {W.dtype: Wv}
        sh = bf16_shadow(W) if any(dt == torch.bfloat16 for _, dt in stacks) else None
        if sh is not None:
            cast[torch.bfloat16] = sh.view(W.shape[0], -1, d)
        for js, dt in stacks:
            if dt not in cast:
                cast[dt] = Wv.to(dt)           # the whole weight once per dtype, as before
            src = cast[dt]
            outs.append(src[:, js[0], :][None] if len(js) == 1 else
                        src.index_select(1, _block_index(js, W.device)).permute(1, 0, 2))
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        d, (rows, cols) = ctx.d, ctx.shape
        nb = cols // d
        if all(g is None for g in grads):
            return None, None, None, None
        dW = torch.empty(ctx.shape, dtype=ctx.dtype, device=ctx.device)
        dWv = dW.view(rows, nb, d)
        covered = [False] * nb
        for j, g in zip(ctx.singles, grads):
            if g is not None:
                dWv[:, j, :].copy_(g)
                covered[j] = True
        for (js, _), g in zip(ctx.stacks, grads[len(ctx.singles):]):
            if g is None:
                continue
            if len(js) == 1:
                dWv[:, js[0], :].copy_(g[0])
            else:
                dWv.index_copy_(1, _block_index(js, ctx.device), g.permute(1, 0, 2).to(ctx.dtype))
            for j in js:
                covered[j] = True
        j = 0
        while j < nb:                           # runs of blocks no output reached
            if covered[j]:
                j += 1
                continue
            e = j
            while e < nb and not covered[e]:
                e += 1
            dWv[:, j:e, :].zero_()
            j = e
        return dW, None, None, None


_BLOCK_INDEX = {}


def _block_index(js, device):
    """Cached device int64 index of block numbers (no host -> device copy per step)."""
    key = (tuple(js), str(device))
    t = _BLOCK_INDEX.get(key)
    if t is None:
        t = _BLOCK_INDEX[key] = torch.tensor(js, dtype=torch.int64).to(device)
    return t


def weight_blocks_sliced(W, d, singles, stacks):
    """weight_blocks' outputs as plain slice / index ops (autograd zero-fills a full-size
    gradient per slice and per stack): the form torch.compile traces, so a compiled
    model keeps one graph through the projections (weight_blocks itself is an explicit
    graph break)."""
    Wv = W.view(W.shape[0], -1, d)
    outs = [Wv[:, j, :] for j in singles]
    cast = {W.dtype: Wv}
    for js, dt in stacks:
        if dt not in cast:
            cast[dt] = Wv.to(dt)
        src = cast[dt]
        outs.append(src[:, js[0], :][None] if len(js) == 1 else
                    src.index_select(1, _block_index(js, W.device)).permute(1, 0, 2))
    return tuple(outs)


@_disable
def weight_blocks(W, d, singles=(), stacks=()):
    """Views of single column blocks and dtype-cast stacks of blocks of ``W`` (see
    _WeightBlocksFn): returns ``(singles..., stacks...)``; ``stacks`` is a sequence
    of (block numbers, dtype)."""
    singles = tuple(int(j) for j in singles)
    stacks = tuple((tuple(int(j) for j in js), dt) for js, dt in stacks)
    nb = W.shape[1] // d
    if W.shape[1] != nb * d or any(not 0 <= j < nb for j in singles + sum((js for js, _ in stacks), ())):
        raise ValueError(f'weight blocks: W {tuple(W.shape)} is not [.., nb * {d}] or a block is outside [0, {nb})')
    seen = list(singles) + [j for js, _ in stacks for j in js]
    if len(seen) != len(set(seen)):
        raise ValueError('weight blocks: every block may appear in one output only')
    return _WeightBlocksFn.apply(W, d, singles, stacks)


@_disable
def group_stack(group, offsets, rows):
    return _GroupStackFn.apply(_ANCHOR, group, tuple(offsets), rows)


PROJ_ROW_ALIGN = 32   # grouped projection: each table's P rows start at a multiple of 32


class _ProjectFn(torch.autograd.Function):
    """The projected feature tables of one dnn on the grouped MFMA GEMMs
    (grk_grouped_gemm / grk_grouped_wgrad; model._projection restates the
    reference's per-feature lookups feeding itemdnn / userdnn,
    model/BaseLine/model.py:254-310, as lookups of P_f = E_f W_f^T).

    Inputs: the dnn weight W [d_out, nb * d] and its column blocks ``singles``
    (returned as views, as weight_blocks does); ``tables`` = [(block j, row offset
    in ``group``, rows, P row offset)] of tables held by one bf16 TableGroup.
    Returns (singles..., P [P rows, d_out] bf16): table f's P rows at its P offset
    (a multiple of 32; the rows between tables are never read).

    Backward: dE_f = dP_f W_f (one launch, bf16) into the group's dense gradient
    sink (group.collect_dense), dW_f = dP_f^T E_f (one launch + the split-K
    reduction) straight into the blocks of ONE fp32 gradient of W's shape, the
    singles' gradients copied into theirs, zeros for blocks no output reached.
    dP's rows between tables are zero (the embedding backward writes only rows
    that are looked up), so the weight gradient sums each table's padded rows
    exactly (B rows past the table read its last row, times zero)."""

    @staticmethod
    def forward(ctx, W, d, singles, tables, group, p_rows):
        ctx.set_materialize_grads(False)
        d_out, cols = W.shape
        nb = cols // d
        Wb = W.detach() if W.dtype == torch.bfloat16 else bf16_shadow(W)
        if Wb is None:
            Wb = W.detach().to(torch.bfloat16)
        E = group.flat
        P = torch.empty(p_rows, d_out, dtype=torch.bfloat16, device=E.device)
        K.grouped_gemm([(E[off:off + rows], Wb[:, j * d:(j + 1) * d], P[poff:poff + rows])
                        for j, off, rows, poff in tables], n=d_out, k=d, b_layout=0)
        ctx.save_for_backward(Wb)
        ctx.meta = (d, nb, tuple(singles), tuple(tables), group, W.dtype, W.shape)
        Wv = W.detach().view(d_out, nb, d)
        return (*[Wv[:, j, :] for j in singles], P)

    @staticmethod
    def backward(ctx, *grads):
        (Wb,) = ctx.saved_tensors
        d, nb, singles, tables, group, wdt, wshape = ctx.meta
        d_out = wshape[0]
        gs, dP = grads[:len(singles)], grads[len(singles)]
        if all(g is None for g in gs) and dP is None:
            return None, None, None, None, None, None
        dW = torch.empty(wshape, dtype=torch.float32, device=Wb.device)
        dWv = dW.view(d_out, nb, d)
        covered = [False] * nb
        for j, g in zip(singles, gs):
            if g is not None:
                dWv[:, j, :].copy_(g)
                covered[j] = True
        if dP is not None:
            if dP.dtype != torch.bfloat16:
                dP = dP.to(torch.bfloat16)
            dP = dP if dP.is_contiguous() else dP.contiguous()
            E = group.flat
            dE = torch.empty(sum(rows for _, _, rows, _ in tables), d, dtype=torch.bfloat16, device=dP.device)
            gg, r = [], 0
            for j, off, rows, poff in tables:
                gg.append((dP[poff:poff + rows], Wb[:, j * d:(j + 1) * d], dE[r:r + rows]))
                r += rows
            K.grouped_gemm(gg, n=d, k=d_out, b_layout=1)
            r = 0
            for j, off, rows, poff in tables:
                group.collect_dense(off, dE[r:r + rows])
                r += rows
            K.grouped_wgrad([(dP[poff:], E[off:], dW[:, j * d:(j + 1) * d], _pad_rows(rows), rows)
                             for j, off, rows, poff in tables], m=d_out, n=d)
            for j, _, _, _ in tables:
                covered[j] = True
        j = 0
        while j < nb:                           # runs of blocks no output reached
            if covered[j]:
                j += 1
                continue
            e = j
            while e < nb and not covered[e]:
                e += 1
            dWv[:, j:e, :].zero_()
            j = e
        return (dW if wdt == torch.float32 else dW.to(wdt)), None, None, None, None, None


def _pad_rows(rows):
    return -(-int(rows) // PROJ_ROW_ALIGN) * PROJ_ROW_ALIGN


def proj_layout(rows_list):
    """P row offsets of tables with the given row counts (each a multiple of
    PROJ_ROW_ALIGN) and the padded total."""
    offs, r = [], 0
    for rows in rows_list:
        offs.append(r)
        r += _pad_rows(rows)
    return offs, r


def project_blocks(W, d, singles, tables, group, p_rows):
    """(singles..., P): see _ProjectFn.  tables: [(block j, group row offset, rows, P row offset)]."""
    singles = tuple(int(j) for j in singles)
    tables = tuple((int(j), int(o), int(r), int(p)) for j, o, r, p in tables)
    return _ProjectFn.apply(W, int(d), singles, tables, group, int(p_rows))


# ------------------------------------------------------------- attention ----
def _seed(seed):
    """A dropout seed: an int, or an int64 [1] device tensor read by the kernels at run time."""
    return seed if isinstance(seed, torch.Tensor) else int(seed)


def softmax_mha(qkv, key_valid, B, T, H, hd, dropout_p=0.0, seed=0, precise=True, seq_range=None, row_base=None):
    """Causal + key-padding softmax attention on a packed [B*T, 3D] (q|k|v) tensor
    (custom op grk::softmax_attention; returns qkv's dtype).  fp32 / fp16 inputs
    run the fp32-fidelity kernels where the shape allows (ops.py); bf16 inputs
    the product kernels, precise (default: P and dS as bf16 hi + lo pairs, 1-4 %
    slower than precise=False, which rounds them and is held only to 1e-2)."""
    if key_valid is None:
        key_valid = torch.ones(B, T, dtype=torch.uint8, device=qkv.device)
    sd = seed if isinstance(seed, torch.Tensor) else None
    out, _ = torch.ops.grk.softmax_attention(qkv, key_valid, H, hd, float(dropout_p), 0 if sd is not None else int(seed),
                                             sd, int(precise), seq_range, row_base)
    return out if out.dtype == qkv.dtype else out.to(qkv.dtype)


def hstu_core(pre, rab, ln_w, ln_b, key_valid, B, T, H, hd, inv_n, eps=1e-8, precise=True, dropout_p=0.0, seed=0,
              seq_range=None, timestamps=None, rab_t=None, row_base=None):
    """Fused HSTU layer core on the [B*T, 4D] (u|v|q|k) pre-activation (custom op
    grk::hstu_core, ops.py): three kernels forward (attention with SiLU on load,
    LayerNorm * SiLU(u) gate with dropout), two backward; no eager glue.
    timestamps (int64 [B, T]) with rab_t ([H, nbt], nbt <= 64) add the time bias
    rab_t[h, time_bucket(t_q - t_k)] to every score (oracle/hstu.py time_bucket)."""
    if key_valid is None:
        key_valid = torch.ones(B, T, dtype=torch.uint8, device=pre.device)
    if (timestamps is None) != (rab_t is None):
        raise ValueError('the time bias needs both timestamps and rab_t')
    if timestamps is not None:
        timestamps = timestamps.to(device=pre.device, dtype=torch.int64).contiguous()
    sd = seed if isinstance(seed, torch.Tensor) else None
    y, _, _ = torch.ops.grk.hstu_core(pre, rab, ln_w, ln_b, key_valid, H, hd, float(inv_n), float(eps), int(precise),
                                      float(dropout_p), 0 if sd is not None else int(seed), sd, seq_range,
                                      timestamps, rab_t, row_base)
    return y if pre.dtype == torch.bfloat16 else y.to(pre.dtype)


class _HSTUFp8Fn(torch.autograd.Function):
    """HSTU layer core with fp8 q/k/v (config C5, BASELINE.json configs[4]):
    SiLU'd v|q|k quantised once to e4m3 (grk_silu_fp8), attention on the fp8
    kernels (QK^T on the fp8 MFMA, P V on bf16 over the exactly widened values),
    then the same LayerNorm * SiLU(u) gate as the bf16 layer.  Backward is
    straight-through at the quantiser: the attention's gradients w.r.t. the fp8
    values times dSiLU(pre) (grk_dsilu_mul)."""

    @staticmethod
    def forward(ctx, pre, rab, ln_w, ln_b, key_valid, H, hd, inv_n, eps, dropout_p, seed, seq_range):
        D = H * hd
        B, T = key_valid.shape
        pb = pre.to(torch.bfloat16).contiguous()
        x8 = K.silu_fp8(pb[:, D:])                       # v | q | k
        rab32 = rab.float().contiguous()
        args = K.attn_args(L.ATTN_HSTU, x8[:, D:2 * D], x8[:, 2 * D:], x8[:, :D], B, T, H, hd, key_valid=key_valid,
                           scale=hd ** -0.5, rab=rab32, inv_n=inv_n, precise=1, out_dtype=torch.bfloat16,
                           seq_range=seq_range)
        o = torch.empty(pb.shape[0], D, dtype=torch.bfloat16, device=pb.device)
        K.attention_fwd(args, o)
        lw, lb = ln_w.float().contiguous(), ln_b.float().contiguous()
        y, stats = K.norm_gate_fwd(o, pb[:, :D], lw, lb, eps, dropout_p, seed)
        ctx.save_for_backward(pb, x8, o, stats, rab32, lw, lb, key_valid, seq_range,
                              seed if isinstance(seed, torch.Tensor) else None)
        ctx.meta = (H, hd, inv_n, dropout_p, seed if not isinstance(seed, torch.Tensor) else None, pre.dtype,
                    rab.dtype, ln_w.dtype)
        return y if pre.dtype == torch.bfloat16 else y.to(pre.dtype)

    @staticmethod
    def backward(ctx, gy):
        pb, x8, o, stats, rab32, lw, lb, key_valid, seq_range, seed_dev = ctx.saved_tensors
        H, hd, inv_n, dropout_p, seed, pdt, rdt, ldt = ctx.meta
        D = H * hd
        B, T = key_valid.shape
        seed = seed_dev if seed_dev is not None else seed
        dpre = torch.empty(pb.shape[0], 4 * D, dtype=torch.bfloat16, device=pb.device)
        do, _, dw, db = K.norm_gate_bwd(gy.to(torch.bfloat16).contiguous(), o, pb[:, :D], lw, lb, stats, dropout_p,
                                        seed, du=dpre[:, :D])
        drab = torch.zeros_like(rab32)
        args = K.attn_args(L.ATTN_HSTU, x8[:, D:2 * D], x8[:, 2 * D:], x8[:, :D], B, T, H, hd, key_valid=key_valid,
                           scale=hd ** -0.5, rab=rab32, inv_n=inv_n, precise=1, out_dtype=torch.bfloat16,
                           seq_range=seq_range)
        K.attention_bwd(args, None, do, None, None, dpre[:, 2 * D:3 * D], dpre[:, 3 * D:], dpre[:, D:2 * D], drab)
        K.dsilu_mul_(dpre[:, D:], pb[:, D:])
        return (dpre.to(pdt), drab.to(rdt), dw.to(ldt), db.to(ldt), None, None, None, None, None, None, None, None)


@_disable
def hstu_core_fp8(pre, rab, ln_w, ln_b, key_valid, B, T, H, hd, inv_n, eps=1e-8, dropout_p=0.0, seed=0,
                  seq_range=None):
    """hstu_core with fp8 q/k/v (config C5): padded [B*T, 4D] layout, no time bias
    (the fp8 kernels are the chunked ones)."""
    if key_valid is None:
        key_valid = torch.ones(B, T, dtype=torch.uint8, device=pre.device)
    return _HSTUFp8Fn.apply(pre, rab, ln_w, ln_b, key_valid, H, hd, float(inv_n), float(eps), float(dropout_p), seed,
                            seq_range)


# ---------------------------------------------------------------- logits ----
def _rows2d(x):
    x = x.reshape(-1, x.shape[-1])
    return x if x.stride(-1) == 1 else x.contiguous()


def _shape_grads(ctx, *gs):
    out = [None if g is None else g.view(shape).to(dt) for g, shape, dt in zip(gs, ctx.shapes, ctx.dtypes)]
    return (*out, None)


def pair_logits(h, e_pos, e_neg, next_token_type):
    """(pos, neg) logits = rowwise <h, e> masked by next_token_type == 1 (fp32, shape of h[..., 0]);
    custom op grk::pair_logits."""
    ntt = next_token_type.reshape(-1).to(torch.int32).contiguous()
    D = h.shape[-1]
    pos, neg = torch.ops.grk.pair_logits(h.reshape(-1, D), e_pos.reshape(-1, D), e_neg.reshape(-1, D), ntt)
    shape = h.shape[:-1]
    return pos.view(shape), neg.view(shape)


class _BCELossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, ep, en, ntt):
        if h.dtype == torch.float32 and ep.dtype == en.dtype == torch.bfloat16:
            # fp32 log_feats, bf16 item embeddings (autocast): the kernels read both as they are
            # (the logits of promoting e to fp32, bitwise, without the casts)
            h2, p2, n2 = _rows2d(h), _rows2d(ep), _rows2d(en)
        else:
            dt = torch.promote_types(torch.promote_types(h.dtype, ep.dtype), en.dtype)
            h2, p2, n2 = (_rows2d(x.to(dt)) for x in (h, ep, en))
        pos, neg, loss, count = K.pair_logits_fwd(h2, p2, n2, ntt, with_loss=True)
        ctx.save_for_backward(h2, p2, n2, pos, neg, ntt, count)
        ctx.dtypes = (h.dtype, ep.dtype, en.dtype)
        ctx.shapes = (h.shape, ep.shape, en.shape)
        return loss

    @staticmethod
    def backward(ctx, gloss):
        h2, p2, n2, pos, neg, ntt, count = ctx.saved_tensors
        need = ctx.needs_input_grad[:3]
        dh, dp, dn = K.pair_logits_bwd(h2, p2, n2, pos_logits=pos, neg_logits=neg, next_token_type=ntt, count=count,
                                       grad_loss=gloss, need=need, stacked=True)
        return _shape_grads(ctx, dh, dp, dn)


@_disable
def bce_loss(h, e_pos, e_neg, next_token_type):
    """Fused logits + the reference BCE loss (main.py:177-182), no host sync."""
    ntt = next_token_type.reshape(-1).to(torch.int32).contiguous()
    return _BCELossFn.apply(h, e_pos, e_neg, ntt)


# -------------------------------------------------------- sampled softmax ----
class _SampledSoftmaxFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, e, item_ids, valid, tau, log_q):
        hb = _rows2d(h.to(torch.bfloat16))
        eb = _rows2d(e.to(torch.bfloat16))
        loss, lse2, count = K.sampled_softmax_fwd(hb, eb, item_ids, valid, tau, log_q)
        ctx.save_for_backward(hb, eb, item_ids, valid, lse2, count, log_q)
        ctx.meta = (tau, h.shape, e.shape, h.dtype, e.dtype)
        return loss

    @staticmethod
    def backward(ctx, gloss):
        hb, eb, ids, valid, lse2, count, log_q = ctx.saved_tensors
        tau, hs, es, hdt, edt = ctx.meta
        dh, de = K.sampled_softmax_bwd(hb, eb, ids, valid, tau, lse2, gloss, log_q)
        dh = dh.view(hs).to(hdt) if ctx.needs_input_grad[0] else None
        de = de.view(es).to(edt) if ctx.needs_input_grad[1] else None
        return dh, de, None, None, None, None


@_disable
def sampled_softmax_loss(h, pos_emb, pos_ids, next_token_type, tau, log_q=None):
    """In-batch sampled softmax over every valid position's positive item
    (north star; oracle/loss.py::sampled_softmax): one flash-style MFMA pass
    for the loss, two fused passes (dH, dE) for the gradients, all over the
    valid positions only.  log_q (optional, [B, T] or [N], natural log): the
    logQ correction -- the log sampling probability of each position's item,
    subtracted from its column's logits (no gradient flows into it)."""
    ids = pos_ids.reshape(-1).to(torch.int64).contiguous()
    valid = (next_token_type.reshape(-1) == 1).to(torch.uint8).contiguous()
    if log_q is not None:
        log_q = log_q.detach().reshape(-1).to(torch.float32).contiguous()
    return _SampledSoftmaxFn.apply(h, pos_emb, ids, valid, float(tau), log_q)


def batch_log_q(pos_ids, next_token_type):
    """log q of each position's item estimated from the batch itself: log(count of
    the item among the valid positions / number of valid positions) -- the
    in-batch sampling probability of that item (the logQ correction when no
    corpus frequency table is given).  Device ops, no host sync."""
    ids = pos_ids.reshape(-1).to(torch.int64)
    valid = next_token_type.reshape(-1) == 1
    key = torch.where(valid, ids, torch.full_like(ids, -1))
    srt, inv = torch.sort(key)
    head = torch.ones_like(srt, dtype=torch.bool)
    head[1:] = srt[1:] != srt[:-1]
    run = torch.cumsum(head.to(torch.int64), 0) - 1                 # run index of each sorted entry
    counts = torch.zeros_like(srt).scatter_add_(0, run, torch.ones_like(srt))
    cnt = torch.empty_like(srt)
    cnt[inv] = counts[run]
    nv = valid.sum().clamp(min=1).to(torch.float32)
    return torch.where(valid, torch.log(cnt.to(torch.float32) / nv), torch.zeros_like(nv.expand_as(cnt)))
