"""Fused optimizer for the training step: table groups + dense AdamW.

The reference steps ``torch.optim.AdamW(model.parameters(), lr,
betas=(0.9, 0.98), weight_decay)`` over every parameter, embedding tables
included, with dense table gradients (``model/BaseLine/main.py:131,189``;
``model/BaseLineO1/main.py:174,249``).  Here:

* the embedding tables are packed into a few **table groups** (one flat
  ``[rows, D]`` buffer each; every ``nn.Embedding.weight`` becomes a view, so
  state_dict keys and values are unchanged).  Lookups push row-sparse
  gradient sources into their group; ``step()`` reduces each group with ONE
  deterministic ``grk_embedding_backward`` and updates it with ONE
  ``grk_table_adamw``.  ``table_mode="dense"`` moves every row exactly like
  the reference (rows without gradient still decay and update their
  moments); ``"lazy"`` touches only rows that received a gradient (a
  documented deviation);
* the remaining dense parameters use torch's fused AdamW.

Table storage dtype defaults to bf16 (BASELINE config 2); moments are fp32.
"""
from __future__ import annotations

import ctypes as C
import os
import weakref

import torch

from . import _lib as L
from . import functional as G
from . import kernels as K
from .streams import run_branches


class TableGroup:
    """Several tables in one flat buffer, with their AdamW state."""

    def __init__(self, name, tables, dtype, device):
        self.name = name
        # equal-sized tables adjacent (stable in the given order): the dnn
        # projections read each size class as one contiguous [G, rows, D] view
        tables = sorted(tables, key=lambda kv: kv[1].num_embeddings)
        D = tables[0][1].embedding_dim
        self.dim = D
        self.offsets = {}
        rows = 0
        for key, emb in tables:
            if emb.embedding_dim != D:
                raise ValueError('all tables of a group share the embedding dim')
            self.offsets[key] = rows
            rows += emb.num_embeddings
        self.rows = rows
        self.flat = torch.empty(rows, D, dtype=dtype, device=device)
        self.refs = {}
        for key, emb in tables:
            off = self.offsets[key]
            view = self.flat[off:off + emb.num_embeddings]
            with torch.no_grad():
                view.copy_(emb.weight.detach().to(device=device, dtype=dtype))
            emb.weight = torch.nn.Parameter(view, requires_grad=False)
            self.refs[key] = G.TableRef(emb.weight, self, off)
        self.exp_avg = torch.zeros(rows, D, dtype=torch.float32, device=device)
        self.exp_avg_sq = torch.zeros(rows, D, dtype=torch.float32, device=device)
        self.row_slot = torch.full((rows,), -1, dtype=torch.int32, device=device)
        self.pending = []
        self.token_type = None
        self.seq_len = 0
        self.dense_grads = {}  # row offset -> dense gradient of rows [off, off + len) (tables used in dense ops)
        self._identity = None

    def collect_dense(self, row_offset, grad):
        """Dense gradient (any float dtype) for rows [row_offset, row_offset + len(grad))."""
        prev = self.dense_grads.get(row_offset)
        if prev is not None and prev.shape == grad.shape:
            grad = prev.float() + grad
        elif prev is not None:
            raise RuntimeError(f'table group {self.name}: overlapping dense gradients at row {row_offset}')
        self.dense_grads[row_offset] = grad

    def identity(self):
        if self._identity is None:
            self._identity = torch.arange(self.rows, dtype=torch.int32, device=self.flat.device)
        return self._identity

    def dense_gradient(self, padding_idx=0):
        """fp32 [rows, D]: the row-sparse sources reduced densely plus the dense parts."""
        if self.pending:
            dense = K.embedding_backward(self.pending, self.rows, self.dim, padding_idx=padding_idx,
                                         token_type=self.token_type, seq_len=self.seq_len, dense=True).dense
        else:
            dense = torch.zeros(self.rows, self.dim, dtype=torch.float32, device=self.flat.device)
        for off, g in self.dense_grads.items():
            dense[off:off + g.shape[0]] += g
        return dense

    def step_dense_ranges(self, hp):
        """Dense-parity AdamW when every gradient of the group is dense (no
        row-sparse sources): each range from its own gradient (bf16 or fp32,
        no fp32 staging buffer), rows without gradient with g = 0."""
        pos = 0
        for off in sorted(self.dense_grads):
            g = self.dense_grads[off]
            if off > pos:
                K.table_adamw(self.flat[pos:off], self.exp_avg[pos:off], self.exp_avg_sq[pos:off], hp)
            end = off + g.shape[0]
            K.table_adamw_dense(self.flat[off:end], self.exp_avg[off:end], self.exp_avg_sq[off:end], hp, g)
            pos = end
        if pos < self.rows:
            K.table_adamw(self.flat[pos:], self.exp_avg[pos:], self.exp_avg_sq[pos:], hp)

    def collect(self, src, token_type, seq_len):
        self.pending.append(src)
        if token_type is not None:
            if self.token_type is not None and self.token_type is not token_type:
                raise RuntimeError(f'table group {self.name}: two masked lookups with different token_type in one step')
            self.token_type, self.seq_len = token_type, seq_len
        elif src.mode == 3:  # GRK_IDX_POSITION
            self.seq_len = seq_len

    def clear(self):
        self.pending = []
        self.token_type = None
        self.dense_grads = {}


# pos_emb (row-sparse gradients) apart from the feature tables, whose gradients
# are dense (they feed the dnns through projections: model._projection)
DEFAULT_GROUPS = (('item', ('item_emb',)), ('user', ('user_emb',)), ('pos', ('pos_emb',)), ('small', None))


# The rolling flush's per-step slice on a side stream (GRK_SLICE_SIDE=0: in line).
# Measured alternatives, not kept: the slice forked at the backward
# instead of the forward, a lower stream priority for it, the batch rows' catch-up on
# the same side stream.
SLICE_SIDE = os.environ.get('GRK_SLICE_SIDE', '1') != '0'
SLICE_SIDE_STREAM = 7

DENSE_FLAT_DIM = 8   # the flat buffer as [rows, 8] for k_adamw_ranges (16-byte fp32 pairs per lane)


def flat_layout(numels, dim=DENSE_FLAT_DIM):
    """Row offsets of tensors of the given sizes (each a multiple of dim) packed back
    to back in a [rows, dim] buffer: ([row_start...], total rows)."""
    starts, row = [], 0
    for n in numels:
        if n % dim:
            raise ValueError(f'a flat tensor holds a multiple of {dim} elements, not {n}')
        starts.append(row)
        row += n // dim
    return starts, row


def grad_runs(starts, ends, has_grad):
    """Maximal runs [(row_lo, row_hi, [indices])] of consecutive tensors that all have a
    gradient: torch's AdamW skips a parameter without one, so the multi-range update
    (which moves every row of its buffer) is launched per run, never over a gap."""
    runs, cur = [], None
    for i, ok in enumerate(has_grad):
        if not ok:
            cur = None
            continue
        if cur is None or cur[1] != starts[i]:
            cur = [starts[i], ends[i], []]
            runs.append(cur)
        cur[1] = ends[i]
        cur[2].append(i)
    return [tuple(r) for r in runs]


def aligned_rows(g):
    """g itself, or a copy when its fp32 rows are not 16-byte aligned (the multi-range
    kernel reads fp32 gradient rows as 16-byte vectors)."""
    if g.stride(-1) != 1 or (g.dtype == torch.float32 and (g.data_ptr() % 16 or g.stride(0) % 4)):
        return g.contiguous().clone()
    return g


def split_runs(runs, starts, ends, limit):
    """Runs of grad_runs cut into pieces of at most ``limit`` tensors (the multi-range
    kernel's cap); each piece's rows stay contiguous."""
    out = []
    for _lo, _hi, idx in runs:
        for k in range(0, len(idx), limit):
            part = idx[k:k + limit]
            out.append((starts[part[0]], ends[part[-1]], part))
    return out


class DenseFlat:
    """fp32 dense parameters as views of one [rows, 8] buffer with flat AdamW moments,
    stepped by grk_table_adamw_ranges_dev (each parameter's gradient one range).

    shadow=True: a bf16 copy of the buffer, written by the same AdamW launch, serves
    the GEMMs' bf16 weight operands (functional.bf16_shadow) instead of a cast kernel
    per weight and step.  Writes made outside the optimizer are detected by version
    counters and the shadow is refreshed before its next use: in-place ops on a
    parameter (load_state_dict, ``p.mul_``: p's own counter) and writes through ``buf``
    or any view of it (the counter every view of ``buf`` shares).  One kind of write
    cannot be seen: through ``p.data`` (a fresh counter each time) -- call
    ``sync_shadow(force=True)`` after such writes.  Refreshes write the shadow through
    a ``.data`` alias, so they never bump the counter the shadow views share: a view
    an earlier GEMM saved for backward stays valid."""

    def __init__(self, params, device, shadow=False):
        self.params = list(params)
        self.starts, rows = flat_layout([p.numel() for p in self.params])
        self.ends = [s + p.numel() // DENSE_FLAT_DIM for s, p in zip(self.starts, self.params)]
        self.buf = torch.empty(rows, DENSE_FLAT_DIM, dtype=torch.float32, device=device)
        for p, s, e in zip(self.params, self.starts, self.ends):
            view = self.buf[s:e].view(p.shape)
            with torch.no_grad():
                view.copy_(p.detach())
            p.data = view            # the Parameter object (and the model's references) stays
        self.exp_avg = torch.zeros_like(self.buf)
        self.exp_avg_sq = torch.zeros_like(self.buf)
        self._ptrs = [p.data_ptr() for p in self.params]
        self._prep_key, self._prepared = None, []
        self.shadow = None
        if shadow:
            self.shadow = self.buf.to(torch.bfloat16)
            self._index = {id(p): i for i, p in enumerate(self.params)}
            self._versions = [p._version for p in self.params]
            self._buf_version = self.buf._version
            G.register_shadows(self.params, self)

    def _refresh_all(self):
        with torch.no_grad():
            self.shadow.data.copy_(self.buf)
        self._versions = [p._version for p in self.params]
        self._buf_version = self.buf._version

    def sync_shadow(self, force=False):
        """Refresh the shadow of every parameter changed outside the optimizer (a
        graph replay reads the shadow without running the Python forward);
        force=True recasts all of it (after writes through ``p.data``)."""
        if self.shadow is None:
            return
        if force or self.buf._version != self._buf_version:
            self._refresh_all()
            return
        for p, ver in zip(self.params, self._versions):
            if p._version != ver:
                self.shadow_of(p)

    def shadow_of(self, p):
        """bf16 view of p's rows in the shadow buffer, refreshed first if p changed
        outside the optimizer since the shadow last matched it."""
        i = self._index[id(p)]
        if p.data_ptr() != self._ptrs[i]:
            return None        # no longer lives in the flat buffer (DenseFlat.step refuses too)
        if self.buf._version != self._buf_version:
            self._refresh_all()
        s, e = self.starts[i], self.ends[i]
        view = self.shadow[s:e].view(p.shape)
        if p._version != self._versions[i]:
            with torch.no_grad():
                view.data.copy_(p.detach())
            self._versions[i] = p._version
        return view

    def zero_grad(self, set_to_none=True):
        for p in self.params:
            if set_to_none:
                p.grad = None
            elif p.grad is not None:
                p.grad.zero_()

    def step(self, clock):
        if any(p.data_ptr() != q for p, q in zip(self.params, self._ptrs)):
            # e.g. model.to() / load_state_dict(assign=True) after the optimizer was built:
            # the update would land in the old buffer
            raise RuntimeError('dense_flat: a parameter no longer lives in the flat buffer')
        grads = [p.grad for p in self.params]
        # the launches' arguments are kept while every gradient is the same storage
        # as last step (row-sharded: views of the all-reduce buckets; graph replays):
        # rebuilding the ctypes range arrays of ~50 parameters costs more host time
        # than the update takes on the device
        key = (tuple(None if g is None else (g.data_ptr(), g.dtype, g.is_contiguous()) for g in grads),
               id(clock))
        if key == self._prep_key:
            for call in self._prepared:
                K.launch_prepared(call)
            return
        calls, reusable = [], True
        for lo, hi, idx in split_runs(grad_runs(self.starts, self.ends, [g is not None for g in grads]),
                                      self.starts, self.ends, K.MAX_GRAD_RANGES):
            ranges = []
            for i in idx:
                g = grads[i]
                if g.dtype not in (torch.float32, torch.bfloat16):
                    g, reusable = g.float(), False
                if not g.is_contiguous():
                    g, reusable = g.contiguous(), False
                if g.data_ptr() % 16:          # the kernel reads fp32 gradients as 16-byte vectors
                    g, reusable = g.clone(), False
                ranges.append((self.starts[i] - lo, g.view(-1, DENSE_FLAT_DIM)))
            calls.append(K.prepare_table_adamw_ranges(self.buf[lo:hi], self.exp_avg[lo:hi], self.exp_avg_sq[lo:hi],
                                                      clock, ranges,
                                                      shadow=None if self.shadow is None else self.shadow[lo:hi]))
        for call in calls:
            K.launch_prepared(call)
        # copies made for the launch are fresh each step: only a copy-free plan is kept
        self._prep_key, self._prepared = (key, calls) if reusable else (None, [])

    def state(self, p):
        """{'exp_avg', 'exp_avg_sq'} views of parameter p (torch AdamW's state names)."""
        i = next(i for i, q in enumerate(self.params) if q is p)
        s, e = self.starts[i], self.ends[i]
        return {'exp_avg': self.exp_avg[s:e].view(p.shape), 'exp_avg_sq': self.exp_avg_sq[s:e].view(p.shape)}


class FusedAdamW:
    """AdamW over a BaselineModel: table groups on grk kernels, dense params on torch fused AdamW."""

    def __init__(self, model, lr=1e-3, betas=(0.9, 0.98), eps=1e-8, weight_decay=0.01, table_mode='dense',
                 table_dtype=torch.bfloat16, groups=DEFAULT_GROUPS, defer_period=16, l2_emb=0.0, parallel=False,
                 dense_flat=True, rolling=True):
        """l2_emb > 0: the BaseLine script's ``loss += l2_emb * ||item_emb.weight||_F``
        (model/BaseLine/main.py:184-185) -- ``l2_term()`` gives the loss term (Trainer
        adds it), ``step()`` adds its gradient l2 * W / ||W|| to every item row.  Every
        row then moves every step, so the item table is updated densely (not deferred).

        dense_flat=True (GPU; the default since round 4, measured -0.06 ms per C2 step):
        the fp32 dense parameters whose sizes are multiples of 8 become views of ONE flat
        buffer (DenseFlat) updated by grk's multi-range AdamW (one k_adamw_ranges launch
        per run of <= 64 parameters with a gradient) instead of torch's fused AdamW
        (~0.14-0.19 ms per C2 step).  The element update is the tables' (hardware sqrt /
        reciprocal): within a few ulp of torch's.  A parameter without a
        gradient in a step is not moved (torch's rule); its bias correction afterwards
        follows the global step (the device clock) where torch counts each parameter's
        steps -- the same whenever every dense parameter gets a gradient every step, as
        in the model's training step.

        rolling=True (the default since round 5; deferred tables only): the deferred
        rows are flushed ROLLING -- every step brings one 1/defer_period slice of each
        deferred table up to date inside the step (grk_table_adamw_catchup_slice_dev,
        captured with the step), so every row is replayed at least every defer_period
        steps at a constant per-step cost, instead of all rows at once at every
        defer_period-th step between graph replays (a ~5.7 ms spike at C2 that made a
        timed window's cost depend on how many segment starts it held).  Same values
        bit for bit: a replayed g = 0 step does not depend on when it runs.  The ring
        then holds 2 x defer_period steps (the pending steps behind a row and the
        steps ahead)."""
        if table_mode not in ('dense', 'lazy'):
            raise ValueError("table_mode must be 'dense' or 'lazy'")
        self.l2_emb = float(l2_emb)
        # parallel=True: step()'s independent updates as parallel stream branches.  Off by
        # default: measured on MI355X / ROCm 7.2, a captured step with these branches
        # replays SLOWER (6.6 vs 5.0 ms per step, host issue spikes of 10 ms) -- the
        # multi-stream graph costs more than the overlap of the small kernels saves
        self.parallel = bool(parallel)
        if self.l2_emb and table_mode == 'lazy':
            raise ValueError('l2_emb moves every item row each step: it needs table_mode="dense"')
        self.model = model
        self.lr, self.betas, self.eps, self.weight_decay = lr, betas, eps, weight_decay
        self.lazy = table_mode == 'lazy'
        dev = model.item_emb.weight.device
        tables = model.table_modules()
        taken, self.groups, refs = set(), [], {}
        for gname, keys in groups:
            keys = [k for k in tables if k not in taken] if keys is None else list(keys)
            if not keys:
                continue
            taken.update(keys)
            grp = TableGroup(gname, [(k, tables[k]) for k in keys], table_dtype, dev)
            self.groups.append(grp)
            refs.update(grp.refs)
        model._table_refs = refs
        dense = [p for p in model.parameters() if p.requires_grad]
        cuda = dev.type == 'cuda'
        self._flat = None
        if dense_flat and cuda:
            flat_ps = [p for p in dense if p.dtype == torch.float32 and p.numel() % DENSE_FLAT_DIM == 0]
            if flat_ps:
                self._flat = DenseFlat(flat_ps, dev, shadow=True)
                dense = [p for p in dense if all(p is not q for q in flat_ps)]
        # capturable: the dense AdamW keeps its step count on the device, so the
        # whole training step can be captured in a HIP graph (train.Trainer)
        self.dense = torch.optim.AdamW(dense, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                                       fused=cuda, capturable=cuda) if dense else None
        self.t = 0
        # Deferred dense parity for the big item/user tables: a row outside the
        # step's batch takes a g = 0 update that depends on nothing but (p, m, v)
        # and the step's hyper-parameters, so it is replayed in registers when
        # the row is next read (begin_step: the batch rows), at every
        # `defer_period`-th step for all rows, and before state_dict (flush) --
        # bit-identical to moving every row every step, without streaming the
        # whole table through HBM each step.  Needs Trainer.step (begin_step).
        self.defer = int(defer_period) if (defer_period and not self.lazy and cuda) else 0
        deferrable = ('user',) if self.l2_emb else ('item', 'user')
        self._deferred = {g.name: g for g in self.groups if g.name in deferrable} if self.defer else {}
        self._seg = None     # step every deferred row was last brought up to (segment start)
        self._begun = None   # step for which begin_step caught the batch rows up
        for g in self._deferred.values():
            g.last = torch.zeros(g.rows, dtype=torch.int32, device=dev)
        # The table kernels read the step and its hyper-parameters on the device
        # (K.DeviceClock): the ring holds the steps of the current segment,
        # refilled at segment starts from alternating pinned buffers.
        self.rolling = bool(rolling) and bool(self._deferred)
        self.clock = K.DeviceClock((2 if self.rolling else 1) * (self.defer or 16), dev) if cuda else None
        if self.clock is not None:
            self._pinned = [torch.zeros_like(self.clock.ring, device='cpu').pin_memory() for _ in range(2)]
            self._uploads = 0
        self._l2_group = next((g for g in self.groups if g.name == 'item'), None) if self.l2_emb else None
        if self.l2_emb and (self._l2_group is None or self.clock is None):
            raise ValueError('l2_emb needs the item table in a table group on the GPU')
        if self._l2_group is not None:
            self._l2_norm = torch.zeros(1, dtype=torch.float32, device=dev)
            self._l2_coef = torch.zeros(1, dtype=torch.float32, device=dev)
        self._l2_ready = None  # step whose norm / gradient scale l2_term computed
        if self.defer:
            model.register_state_dict_pre_hook(lambda *args, **kw: self.flush())
            if hasattr(model, '_flushers'):  # predict / save_item_emb / eval() read fresh rows
                model._flushers.append(weakref.WeakMethod(self.flush))

    @property
    def _ring(self):
        return self.clock.ring

    def _hp(self, step):
        return K.adamw_hparams(self.lr, self.betas[0], self.betas[1], self.eps, self.weight_decay, step)

    @property
    def _period(self):
        """Steps between segment starts (ring refills; full flushes unless rolling)."""
        return self.clock.ring_len // 2 if self.rolling else self.clock.ring_len

    def _upload_ring(self, t):
        """Hyper-parameters of steps t+1 .. t+period into the device ring (slot s % ring_len);
        rolling: also steps t-period+1 .. t, which rows behind by up to a period replay."""
        n = self.clock.ring_len
        k = self._uploads % 2  # alternate buffers; the host may run many (graph-replayed) steps ahead
        self._uploads += 1
        done = getattr(self, '_pinned_done', None)
        if done is None:
            done = self._pinned_done = [None, None]
        if done[k] is not None:
            done[k].synchronize()  # the copy out of this buffer two segments ago has run
        buf = self._pinned[k]
        lo = t - n // 2 + 1 if self.rolling else t + 1
        for step in range(max(lo, 1), lo + n):
            hp = self._hp(step)
            buf[step % n] = torch.tensor([getattr(hp, f) for f, _ in hp._fields_], dtype=torch.float32)
        self.clock.ring.copy_(buf, non_blocking=True)
        done[k] = torch.cuda.Event()
        done[k].record()

    def _segment(self, t):
        """Start a new segment at step t: bring every deferred row to t (not when rolling:
        the per-step slices do), refill the ring."""
        if self._seg is not None and self._seg < t and not self.rolling:
            for g in self._deferred.values():
                K.table_adamw_catchup(g.flat, g.exp_avg, g.exp_avg_sq, g.last, None, self.clock)
        self._upload_ring(t)
        self._seg = t

    def maybe_segment(self):
        """Host-side segment bookkeeping due before step self.t + 1 (eager; never inside a captured step).
        Also brings the dense weights' bf16 shadows up to date with writes made outside
        the optimizer (load_state_dict between graph replays)."""
        if self._flat is not None:
            self._flat.sync_shadow()
        if self.clock is not None and (self._seg is None or self.t - self._seg >= self._period):
            self._segment(self.t)

    def graph_replayed(self):
        """Host state after a replay of a captured step (the device state advanced inside the graph)."""
        self.t += 1
        self._begun = None

    @torch.no_grad()
    def begin_step(self, batch):
        """Bring the rows the coming step reads up to date (deferred tables).

        batch = (seq, pos, neg, token_type, ...) as Trainer.step gets it: the
        item table's rows are seq (item tokens), pos and neg; the user table's
        are seq (user tokens)."""
        self.maybe_segment()
        if not self._deferred:
            return
        # Padding (id 0, and tokens of the other type) -> -1, skipped by the kernel:
        # thousands of duplicate claims on row 0 would serialise on one atomic.
        # The padding row is brought up at the segment flush; it is zero and gets
        # no gradient (nn.Embedding padding_idx), and a g = 0 step maps a zero
        # (p, m, v) row to exactly zero, so reading it early changes nothing.
        side = self.rolling and SLICE_SIDE and not self.l2_emb and self.clock.ring.is_cuda
        item, user = K.batch_row_ids(*batch[:4], with_user='user' in self._deferred)
        ids = {'item': item, 'user': user}
        for name, g in self._deferred.items():
            if self.rolling and not side:   # this step's slice of every row
                K.table_adamw_catchup_slice(g.flat, g.exp_avg, g.exp_avg_sq, g.last, self.clock, self._period)
            K.table_adamw_catchup(g.flat, g.exp_avg, g.exp_avg_sq, g.last, None, self.clock, ids[name])
        if side:
            # the slice after the batch rows (which it then skips: their step stamps are
            # current) on a side stream: VALU-bound replay under the step's GEMMs and
            # attention; no kernel of the step reads or writes the rows it touches (the
            # gathers read batch rows only), joined before step() updates any row
            def slices():
                for g in self._deferred.values():
                    K.table_adamw_catchup_slice(g.flat, g.exp_avg, g.exp_avg_sq, g.last, self.clock, self._period)
            G.run_on_side(slices, self.clock.ring.device, SLICE_SIDE_STREAM)
        self._begun = self.t

    @torch.no_grad()
    def l2_term(self):
        """l2_emb * ||item_emb.weight||_F at the current parameters (a device scalar, no
        host sync) -- the BaseLine loss term; its gradient goes straight into the
        item table's AdamW in step()."""
        if not self.l2_emb:
            return None
        g = self._l2_group
        K.table_l2_norm(g.flat, self.l2_emb, self._l2_norm, self._l2_coef)
        self._l2_ready = self.t
        return (self.l2_emb * self._l2_norm).reshape(())

    @torch.no_grad()
    def flush(self):
        """Bring every row of the deferred tables to the current step (before reading them)."""
        G.join_side_work()
        if self._deferred and self._seg is not None:
            for g in self._deferred.values():
                K.table_adamw_catchup(g.flat, g.exp_avg, g.exp_avg_sq, g.last, None, self.clock)

    def zero_grad(self, set_to_none=True):
        if self.dense is not None:
            self.dense.zero_grad(set_to_none=set_to_none)
        if self._flat is not None:
            self._flat.zero_grad(set_to_none)
        for g in self.groups:
            g.clear()

    @torch.no_grad()
    def step(self):
        G.join_side_work()   # the flush slice still running on its side stream
        self.maybe_segment()
        if self._deferred and self._begun != self.t:  # no begin_step: every row to step t, then dense
            self.flush()
        begun, self._begun = self._begun == self.t, None
        if self.l2_emb and self._l2_ready != self.t:   # no l2_term this step: its gradient scale now
            self.l2_term()
        self._l2_ready = None
        self.t += 1
        if self.clock is not None:
            self.clock.advance()
        hp = self.clock if self.clock is not None else self._hp(self.t)
        # the dense AdamW and every table group's reduction + update are independent
        # chains of (mostly small) kernels: on the GPU they run as parallel branches
        # (private streams forked from and joined into the step's stream)
        work = [self._dense_step(hp)] + [self._group_work(g, hp, begun) for g in self.groups]
        dev = self.groups[0].flat.device if self.groups else torch.device('cpu')
        if self.parallel and self.clock is not None:
            run_branches(work, dev)
        else:
            for f in work:
                f()

    def _dense_step(self, hp):
        """The dense parameters' update this step, as a closure (run_branches)."""
        def work():
            if self.dense is not None:
                self.dense.step()
            if self._flat is not None:
                self._flat.step(hp)
        return work

    def _group_work(self, g, hp, begun):
        """The update of one table group this step, as a closure (run_branches)."""
        def work():
            self._group_step(g, hp, begun)
        return work

    def _group_step(self, g, hp, begun):
        if g.name in self._deferred:
            if begun:  # rows outside the batch stay deferred; the batch rows move now
                if g.pending:
                    res = K.embedding_backward(g.pending, g.rows, g.dim, padding_idx=0, token_type=g.token_type,
                                               seq_len=g.seq_len, dense=False, sparse=True, row_slot=g.row_slot)
                    K.table_adamw(g.flat, g.exp_avg, g.exp_avg_sq, hp, res.ids, res.rows, res.count,
                                  res.capacity, g.row_slot, lazy=True)
                    K.stamp_rows(g.last, res.ids, res.count, res.capacity, self.clock)
                g.clear()
                return
            g.last.fill_(self.t)  # dense update below moves every row
        if g is self._l2_group:  # every row: its sparse gradient + l2 * p / ||W||
            res = None
            if g.pending:
                res = K.embedding_backward(g.pending, g.rows, g.dim, padding_idx=0, token_type=g.token_type,
                                           seq_len=g.seq_len, dense=False, sparse=True, row_slot=g.row_slot)
            if g.dense_grads:
                raise RuntimeError('l2_emb: the item table takes row-sparse gradients only')
            if res is None:
                K.table_adamw_l2(g.flat, g.exp_avg, g.exp_avg_sq, self.clock, self._l2_coef)
            else:
                K.table_adamw_l2(g.flat, g.exp_avg, g.exp_avg_sq, self.clock, self._l2_coef, res.ids, res.rows,
                                 res.count, res.capacity, g.row_slot)
            g.clear()
            return
        if g.dense_grads and not g.pending and isinstance(hp, K.DeviceClock) \
                and len(g.dense_grads) <= K.MAX_GRAD_RANGES:  # dense gradient blocks only: one multi-range launch
            K.table_adamw_ranges(g.flat, g.exp_avg, g.exp_avg_sq, hp,
                                 [(off, aligned_rows(x)) for off, x in g.dense_grads.items()])
        elif g.dense_grads and not g.pending:  # dense gradients only: per-range updates
            g.step_dense_ranges(hp)
        elif g.dense_grads:  # mixed: one dense fp32 gradient
            K.table_adamw(g.flat, g.exp_avg, g.exp_avg_sq, hp, None, g.dense_gradient(), None, 0, g.identity())
        elif g.pending:
            res = K.embedding_backward(g.pending, g.rows, g.dim, padding_idx=0, token_type=g.token_type,
                                       seq_len=g.seq_len, dense=False, sparse=True, row_slot=g.row_slot)
            K.table_adamw(g.flat, g.exp_avg, g.exp_avg_sq, hp, res.ids, res.rows, res.count, res.capacity,
                          None if self.lazy else g.row_slot, lazy=self.lazy)
        elif not self.lazy:
            K.table_adamw(g.flat, g.exp_avg, g.exp_avg_sq, hp)
        g.clear()
