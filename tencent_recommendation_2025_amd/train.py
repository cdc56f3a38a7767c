"""Training step of the TencentGR script on the grk path (model/BaseLine/main.py:163-190;
model/BaseLineO1/main.py:200-250): forward, loss, backward, optimizer -- with
no host synchronisation inside the step (the reference's ``np.where`` index
set and ``loss.item()`` are replaced by device-side counts).

Because the step never waits on the device, it can be captured once as a HIP
graph and replayed (``graph=True``): the ~470 kernel launches and all the
Python between them collapse into one graph launch per step, so the host no
longer paces the GPU.  Everything step-dependent lives on the device: the
table kernels read the step and its hyper-parameters from the optimizer's
``DeviceClock``, torch's AdamW runs ``capturable``, and the batch is copied
into the captured input buffers before each replay.  Segment work of the
deferred table updates (every ``defer_period`` steps) runs eagerly between
replays.

With row-sharded tables (sharding.ShardedFusedAdamW) the all-to-all sizes
change every step, so only the forward + backward is captured: the row
exchange (``prepare``, into fixed buffers) runs eagerly before each replay and
the gradient exchange + updates (``step``) after it.  Passing the next batch
(``step(batch, next_batch)``) routes it one step ahead, so no step waits for
the device to drain before its all-to-alls."""
from __future__ import annotations

import contextlib

import torch

from . import _lib as L
from . import functional as G
from . import jagged as J
from . import kernels as K
from . import streams as S


def private_stream(device):
    """The process's own capture stream for ``device`` (streams.private_stream):
    never one of torch's pooled streams, which a process group may record its
    collectives' events on."""
    return S.private_stream(device, 0)


def _tensors(batch):
    """Flat list of the batch's tensors (tuple items and dict values, in order)."""
    out = []
    for x in batch:
        if isinstance(x, torch.Tensor):
            out.append(x)
        elif isinstance(x, dict):
            out.extend(v for _, v in sorted(x.items()) if isinstance(v, torch.Tensor))
    return out


class PackedBatch(tuple):
    """A batch whose tensors are views of ONE byte arena (pack_batch): a graph
    replay's input copy is then a single copy of the arena instead of a
    multi-tensor copy per dtype over ~70 tensors (~83 us per C2 step measured)."""
    arena: torch.Tensor
    layout: tuple


_ARENA_ALIGN = 256


def _arena_layout(tensors):
    offs, off = [], 0
    for t in tensors:
        offs.append(off)
        off += -(-t.numel() * t.element_size() // _ARENA_ALIGN) * _ARENA_ALIGN
    return offs, off


def _rebuild(batch, views):
    """batch's structure with its tensors (in _tensors order) replaced by views."""
    it = iter(views)
    res = []
    for x in batch:
        if isinstance(x, torch.Tensor):
            res.append(next(it))
        elif isinstance(x, dict):
            d = dict(x)
            for k, v in sorted(x.items()):
                if isinstance(v, torch.Tensor):
                    d[k] = next(it)
            res.append(d)
        else:
            res.append(x)
    return res


def _views(arena, tensors, offs):
    out = []
    for t, o in zip(tensors, offs):
        nb = t.numel() * t.element_size()
        out.append(arena[o:o + nb].view(t.dtype).view(t.shape))
    return out


def pack_batch(batch):
    """The batch with every tensor moved into one arena on its device (same values,
    dtypes and shapes; contiguous views).  All tensors must share one device."""
    ts = _tensors(batch)
    if not ts or len({t.device for t in ts}) != 1:
        raise ValueError('pack_batch: a batch with tensors on one device')
    offs, total = _arena_layout(ts)
    arena = torch.empty(total, dtype=torch.uint8, device=ts[0].device)
    views = _views(arena, ts, offs)
    for v, t in zip(views, ts):
        v.copy_(t)
    out = PackedBatch(_rebuild(batch, views))
    out.arena = arena
    out.layout = tuple((o, t.dtype, tuple(t.shape)) for o, t in zip(offs, ts))
    return out


def _clone_batch(batch):
    if isinstance(batch, PackedBatch):
        ts = _tensors(batch)
        arena = batch.arena.clone()
        out = PackedBatch(_rebuild(batch, _views(arena, ts, [o for o, _, _ in batch.layout])))
        out.arena, out.layout = arena, batch.layout
        return out
    res = []
    for x in batch:
        if isinstance(x, torch.Tensor):
            res.append(x.clone())
        elif isinstance(x, dict):
            res.append({k: (v.clone() if isinstance(v, torch.Tensor) else v) for k, v in x.items()})
        else:
            res.append(x)
    return tuple(res)


def jagged_remaps(remaps, parts, row_map, token_type=None):
    """Row-sharded tables + jagged rows: the remaps ShardedFusedAdamW.prepare built
    for the [B, T] batch ({(table, role, mode): (fetched rows, fetched-row index
    [B, T])}) re-indexed to the jagged order -- index[r] = index[row_map[r]].  A row
    past the span rows (row_map -1, a dead row: zero ids, no loss term, exact-zero
    gradient) reads the fetched row of the role's first padding id, as its zero id
    would.  ``parts``: ShardedFusedAdamW._parts(batch) (each role's ids).  Device
    ops only (no host sync: capturable)."""
    ids = {(name, role, mode): v for name, plist in parts.items() for role, _, mode, v in plist}
    if row_map.is_cuda and token_type is not None:
        # every role in one grk_jagged_remap launch (was ~8 torch kernels per role)
        raw = {(name, role, mode): idx for name, plist in parts.items() for role, idx, mode, _ in plist}
        want = {L.IDX_ITEM_MASK: 1, L.IDX_USER_MASK: 2}
        keys = [k for k in remaps if k in raw]
        roles = [(remaps[k][1], raw[k], token_type if k[2] in want else None, want.get(k[2], 0)) for k in keys]
        outs = K.jagged_remap(roles, row_map)
        return {k: (remaps[k][0], o.unsqueeze(0)) for k, o in zip(keys, outs)}
    rm = row_map.long()
    src = rm.clamp(min=0)
    out = {}
    for key, (ref, inv) in remaps.items():
        flat = inv.reshape(-1)
        v = ids.get(key)
        if v is None:   # a derived role (feat2emb_pair's 'pair' is rebuilt from pos / neg)
            continue
        pad = torch.argmax((v().reshape(-1) == 0).to(torch.int8))   # first padding position (0 if none)
        # index_select with a 1-element index: flat[pad] with a 0-d tensor would read it on
        # the host (a sync, illegal while the step is being captured)
        out[key] = (ref, torch.where(rm >= 0, flat[src], flat.index_select(0, pad.reshape(1))).unsqueeze(0))
    return out


class Trainer:
    """``step(batch)`` = one training step on a tensorised batch
    (``MyDataset.collate_tensor_fn`` layout, tensors on the device).

    loss: "bce" -- the reference loss (pos/neg BCE, main.py:177-182);
          "sampled_softmax" -- north-star in-batch sampled softmax.
    log_q (sampled softmax): the logQ correction -- None (off), "batch" (each
          item's in-batch frequency, functional.batch_log_q) or a tensor of
          per-item log sampling probabilities [num_items + 1] indexed by item id.
    graph: capture the step in a HIP graph after ``graph_warmup`` eager steps
          and replay it (needs a fused optimizer with a device clock and batches
          of one fixed shape; a batch of another shape runs eagerly).  Dropout
          seeds are drawn on the device (model.dropout_seed), so dropout runs
          inside the replayed step.
    jagged: run the token-wise step on each sequence's span [first valid token,
          T) only, packed back to back (jagged.py; the padding rows before it are
          dead in the reference), in ``capacity_for(span rows, jagged_quantum)``
          rows.  ``step(batch, rows=n)`` takes the batch's span-row count from the
          caller (jagged.span_rows; computed with one host sync otherwise).  With
          graph=True one HIP graph is captured per capacity (sharing one memory pool).
    """

    def __init__(self, model, optimizer, loss='bce', amp_dtype=torch.bfloat16, temperature=0.05, graph=False,
                 graph_warmup=3, graph_audit=False, log_q=None, jagged=False, jagged_quantum=1024):
        if loss not in ('bce', 'sampled_softmax'):
            raise ValueError("loss must be 'bce' or 'sampled_softmax'")
        if log_q is not None and (loss != 'sampled_softmax' or not (isinstance(log_q, torch.Tensor) or log_q == 'batch')):
            raise ValueError("log_q: None, 'batch' or a per-item tensor, with loss='sampled_softmax'")
        self.log_q = log_q
        self.model, self.opt, self.loss_kind = model, optimizer, loss
        self.amp_dtype, self.temperature = amp_dtype, temperature
        self.graph, self.graph_warmup = bool(graph), int(graph_warmup)
        self.graph_audit = bool(graph_audit)  # keep the captured graph and census its nodes (graph_nodes)
        self.graph_nodes = None
        self._seeds = {}   # cached backward seeds (_backward)
        if self.graph:
            why = self._graph_blocker()
            if why:
                raise ValueError(f'graph=True: {why}')
        self._g = None
        self._static = None
        self._static_loss = None
        self._graphs = {}        # capacity (jagged) or None -> (graph, static batch, static loss)
        self._cap_states = {}    # row-sharded: capacity -> the optimizer's capture_state() of that graph
        self._warm = {}
        self._pool = None
        self._side = None
        self._sharded = hasattr(optimizer, 'prepare')
        self.jagged, self.jagged_quantum = bool(jagged), int(jagged_quantum)
        self._cap = None         # jagged capacity of the current step (set by step(), cleared after it)
        self._jag_err = None     # jagged layout error flags, OR-ed over steps (int32 [1], device)
        self._err_host = None    # pinned copy of the flags, polled every ERR_POLL graph replays
        self._err_evt = None     # event after the copy into _err_host (None: no copy in flight)
        self._replays = 0

    def _graph_blocker(self):
        if not torch.cuda.is_available():
            return 'needs a GPU'
        if getattr(self.opt, 'clock', None) is None:
            return 'the optimizer must keep a device clock (optim.FusedAdamW on the GPU)'
        return None

    def compute_loss(self, batch):
        """batch: the nine collate_fn fields (dataset.py), optionally a tenth --
        int64 [B, T] event times for the HSTU time bias (model.hstu_time_buckets)."""
        seq, pos, neg, tt, ntt, _nat, sf, pf, nf = batch[:9]
        ts = batch[9] if len(batch) > 9 else None
        amp = (torch.autocast('cuda', dtype=self.amp_dtype) if self.amp_dtype is not None
               else contextlib.nullcontext())
        jag = pidx = None
        if self.jagged:
            # a direct compute_loss / eager_step call (no step()) counts the batch's rows itself
            cap = self._cap if self._cap is not None else J.capacity_for(J.span_rows(tt), self.jagged_quantum)
            if self._jag_err is None:
                self._jag_err = torch.zeros(1, dtype=torch.int32, device=tt.device)
            # rows under-stated by the caller: the layout drops the spans past cap (no kernel
            # addresses a row beyond it) and raises err bit 2, checked by check_jagged()
            jag = J.layout(tt, cap, ntt, err=self._jag_err)
            if self._sharded and getattr(self.model, '_remaps', None) is not None:
                # prepare() routed the [B, T] batch: its lookups' fetched-row indices follow
                # the batch into the jagged row order
                self.model._remaps = jagged_remaps(self.model._remaps, self.opt._parts(batch), jag.row_map,
                                                   batch[3])
            seq, pos, neg, tt, ntt, _nat, sf, pf, nf, ts, pidx = J.compact(batch, jag)
        with amp:
            h, pe, ne = self.model.encode(seq, pos, neg, tt, sf, pf, nf, timestamps=ts, jagged=jag, pos_idx=pidx)
            if self.loss_kind == 'bce':
                loss = G.bce_loss(h, pe, ne, ntt)
            else:
                lq = None
                if isinstance(self.log_q, torch.Tensor):
                    lq = self.log_q.to(pos.device)[pos.long()]
                elif self.log_q == 'batch':
                    lq = G.batch_log_q(pos, ntt)
                loss = G.sampled_softmax_loss(h, pe, pos, ntt, self.temperature, log_q=lq)
        # BaseLine's l2_emb * ||item_emb.weight|| (main.py:184-185): value here, gradient in the optimizer
        l2 = self.opt.l2_term() if getattr(self.opt, 'l2_emb', 0.0) else None
        return loss if l2 is None else loss + l2

    def _backward(self, loss):
        """loss.backward() seeded with a cached ones tensor: autograd's own seed is a
        fill kernel per step (inside the captured graph too)."""
        key = (loss.shape, loss.dtype, loss.device)
        seed = self._seeds.get(key)
        if seed is None:
            seed = self._seeds[key] = torch.ones_like(loss)
        loss.backward(seed)

    def eager_step(self, batch, next_batch=None):
        self.opt.zero_grad()
        if hasattr(self.opt, 'prepare'):  # row-sharded tables: fetch this batch's rows from their owners
            self.opt.prepare(batch)
            if next_batch is not None:
                self.opt.prefetch(next_batch)
        if hasattr(self.opt, 'begin_step'):  # deferred table updates: bring this batch's rows up to date
            self.opt.begin_step(batch)
        loss = self.compute_loss(batch)
        self._backward(loss)
        self.opt.step()
        if self.jagged and not torch.cuda.is_current_stream_capturing():
            self.check_jagged()   # eager: one host sync per step
        return loss.detach()

    ERR_POLL = 4

    def check_jagged(self):
        """Raise ValueError if any jagged layout so far flagged an error (host sync)."""
        if self._jag_err is not None:
            J.check_error(self._jag_err)

    def _poll_jagged(self):
        """Graph replays: every ERR_POLL replays (one copy in flight at a time) the flags
        are copied to pinned memory behind an event; the copy is read only once its
        event has completed (event query: no host wait).  An error (e.g. a jagged
        capacity overflow from under-stated ``rows``: the trailing spans were dropped)
        therefore raises within about ERR_POLL + the host's lead in replays -- those
        steps have trained on the truncated batch.  check_jagged() reads the flags
        synchronously."""
        if self._jag_err is None:
            return
        self._replays += 1
        if self._err_evt is not None and self._err_evt.query():
            self._err_evt = None
            if int(self._err_host[0]):
                J.check_error(self._err_host)
        if self._err_evt is None and self._replays % self.ERR_POLL == 0:
            if self._err_host is None:
                self._err_host = torch.zeros(1, dtype=torch.int32).pin_memory()
            self._err_host.copy_(self._jag_err, non_blocking=True)
            self._err_evt = torch.cuda.Event()
            self._err_evt.record()

    def step(self, batch, next_batch=None, rows=None):
        """One training step; ``next_batch`` (optional) is the batch of the following
        step, routed ahead when the tables are row-sharded.  ``rows`` (jagged): the
        batch's span-row count (jagged.span_rows), known to the host."""
        key = None
        if self.jagged:
            n = int(rows) if rows is not None else J.span_rows(batch[3])
            self._cap = key = J.capacity_for(n, self.jagged_quantum)
        try:
            return self._step(batch, next_batch, key)
        finally:
            self._cap = None

    def _step(self, batch, next_batch, key):
        if not self.graph:
            return self.eager_step(batch, next_batch)
        entry = self._graphs.get(key)
        if entry is None:
            warm = self._warm.get(key, 0)
            # the first graph: graph_warmup eager steps; a later capacity only needs its
            # GEMM plans tuned (one eager step of that shape)
            if warm < (self.graph_warmup if not self._graphs else 1):
                # warm-up on the stream the capture will use: GEMM plans tuned,
                # per-stream workspaces and the caching allocator's blocks in place.
                # Row-sharded: on the current stream -- its collectives must never run
                # on the capture stream (the process group's watchdog polls their
                # events; polling one recorded on a stream that is now capturing is
                # fatal, seen when a second capacity was warmed up and captured at
                # once); the capture stream gets its GEMM workspace in _capture.
                self._warm[key] = warm + 1
                if self._sharded:
                    return self._sharded_warm_step(batch, next_batch)
                return self._on_side(lambda: self.eager_step(batch, next_batch))
            return self._capture(batch, next_batch, key)
        self._g, self._static, self._static_loss = entry
        src = _tensors(batch)
        dst = _tensors(self._static)
        if len(src) != len(dst) or any(a.shape != b.shape or a.dtype != b.dtype for a, b in zip(src, dst)):
            return self.eager_step(batch, next_batch)
        S.host_lap()
        if self._sharded and next_batch is not None:
            # route the next batch before anything of this step is queued: its side
            # stream then waits only for the previous step, and prepare(next) finds
            # the split sizes on the host a whole step early
            self.opt.prefetch(next_batch)
            S.host_lap('prefetch')
        if isinstance(batch, PackedBatch) and isinstance(self._static, PackedBatch) \
                and batch.layout == self._static.layout:
            self._static.arena.copy_(batch.arena, non_blocking=True)   # one copy for the whole batch
        else:
            _copy_batch(dst, src)
        if self._sharded:
            S.host_lap('batch_copy')
            self.opt.prepare(self._static, key=batch[0])
            self._g.replay()
            S.host_mark('replay_end')
            self.opt.restore_captured(self._cap_states.get(key))
            S.host_lap('replay')
            self.opt.step()
            S.host_mark('step_end')
            S.host_lap('step', step=True)
        else:
            self.opt.maybe_segment()
            self._g.replay()
            self.opt.graph_replayed()
        if self.jagged:
            self._poll_jagged()
        return self._static_loss.clone()

    def _sharded_warm_step(self, batch, next_batch):
        """Row-sharded warm-up step: the exchange, the dense all-reduces and the update
        on the current stream (never the capture stream, see _step), the forward and
        backward on the capture stream.  The dense parameters' AccumulateGrad nodes
        outlive a step (the bucket all-reduce hooks keep them) and stay bound to the
        stream of the backward that created them: created here on the capture stream,
        the captured backward accumulates on its own stream.  Created on the current
        (default) stream instead, every capture joined the default stream inside the
        capture (torch's AccumulateGrad stream-mismatch warning), and capturing a second
        jagged capacity that way crashed in capture_end (round 4, bench --sharded 1)."""
        self.opt.zero_grad()
        self.opt.prepare(batch)
        if next_batch is not None:
            self.opt.prefetch(next_batch)
        if hasattr(self.opt, 'begin_step'):
            self.opt.begin_step(batch)
        buckets = getattr(self.opt, 'buckets', None)
        if buckets is not None:
            buckets.enabled = False   # no collectives from the side stream: step() reduces the buckets
        try:
            def fwd_bwd():
                loss = self.compute_loss(batch)
                self._backward(loss)
                G.join_side_work()
                return loss.detach()
            loss = self._on_side(fwd_bwd)
        finally:
            if buckets is not None:
                buckets.enabled = True
        self.opt.step()
        if self.jagged:
            self.check_jagged()
        return loss

    def _on_side(self, fn):
        cur = torch.cuda.current_stream()
        if self._side is None:
            self._side = private_stream(cur.device)
        self._side.wait_stream(cur)
        with torch.cuda.stream(self._side):
            out = fn()
        cur.wait_stream(self._side)
        return out

    def _capture(self, batch, next_batch=None, key=None):
        """Record one step (host state advances once here), then replay it for this batch."""
        if self._side is None:
            self._side = private_stream(torch.cuda.current_stream().device)
        if self._sharded:
            _gemm_stream_ready(self._side)
        self._static = _clone_batch(batch)
        self.opt.zero_grad(set_to_none=True)
        if self._sharded:  # exchange eagerly, capture forward + backward only
            self.opt.prepare(self._static, key=batch[0])
            if next_batch is not None:
                self.opt.prefetch(next_batch)
            buckets = getattr(self.opt, 'buckets', None)
            if buckets is not None:
                buckets.enabled = False  # no collectives inside the graph: step() reduces the buckets
        else:
            self.opt.maybe_segment()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph(keep_graph=self.graph_audit)
        if self._pool is None:
            # one memory pool for every captured capacity: the graphs never run at once,
            # and nothing a replay leaves behind is read after another graph ran (the
            # loss is cloned right after its replay; parameters and optimizer state
            # live outside the pool; row-sharded, the eager step() reads the replayed
            # graph's own gradient buffers, kept alive by its _cap_states entry)
            self._pool = torch.cuda.graph_pool_handle()
        cur = torch.cuda.current_stream()
        self._side.wait_stream(cur)
        # thread_local: the process group's watchdog thread polls its collectives'
        # events (hipEventQuery) while we capture.  Under the default global mode a
        # capture forbids such calls from EVERY thread: the poll fails with a
        # capture error, which the watchdog treats as fatal and aborts the process
        # (seen in round 1).  thread_local confines the restriction to this thread,
        # so the watchdog's polls are legal and nothing needs to wait for it.
        with torch.cuda.graph(g, pool=self._pool, stream=self._side, capture_error_mode='thread_local'):
            if self._sharded:
                loss = self.compute_loss(self._static)
                self._backward(loss)
                G.join_side_work()   # every side-stream branch rejoins the capture stream
                self._static_loss = loss.detach()
            else:
                self._static_loss = self.eager_step(self._static)
        cur.wait_stream(self._side)
        if self.graph_audit:
            self.graph_nodes = graph_node_census(g)
            g.instantiate()
        self._g = g
        self._graphs[key] = (g, self._static, self._static_loss)
        g.replay()               # the captured step itself (host state already advanced)
        if self._sharded:
            if buckets is not None:
                buckets.enabled = True
            self._cap_states[key] = self.opt.capture_state()
            self.opt.step()
        return self._static_loss.clone()


def _gemm_stream_ready(stream):
    """grk_gemm allocates its per-stream hipBLASLt workspace on a stream's first GEMM,
    which must not happen inside a capture: one tiny GEMM on ``stream`` first."""
    from . import kernels as K
    cur = torch.cuda.current_stream()
    stream.wait_stream(cur)
    with torch.cuda.stream(stream):
        a = torch.zeros(16, 16, dtype=torch.bfloat16, device=cur.device)
        K.gemm(a, a, trans_b=True)
    cur.wait_stream(stream)


_NODE_TYPES = {0: 'kernel', 1: 'memcpy', 2: 'memset', 3: 'host', 4: 'graph', 5: 'empty', 6: 'wait_event',
               7: 'event_record', 10: 'mem_alloc', 11: 'mem_free'}


def graph_node_census(g):
    """{node type: count} of a captured torch.cuda.CUDAGraph(keep_graph=True), plus
    'memset_bytes': the byte count of every memset node.  A memset node does not
    re-zero its buffer on the second and later replays (ROCm 7.2,
    scripts/graph_memset_check.py), so the training step must contain none
    larger than 4 bytes (the one size that replays correctly)."""
    import ctypes as C
    hip = C.CDLL('libamdhip64.so.7')
    graph = C.c_void_p(g.raw_cuda_graph())
    n = C.c_size_t(0)
    if hip.hipGraphGetNodes(graph, None, C.byref(n)) != 0:
        raise RuntimeError('hipGraphGetNodes failed')
    nodes = (C.c_void_p * n.value)()
    if hip.hipGraphGetNodes(graph, nodes, C.byref(n)) != 0:
        raise RuntimeError('hipGraphGetNodes failed')

    class MemsetParams(C.Structure):
        _fields_ = [('dst', C.c_void_p), ('elementSize', C.c_uint), ('height', C.c_size_t), ('pitch', C.c_size_t),
                    ('value', C.c_uint), ('width', C.c_size_t)]

    out = {'memset_bytes': []}
    for i in range(n.value):
        t = C.c_int(-1)
        hip.hipGraphNodeGetType(C.c_void_p(nodes[i]), C.byref(t))
        name = _NODE_TYPES.get(t.value, f'type{t.value}')
        out[name] = out.get(name, 0) + 1
        if name == 'memset':
            prm = MemsetParams()
            hip.hipGraphMemsetNodeGetParams(C.c_void_p(nodes[i]), C.byref(prm))
            out['memset_bytes'].append(prm.elementSize * prm.width * max(prm.height, 1))
    return out


def _copy_batch(dst, src):
    """Batch tensors into the captured step's inputs: one multi-tensor copy per
    dtype.  A single _foreach_copy_ over the mixed int32 / int64 / fp32 batch
    leaves the multi-tensor fast path and issues one memcpy per tensor (~50
    copies of ~5 us each per step, measured)."""
    groups = {}
    for d, s in zip(dst, src):
        g = groups.setdefault((d.dtype, s.dtype, d.device, s.device), ([], []))
        g[0].append(d)
        g[1].append(s)
    for d, s in groups.values():
        torch._foreach_copy_(d, s, non_blocking=True)
