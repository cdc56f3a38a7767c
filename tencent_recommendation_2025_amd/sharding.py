"""Multi-GPU training: row-sharded tables over RCCL all-to-all, DP all-reduce.

The reference is single-process (no torch.distributed); this is
the north star's scale-out:

* one process per GPU, ``torch.distributed`` with the "nccl" backend (RCCL
  over xGMI); every rank trains on its own batch (data parallel, weak scaling);
* the big tables (``item_emb``, ``user_emb``) are **row-sharded**: global row
  ``g`` lives on rank ``g % G`` at local row ``g // G`` (row 0 -- the padding
  row -- is local row 0 of rank 0).  At the start of a step ``prepare`` routes
  the batch's unique ids to their owners (``all_to_all``), owners gather the
  rows, and the rows come back (``all_to_all``); the model's fused gather then
  reads the fetched rows.  After backward, each rank first reduces its
  gradients per unique id (deterministic), routes them to the owners
  (``all_to_all``), and each owner reduces what it received in rank order
  (deterministic) and runs the table AdamW on its shard;
* the small tables (pos + feature tables, ~48k rows) are replicated; their
  dense fp32 gradient and every dense parameter's gradient are averaged with
  one flat ``all_reduce`` each.

Gradients are averaged over ranks (DP convention: the global loss is the mean
of the per-rank losses).  One host synchronisation per step remains: the
all-to-all split sizes.

The collective logic here is device-agnostic (the CPU test suite drives it
with gloo); the device work is injected: on HIP tensors the row gather and
the gradient reductions are the grk kernels.
"""
from __future__ import annotations

import dataclasses
import os

import torch
import torch.distributed as dist

from . import _lib as L
from . import functional as G
from . import kernels as K
from . import streams as S
from .streams import host_lap
from .optim import SLICE_SIDE, SLICE_SIDE_STREAM, FusedAdamW, TableGroup


# GRK_ROUTE=torch: device ids take the sort-based torch route (_route_torch) instead of
# grk_route, so a multi-GPU run can A/B the two (grk_route is the default since round 5)
ROUTE_TORCH = os.environ.get('GRK_ROUTE', 'grk') == 'torch'


# ----------------------------------------------------------- device work ----
def kernel_gather(shard, local_ids):
    """rows = shard[local_ids] (grk_embedding_gather)."""
    out = torch.empty(local_ids.numel(), shard.shape[1], dtype=shard.dtype, device=shard.device)
    if local_ids.numel():
        K.embedding_gather([K.Lookup(shard, local_ids, 0)], out, local_ids.numel())
    return out


def kernel_reduce(sources, num_rows, dim, padding_idx, row_slot):
    """Deterministic row-sparse reduction (grk_embedding_backward)."""
    return K.embedding_backward(sources, num_rows, dim, padding_idx=padding_idx, dense=False, sparse=True,
                                row_slot=row_slot)


def kernel_dense_reduce(sources, num_rows, dim, token_type=None, seq_len=0, padding_idx=0):
    return K.embedding_backward(sources, num_rows, dim, padding_idx=padding_idx, token_type=token_type,
                                seq_len=seq_len, dense=True).dense


# ----------------------------------------------------------- collectives ----
# RCCL ("nccl") takes device tensors directly.  With gloo (CPU tests, and
# rehearsing several ranks on one GPU) device tensors are staged via host.
def _staged(pg, *ts):
    return dist.get_backend(pg) == 'gloo' and any(t.is_cuda for t in ts)


def a2a(out, inp, out_split=None, in_split=None, pg=None):
    if _staged(pg, out, inp):
        o = out.cpu()
        dist.all_to_all_single(o, inp.cpu(), out_split, in_split, group=pg)
        out.copy_(o)
    else:
        dist.all_to_all_single(out, inp, out_split, in_split, group=pg)


def all_reduce(t, pg=None):
    if _staged(pg, t):
        c = t.cpu()
        dist.all_reduce(c, group=pg)
        t.copy_(c)
    else:
        dist.all_reduce(t, group=pg)


# ------------------------------------------------------------- exchange ----
class ShardedRef(G.TableRef):
    """Marks a lookup of a row-sharded table (must be remapped by prepare())."""
    __slots__ = ('name',)

    def __init__(self, name, weight):
        super().__init__(weight)
        self.name = name


class FetchSink:
    """Collects the gradient sources of lookups into a fetched-row buffer."""

    def __init__(self):
        self.sources = []

    def collect(self, src, token_type, seq_len):
        self.sources.append(src)


class ShardExchange:
    """Routes ids / rows / gradients of one row-sharded table."""

    def __init__(self, name, shard, dim, pg=None, gather_fn=kernel_gather, global_rows=None):
        self.name, self.shard, self.dim, self.pg = name, shard, dim, pg
        self.world = dist.get_world_size(pg)
        self.rank = dist.get_rank(pg)
        # rows of the whole table (ids past it are refused); default: this shard's rows x world
        self.global_rows = int(global_rows) if global_rows is not None else shard.shape[0] * self.world
        self.gather_fn = gather_fn
        self.plan = None

    @staticmethod
    def _stable_sort(keys, bound):
        """(sorted keys, permutation) of int64 keys in [0, bound): grk's radix sort on the
        GPU (a few launches over ceil(log2 bound) bits; torch.sort runs ~30 rocprim
        merge-sort launches here), torch.sort on the CPU.  Keys outside [0, bound) are
        mis-ordered by the radix sort: route() counts out-of-range ids on the device
        and prepare() raises on them at the step's host read of the split sizes."""
        if not keys.is_cuda or bound >= (1 << 31):
            return torch.sort(keys, stable=True)
        n = keys.numel()
        k32, perm = K.sort_pairs(keys.to(torch.int32), torch.arange(n, dtype=torch.int64, device=keys.device),
                                 max(1, int(bound - 1).bit_length()))
        return k32.to(keys.dtype), perm

    def route(self, ids, pg=None):
        """Phase 1 (before the single host sync): unique ids, owner order, counts.
        pg: communicator for the counts exchange (default: the table's).  Device ids:
        grk_route (K.route: a presence bitmap, five launches); host ids: the
        sort-based restatement below (_route_torch), the same plan."""
        if ids.is_cuda and not ROUTE_TORCH:
            rows_per_owner = -(-self.global_rows // self.world)
            r = K.route(ids, self.world, max(rows_per_owner, 1), self.global_rows)
            recv_counts = torch.empty_like(r['send_counts'])
            a2a(recv_counts, r['send_counts'], pg=self.pg if pg is None else pg)
            return dict(uniq=r['send_ids'], inverse=r['inverse'], send_ids=r['send_ids'],
                        send_counts=r['send_counts'], recv_counts=recv_counts, bad=r['bad'])
        return self._route_torch(ids, pg)

    def _route_torch(self, ids, pg=None):
        """route() on host tensors (and the reference the GPU test holds grk_route to).

        Every output has a fixed size (len(ids)), so nothing here waits for the
        device (torch.unique / bincount would: their output sizes are data
        dependent): uniq holds the distinct ids ascending in its first n_uniq
        slots, the tail is padding whose owner is the overflow bin ``world``, so
        the stable owner order lists every real id first.  n_uniq reaches the
        host as sum(send_counts) with the split sizes."""
        n = ids.numel()
        # ids a shard cannot hold (negative, or past the last global row): counted here,
        # raised by prepare() when the counts reach the host (no sync of its own)
        bad = ((ids < 0) | (ids >= self.global_rows)).sum()
        srt, perm = self._stable_sort(ids, self.shard.shape[0] * self.world + self.world)
        head = torch.ones_like(srt, dtype=torch.bool)
        if n > 1:
            head[1:] = srt[1:] != srt[:-1]
        upos = torch.cumsum(head, 0) - 1                 # unique index of each sorted occurrence
        inverse = torch.empty_like(upos)
        inverse[perm] = upos
        uniq = torch.zeros_like(srt)
        uniq.scatter_(0, upos, srt)                      # duplicates write the same value
        n_uniq = upos[-1:] + 1 if n else upos.new_zeros(1)
        owner = torch.where(torch.arange(n, device=ids.device) < n_uniq, uniq % self.world, self.world)
        order = self._stable_sort(owner, self.world + 1)[1]
        send_ids = uniq[order]
        # fetched rows and per-unique gradients live in owner order (slot s holds
        # send_ids[s]): rows come back from the owners already in place and the
        # gradients go out without a permutation; tokens index their id's slot
        slot = torch.empty_like(order)
        slot[order] = torch.arange(n, device=ids.device)
        inverse = slot[inverse]
        send_counts = torch.zeros(self.world + 1, dtype=torch.int64, device=ids.device)
        send_counts.scatter_add_(0, owner, torch.ones_like(owner))
        send_counts = send_counts[:self.world].contiguous()
        recv_counts = torch.empty_like(send_counts)
        a2a(recv_counts, send_counts, pg=self.pg if pg is None else pg)
        return dict(uniq=uniq, inverse=inverse, order=order, send_ids=send_ids, send_counts=send_counts,
                    recv_counts=recv_counts, bad=bad)

    def fetch(self, r, send_split, recv_split, before_gather=None, out=None):
        """Phase 2: ids to owners, owners gather, rows back; returns rows in slot (owner) order.

        before_gather(local ids) runs on the owner before its gather (the
        deferred-AdamW catch-up of the requested rows).  out: a buffer of at
        least n_uniq rows to receive them (a fixed buffer lets a captured
        forward read the rows of every step)."""
        n_uniq = sum(send_split)
        recv_ids = r['send_ids'].new_empty(sum(recv_split))
        a2a(recv_ids, r['send_ids'][:n_uniq], recv_split, send_split, self.pg)
        local = recv_ids // self.world
        if before_gather is not None and local.numel():
            before_gather(local)
        rows = self.gather_fn(self.shard, local)
        fetched = rows.new_empty((n_uniq, self.dim)) if out is None else out
        a2a(fetched[:n_uniq], rows, send_split, recv_split, self.pg)
        self.plan = dict(send_split=send_split, recv_split=recv_split, recv_local=local, n_uniq=n_uniq)
        return fetched

    def push_grads(self, uniq_grads):
        """Route per-slot gradients [>= n_uniq, D] (slot order, as fetch() returned the
        rows) to the owners; returns (local ids, rows) received."""
        p = self.plan
        send = uniq_grads[:p['n_uniq']]
        send = send if send.is_contiguous() else send.contiguous()
        recv = send.new_empty((sum(p['recv_split']), self.dim))
        a2a(recv, send, p['recv_split'], p['send_split'], self.pg)
        return p['recv_local'], recv


def shard_rows(full_rows, world, rank):
    return (full_rows - rank + world - 1) // world


# ------------------------------------------------------ DP gradient sync ----
class GradBuckets:
    """Dense-parameter gradients averaged over ranks while backward still runs.

    Parameters are bucketed in reverse registration order (the order autograd
    finishes their gradients); a bucket's ``all_reduce`` is issued from a
    post-accumulate-grad hook as soon as it and every earlier bucket are
    complete, so the launch order is the same on every rank and RCCL overlaps
    the reduction with the rest of backward.  ``finish()`` (in the optimizer
    step) issues what is left (parameters without a gradient this step count
    as zero on this rank), waits, and writes the means back into ``p.grad``."""

    def __init__(self, params, pg=None, bucket_bytes=32 << 20):
        self.pg = pg
        self.world = dist.get_world_size(pg)
        self.params = list(params)
        self.buckets, cur, size = [], [], 0
        for p in reversed(self.params):
            cur.append(p)
            size += p.numel() * 4
            if size >= bucket_bytes:
                self.buckets.append(cur)
                cur, size = [], 0
        if cur:
            self.buckets.append(cur)
        self.where = {id(p): b for b, ps in enumerate(self.buckets) for p in ps}
        dev = self.params[0].device if self.params else torch.device('cpu')
        self.flat = [torch.empty(sum(p.numel() for p in ps), dtype=torch.float32, device=dev) for ps in self.buckets]
        # each parameter's gradient view of its bucket, made once (finish() hands them out)
        self._views = []
        for b, ps in enumerate(self.buckets):
            off, vs = 0, []
            for p in ps:
                vs.append(self.flat[b][off:off + p.numel()].view_as(p))
                off += p.numel()
            self._views.append(vs)
        self.async_ok = dev.type == 'cuda' and dist.get_backend(pg) != 'gloo'
        self.enabled = True  # off while a backward is being captured into a HIP graph
        self._reset()
        for p in self.params:
            p.register_post_accumulate_grad_hook(self._hook)

    def _reset(self):
        self.ready = [0] * len(self.buckets)
        self.works = [None] * len(self.buckets)
        self.next = 0

    def _hook(self, p):
        if not self.enabled:
            return
        b = self.where[id(p)]
        self.ready[b] += 1
        while self.next < len(self.buckets) and self.ready[self.next] == len(self.buckets[self.next]):
            self._launch(self.next)
            self.next += 1

    def _launch(self, b):
        """Bucket b's gradients into its flat buffer (device: one grk_flat_pack launch;
        host: one cat), then its all-reduce."""
        flat = self.flat[b]
        if flat.is_cuda and all(p.grad is None or p.grad.data_ptr() < flat.data_ptr()
                                or p.grad.data_ptr() >= flat.data_ptr() + flat.numel() * 4
                                for p in self.buckets[b]):
            parts, off = [], 0
            for p in self.buckets[b]:
                parts.append((p.grad, off, p.numel()))
                off += p.numel()
            K.flat_pack(flat, parts)
            if self.async_ok:
                self.works[b] = dist.all_reduce(flat, group=self.pg, async_op=True)
            else:
                all_reduce(flat, self.pg)
            return
        off, src, alias = 0, [], 0
        for p in self.buckets[b]:
            n = p.numel()
            if p.grad is None:
                src.append(flat.new_zeros(n))
            else:
                src.append(p.grad.reshape(-1))
                alias += src[-1].data_ptr() == flat[off:].data_ptr()
            off += n
        if alias == 0:
            torch.cat(src, out=flat)
        elif alias < len(src):  # zero_grad(set_to_none=False): some grads already live in the bucket
            off = 0
            for t in src:
                if t.data_ptr() != flat[off:].data_ptr():
                    flat[off:off + t.numel()].copy_(t)
                off += t.numel()
        if self.async_ok:
            self.works[b] = dist.all_reduce(flat, group=self.pg, async_op=True)
        else:
            all_reduce(flat, self.pg)

    def launch_rest(self):
        """Issue every bucket not issued yet (in bucket order)."""
        while self.next < len(self.buckets):
            self._launch(self.next)
            self.next += 1

    def finish(self):
        """Issue the remaining buckets, wait, and make every p.grad the mean (a view of its bucket)."""
        self.launch_rest()
        inv = 1.0 / self.world
        for b, ps in enumerate(self.buckets):
            if self.works[b] is not None:
                self.works[b].wait()
            if self.world > 1:
                self.flat[b].mul_(inv)
            for p, v in zip(ps, self._views[b]):
                p.grad = v
        self._reset()


# ------------------------------------------------------------ optimizer ----
class ShardedFusedAdamW(FusedAdamW):
    """FusedAdamW across ranks: sharded item/user tables, replicated small tables, DP dense params.

    Sharded tables keep dense parity the deferred way (optim.FusedAdamW): an
    owner brings the rows it is asked for up to the current step inside
    ``prepare`` (catch-up replay) before gathering them, updates the rows it
    receives gradients for after backward (lazy update + step stamp), and the
    rows nobody asked for stay deferred until the rolling flush reaches them
    (one 1/defer_period slice of each shard per step, in ``prepare``; rolling=False:
    all rows every ``defer_period`` steps), or before ``state_dict``."""

    SHARDED = ('item_emb', 'user_emb')

    def __init__(self, model, lr=1e-3, betas=(0.9, 0.98), eps=1e-8, weight_decay=0.01, table_mode='dense',
                 table_dtype=torch.bfloat16, pg=None, gather_fn=kernel_gather, reduce_fn=kernel_reduce,
                 dense_reduce_fn=kernel_dense_reduce, defer_period=16, bucket_bytes=32 << 20, lookahead=True,
                 init_seed=0, dense_flat=True, rolling=True):
        self.pg = pg
        self.world = dist.get_world_size(pg)
        self.rank = dist.get_rank(pg)
        self.reduce_fn, self.dense_reduce_fn = reduce_fn, dense_reduce_fn
        tables = model.table_modules()
        dev = model.item_emb.weight.device
        self.shards = {}
        sharded_refs = {}
        for name in self.SHARDED:
            emb = tables[name]
            if emb.weight.shape[0] == 0:
                # placeholder (model args.shard_tables): build only this rank's rows
                # -- global rows rank::world, table_init_rows of the whole table's
                # init (the 50M-row tables of config 3 never exist whole anywhere)
                from .model import table_init_rows, table_init_std
                R, D = emb.num_embeddings, emb.embedding_dim
                n = len(range(self.rank, R, self.world))
                shard = torch.empty(n, D, dtype=table_dtype, device=dev)
                ch = 1 << 18
                for s in range(0, n, ch):
                    rows = torch.arange(s, min(n, s + ch), device=dev) * self.world + self.rank
                    shard[s:s + ch] = table_init_rows(rows, D, init_seed + (1 if name == 'user_emb' else 0),
                                                      table_init_std(R, D), table_dtype)
            else:
                full = emb.weight.detach()
                shard = full[self.rank::self.world].to(dtype=table_dtype).contiguous()
            grp = TableGroup(f'{name}@{self.rank}', [(name, _Holder(shard))], table_dtype, dev)
            grp.global_rows = emb.num_embeddings
            self.shards[name] = (grp, ShardExchange(name, grp.flat, emb.embedding_dim, pg, gather_fn,
                                                     global_rows=emb.num_embeddings))
            # the full table is not kept: this rank holds rows rank::world only
            emb.weight = torch.nn.Parameter(torch.empty(0, emb.embedding_dim, dtype=table_dtype, device=dev),
                                            requires_grad=False)
            sharded_refs[name] = ShardedRef(name, emb.weight)
        small_keys = tuple(k for k in tables if k not in self.SHARDED and k != 'pos_emb')
        # dense parameters: their gradients are all-reduced in buckets (GradBuckets), then
        # updated by the flat multi-range AdamW (dense_flat: one launch, bf16 GEMM shadows
        # written with the update) -- parameters it cannot hold stay on torch's AdamW
        super().__init__(model, lr, betas, eps, weight_decay, table_mode, table_dtype,
                         groups=(('pos', ('pos_emb',)), ('small', small_keys)), defer_period=defer_period,
                         dense_flat=dense_flat)
        model._table_refs.update(sharded_refs)
        # replicated groups: their fp32 gradients share one buffer (one all-reduce)
        self.replicated = list(self.groups)
        self.rep_rows = sum(g.rows for g in self.replicated)
        self.rep_identity = torch.arange(max(g.rows for g in self.replicated), dtype=torch.int32, device=dev)
        self.sinks = {}
        # the shards are the deferred groups (FusedAdamW machinery: ring, segments, flush)
        if self.defer:
            self._deferred = {name: grp for name, (grp, _) in self.shards.items()}
            for g in self._deferred.values():
                g.last = torch.zeros(g.rows, dtype=torch.int32, device=dev)
            if rolling and self.clock is not None:
                # the rolling flush (optim.FusedAdamW rolling): prepare() brings one 1/defer_period
                # slice of every shard up to date each step; the ring holds 2 x defer_period steps
                self.rolling = True
                self.clock = K.DeviceClock(2 * self.defer, dev)
                self._pinned = [torch.zeros_like(self.clock.ring, device='cpu').pin_memory() for _ in range(2)]
        params = self._dense_params()
        self.buckets = GradBuckets(params, pg, bucket_bytes) if params else None
        # fixed exchange buffers (rows fetched for a step, inverse indices): a captured
        # forward reads them at the same addresses every step
        self._fbuf, self._ibuf = {}, {}
        # lookahead routing: the next batch's counts exchange on its own communicator
        # and stream, so prepare() needs no device round trip
        self.meta_pg = dist.new_group(backend=dist.get_backend(pg)) if lookahead else None
        self.trace = None  # optional list: host-side diagnostics (scripts/host_issue.py)
        self._ahead = []  # routed batches waiting for their prepare(), oldest first (at most 2)
        self._captured = None

    def begin_step(self, batch):
        """Nothing: prepare() catches up the rows each owner is asked for."""

    def shard_table(self, name):
        """(rows held by this rank, brought to the current step) -- global rows rank::world."""
        self.flush()
        return self.shards[name][0].flat

    # -- input dist -------------------------------------------------------
    @staticmethod
    def _parts(batch):
        """{table: [(role of the model's lookup, index tensor, lookup mode, ids it reads)]}.
        Roles name the model's call sites (model._remap_specs): 'seq' = log2feats,
        'pos' / 'neg' = the two halves of feat2emb_pair."""
        seq, pos, neg, tt = batch[0], batch[1], batch[2], batch[3]
        seq, pos, neg = seq.long(), pos.long(), neg.long()
        tt = tt.to(seq.device)
        return {
            'item_emb': [('seq', seq, L.IDX_ITEM_MASK, lambda: seq * (tt == 1)),
                         ('pos', pos, L.IDX_PLAIN, lambda: pos), ('neg', neg, L.IDX_PLAIN, lambda: neg)],
            'user_emb': [('seq', seq, L.IDX_USER_MASK, lambda: seq * (tt == 2))],
        }

    def _route_all(self, batch, pg):
        routed = {}
        for name, plist in self._parts(batch).items():
            ids = torch.cat([v().reshape(-1) for _, _, _, v in plist])
            routed[name] = self.shards[name][1].route(ids, pg)
        counts = torch.stack([torch.stack([r['send_counts'], r['recv_counts']]) for r in routed.values()])
        # one more [2, world] block: [0][0] = ids out of every table's range (read with the counts)
        flag = torch.zeros_like(counts[:1])
        flag[0, 0, 0] = sum(r['bad'] for r in routed.values())
        return routed, torch.cat([counts, flag])

    def prefetch(self, batch):
        """Route a coming batch ahead of its step (own communicator for the counts):
        its prepare() then finds the all-to-all split sizes already on the host
        instead of waiting for the device to drain.  Every rank must prefetch the
        same sequence of batches."""
        seq = batch[0]
        if self.meta_pg is None or not seq.is_cuda or dist.get_backend(self.pg) == 'gloo':
            return
        # On the current stream, in order: HIP serialises this process's streams on
        # shared hardware queues, and a side stream's work waiting on the main
        # stream was measured to run only after the whole queued step (the host
        # then waited for it in prepare()); issued first in the step on the main
        # stream it runs at once and is long done when prepare() reads the counts.
        routed, counts = self._route_all(batch, self.meta_pg)
        host = self._pinned_counts(counts)
        host.copy_(counts, non_blocking=True)
        done = torch.cuda.Event()
        done.record()
        self._ahead = self._ahead[-1:] + [(seq, routed, host, done)]

    def _pinned_counts(self, counts):
        """Two pinned host buffers used in turn (prepare() has read the older one
        before the next prefetch writes it)."""
        ring = getattr(self, '_pinned_ring', None)
        if ring is None or ring[0].shape != counts.shape:
            ring = self._pinned_ring = [torch.empty(counts.shape, dtype=counts.dtype, pin_memory=True)
                                        for _ in range(2)]
            self._pinned_turn = 0
        self._pinned_turn ^= 1
        return ring[self._pinned_turn]

    def _buffer(self, cache, name, shape, dtype, dev):
        t = cache.get(name)
        if t is None or t.shape[0] < shape[0]:
            t = cache[name] = torch.empty(shape, dtype=dtype, device=dev)
        return t

    def prepare(self, batch, key=None):
        """Fetch every row of the sharded tables this step's batch reads.
        key: the tensor prefetch() was given for this batch (default batch[0])."""
        key = batch[0] if key is None else key
        ahead = next((a for a in self._ahead if a[0] is key), None)
        self._ahead = [a for a in self._ahead if a is not ahead]
        if ahead is not None:
            _, routed, host, done = ahead
            if self.trace is not None:
                self.trace.append(('route done at prepare', done.query()))
            host_lap('prepare.issue')
            S.host_check('replay_end', 'n:prev_replay_done_before_wait')
            S.host_check('step_end', 'n:prev_step_done_before_wait')
            done.synchronize()  # long done: the route ran during the previous step
            host_lap('prepare.route_wait')
            S.host_check('replay_end', 'n:prev_replay_done_after_wait')
            S.host_check('step_end', 'n:prev_step_done_after_wait')
            counts = host.tolist()
            main = torch.cuda.current_stream()
            main.wait_event(done)
            for r in routed.values():
                for t in r.values():
                    t.record_stream(main)
        else:
            routed, counts = self._route_all(batch, self.pg)
            counts = counts.cpu().tolist()  # the one host sync of the step: all-to-all split sizes
        if counts[-1][0][0]:
            raise ValueError(f'row-sharded lookup: {counts[-1][0][0]} ids outside [0, rows) of their table')
        counts = counts[:-1]
        self.maybe_segment()
        remaps = {}
        self.sinks = {}
        # the rolling slice after the fetch (the requested rows are then current and
        # skipped) on a side stream, under the step's forward and backward; step() joins it
        # before any shard row is updated
        slice_side = self.rolling and SLICE_SIDE and self.clock.ring.is_cuda
        for gi, (name, plist) in enumerate(self._parts(batch).items()):
            grp, ex = self.shards[name]
            r = routed[name]
            catchup = None
            if self.rolling and not slice_side:   # this step's slice of the shard (rolling flush)
                K.table_adamw_catchup_slice(grp.flat, grp.exp_avg, grp.exp_avg_sq, grp.last, self.clock,
                                            self._period)
            if self.defer:
                def catchup(local, grp=grp):
                    K.table_adamw_catchup(grp.flat, grp.exp_avg, grp.exp_avg_sq, grp.last, None, self.clock,
                                          local.contiguous())
            n_ids = r['inverse'].numel()
            fbuf = self._buffer(self._fbuf, name, (n_ids, grp.dim), grp.flat.dtype, grp.flat.device)
            host_lap('prepare.issue')
            fetched = ex.fetch(r, counts[gi][0], counts[gi][1], before_gather=catchup, out=fbuf)
            host_lap('prepare.fetch')
            inv_all = self._buffer(self._ibuf, name, (n_ids,), r['inverse'].dtype, grp.flat.device)
            inv_all[:n_ids].copy_(r['inverse'])
            sink = FetchSink()
            self.sinks[name] = sink
            ref = G.TableRef(fetched, sink, 0)
            off = 0
            for role, idx, mode, _ in plist:
                n = idx.numel()
                inv = inv_all[off:off + n].view(idx.shape)
                off += n
                remaps[(name, role, mode)] = (ref, inv)
        self.model._remaps = remaps
        if slice_side:
            def slices():
                for grp, _ in self.shards.values():
                    K.table_adamw_catchup_slice(grp.flat, grp.exp_avg, grp.exp_avg_sq, grp.last, self.clock,
                                                self._period)
            G.run_on_side(slices, self.clock.ring.device, SLICE_SIDE_STREAM)
        self._begun = self.t
        host_lap('prepare.issue')

    # -- HIP graph capture of forward + backward (train.Trainer) ------------
    def _dense_params(self):
        """Every dense parameter: the flat buffer's, then torch AdamW's."""
        out = list(self._flat.params) if self._flat is not None else []
        if self.dense is not None:
            out += [p for grp in self.dense.param_groups for p in grp['params']]
        return out

    def capture_state(self):
        """After the forward + backward of a captured step: what its replays rewrite
        in place (gradient sources of every group and sink, dense gradients).
        Returned to the caller, which keeps it with ITS graph: a trainer holding one
        graph per jagged capacity restores the state of the graph it replays (the
        buffers of another capacity's graph hold that graph's last gradients)."""
        self._captured = dict(
            groups=[(g, list(g.pending), dict(g.dense_grads), g.token_type, g.seq_len) for g in self.replicated],
            sinks={k: list(sk.sources) for k, sk in self.sinks.items()},
            grads=[(p, p.grad) for p in self._dense_params()])
        return self._captured

    def restore_captured(self, state=None):
        """Before step() after a replay: point the groups, sinks and .grad back at the
        buffers of the replayed graph (``state`` from its capture_state(); default the
        last one captured)."""
        c = self._captured if state is None else state
        self._captured = c
        for g, pend, dg, tt, sl in c['groups']:
            g.pending, g.dense_grads, g.token_type, g.seq_len = list(pend), dict(dg), tt, sl
        self.sinks = {}
        for k, src in c['sinks'].items():
            self.sinks[k] = FetchSink()
            self.sinks[k].sources = list(src)
        for p, gr in c['grads']:
            p.grad = gr

    # -- gradient sync + update -------------------------------------------
    @torch.no_grad()
    def step(self):
        G.join_side_work()
        if self._deferred and self._begun != self.t:
            raise RuntimeError('ShardedFusedAdamW: call prepare(batch) before forward (Trainer.step does)')
        self._begun = None
        self.t += 1
        self.clock.advance()
        hp = self.clock
        inv_world = 1.0 / self.world
        # Order on RCCL's stream: the shard gradients' all-to-alls first (the owner
        # updates wait on them), then the all-reduces of the replicated tables and the
        # dense parameters, which run under the owner reductions and updates.
        pushed = []
        for name, (grp, ex) in self.shards.items():
            sink = self.sinks.get(name)
            if sink is not None and sink.sources and ex.plan is not None:
                nu = ex.plan['n_uniq']
                # the lookups read a fixed buffer of >= nu rows; this step's ids index its first nu
                srcs = [dataclasses.replace(sc, table_rows=nu) if isinstance(sc, K.GradSource) else sc
                        for sc in sink.sources]
                ug = self.dense_reduce_fn(srcs, nu, grp.dim, padding_idx=None)
                if self.world > 1:
                    ug.mul_(inv_world)
                pushed.append((grp, ex.push_grads(ug)))
            elif not self.lazy and not self.defer:
                K.table_adamw(grp.flat, grp.exp_avg, grp.exp_avg_sq, hp)
        host_lap('step.shard_grads')
        # replicated tables (pos + feature tables): dense fp32 gradients in one buffer
        dev = self.replicated[0].flat.device
        rep = torch.empty(self.rep_rows, self.replicated[0].dim, dtype=torch.float32, device=dev)
        row = 0
        for g in self.replicated:
            _dense_grad_into(g, rep[row:row + g.rows], self.dense_reduce_fn)
            row += g.rows
        rep_work = None
        if self.world > 1:
            if rep.is_cuda and dist.get_backend(self.pg) != 'gloo':
                rep_work = dist.all_reduce(rep, group=self.pg, async_op=True)
            else:
                all_reduce(rep, self.pg)
        host_lap('step.replicated')
        if self.buckets is not None:
            self.buckets.launch_rest()  # dense parameters (all of them when the backward was a graph replay)
        host_lap('step.buckets_launch')
        # owners: reduce what arrived (rank order: deterministic), update the shard rows
        for grp, (local, rows) in pushed:
            src = [K.GradSource(local, rows, 0)]
            res = self.reduce_fn(src, grp.rows, grp.dim, 0 if self.rank == 0 else -1,
                                 None if self.lazy else grp.row_slot)
            K.table_adamw(grp.flat, grp.exp_avg, grp.exp_avg_sq, hp, res.ids, res.rows, res.count, res.capacity,
                          None if self.lazy else grp.row_slot, lazy=self.lazy or bool(self.defer))
            if self.defer:
                K.stamp_rows(grp.last, res.ids, res.count, res.capacity, self.clock)
        host_lap('step.owner_updates')
        if self.buckets is not None:
            self.buckets.finish()
        host_lap('step.buckets_finish')
        if self.dense is not None:
            self.dense.step()
        if self._flat is not None:
            self._flat.step(hp)
        host_lap('step.dense_update')
        if rep_work is not None:
            rep_work.wait()
        if self.world > 1:
            rep.mul_(inv_world)
        row = 0
        for g in self.replicated:
            K.table_adamw(g.flat, g.exp_avg, g.exp_avg_sq, hp, None, rep[row:row + g.rows], None, 0,
                          self.rep_identity[:g.rows])
            row += g.rows
            g.clear()
        self.sinks = {}
        self.model._remaps = None
        host_lap('step.replicated_update')


def _dense_grad_into(g, out, dense_reduce_fn):
    """out (fp32 [g.rows, D]) = the group's gradient: row-sparse sources reduced
    densely plus the dense ranges (tables used in dense ops), zeros elsewhere."""
    if g.pending:
        out.copy_(dense_reduce_fn(g.pending, g.rows, g.dim, g.token_type, g.seq_len))
        for off, dg in g.dense_grads.items():
            out[off:off + dg.shape[0]] += dg
        return
    D = out.shape[1]
    if out.is_cuda and out.is_contiguous():
        # every range and the gaps between them in one grk_flat_pack launch (bf16 -> fp32)
        parts, pos = [], 0
        for off in sorted(g.dense_grads):
            dg = g.dense_grads[off]
            if off > pos:
                parts.append((None, pos * D, (off - pos) * D))
            parts.append((dg, off * D, dg.shape[0] * D))
            pos = off + dg.shape[0]
        if pos < g.rows:
            parts.append((None, pos * D, (g.rows - pos) * D))
        K.flat_pack(out.view(-1), parts)
        return
    pos = 0
    for off in sorted(g.dense_grads):
        dg = g.dense_grads[off]
        if off > pos:
            out[pos:off].zero_()
        out[off:off + dg.shape[0]].copy_(dg)
        pos = off + dg.shape[0]
    if pos < g.rows:
        out[pos:].zero_()


class _Holder:
    """Minimal nn.Embedding stand-in for TableGroup (a shard buffer)."""

    def __init__(self, w):
        self.weight = w
        self.num_embeddings, self.embedding_dim = w.shape
