#!/usr/bin/env python
"""Training throughput of the TencentGR HSTU recommender on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--loss sampled_softmax|bce] ...

One step = forward + loss + backward + optimizer over one synthetic
TencentGR-shaped batch (BASELINE config 2: HSTU d=512, maxlen=200 -> T=201,
1M-item bf16 table, 1M users, B=128 sequences per GPU, 4 blocks x 8 heads),
inputs resident in HBM.  For N > 1 launch with torch.distributed.run (one
rank per GPU over RCCL); tables are row-sharded, dense grads all-reduced;
every rank processes its own 128 sequences (weak scaling).

Prints ONE JSON line (rank 0) with the metric, the live roofline of the
dominant hand-written kernel (the one with the most device time per step:
average launch x launches per step), every other measured kernel under
`rooflines` (attention, gathers, wgrad, sampled softmax, embedding backward;
each with PMC `traffic` from profiles/), and the CPU baseline (oracle/model_ref.py, the fp32 torch-CPU restatement of
the same model and step, on a bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBPS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8 TB/s spec
BF16_PEAK_TFLOPS = 2500.0   # dense bf16 MFMA spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    # the deferred dense-parity table AdamW flushes rolling (one 1/16 slice of every deferred table
    # per step, inside the step: optim.FusedAdamW rolling), so every step costs the same and the
    # line does not depend on --steps (round 4 flushed every row once per 16 steps, a 5.7 ms spike
    # that a 20-step window held once or twice)
    ap.add_argument('--steps', type=int, default=32)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--batch', type=int, default=128)
    ap.add_argument('--maxlen', type=int, default=200)
    ap.add_argument('--hidden', type=int, default=512)
    ap.add_argument('--blocks', type=int, default=4)
    ap.add_argument('--heads', type=int, default=8)
    ap.add_argument('--items', type=int, default=1_000_000)
    ap.add_argument('--users', type=int, default=1_000_000)
    ap.add_argument('--block', default='hstu', choices=['hstu', 'softmax'])
    ap.add_argument('--loss', default='bce', choices=['bce', 'sampled_softmax'])
    ap.add_argument('--table-mode', default='dense', choices=['dense', 'lazy'])
    ap.add_argument('--zipf', type=float, default=None)
    ap.add_argument('--time-buckets', type=int, default=0,
                    help='HSTU time bias (rab_time) with this many buckets; batches carry event times')
    ap.add_argument('--cpu-baseline', type=int, default=1)
    ap.add_argument('--dropout', type=float, default=0.01,
                    help="dropout_rate (the reference default, model/BaseLine/main.py:30)")
    ap.add_argument('--pool', type=int, default=16,
                    help='distinct device-resident batches cycled by the timed steps (16 x ~41k item rows x 1 KiB '
                         '~ 0.7 GB: more than the 256 MB Infinity Cache, so rows are not re-read warm)')
    ap.add_argument('--cpu-batch', type=int, default=128)
    ap.add_argument('--cpu-steps', type=int, default=10)
    ap.add_argument('--roofline-reps', type=int, default=20)
    ap.add_argument('--rooflines', type=int, default=1,
                    help='0: skip the per-kernel roofline replays (profiling runs: the trace then ends with the '
                         'timed steps)')
    ap.add_argument('--backend', default='nccl', choices=['nccl', 'gloo'],
                    help='gloo: rehearse N ranks on fewer GPUs (collectives staged via host)')
    ap.add_argument('--sharded', type=int, default=None, help='force the row-sharded optimizer (default: N > 1)')
    ap.add_argument('--merge-proj', type=int, default=1,
                    help='1: the projected feature tables\' row gradients of the seq-side and pair lookups in one '
                         'grk_embedding_backward call (functional.DenseMerge); 0: one call per lookup')
    ap.add_argument('--grouped-proj', type=int, default=1,
                    help='1 (default): the projected feature tables on the grouped MFMA GEMMs '
                         '(grk_grouped_gemm / grk_grouped_wgrad); 0: torch.bmm per equal-row-count stack')
    ap.add_argument('--dense-flat', type=int, default=1,
                    help='1: the dense parameters as one flat buffer on grk\'s multi-range AdamW (optim.DenseFlat); '
                         '0: torch\'s fused AdamW')
    ap.add_argument('--sharded-jagged', type=int, default=1,
                    help='1 (default since round 4, hardware-verified): the row-sharded trainer on jagged rows too '
                         '(train.jagged_remaps), so N > 1 trains on the same rows as N = 1; 0: the padded layout')
    ap.add_argument('--shard-tables', type=int, default=None,
                    help='build only each rank\'s table rows (default: sharded and >= 10M items, BASELINE config 3)')
    ap.add_argument('--graph', type=int, default=1,
                    help='capture the training step in a HIP graph and replay it (row-sharded: forward + backward)')
    ap.add_argument('--semantic-ids', type=int, default=0,
                    help='config 4: RQ-VAE semantic-id levels added as O1 item_sparse features (0 = off)')
    ap.add_argument('--sid-codes', type=int, default=256, help='config 4: codes per RQ-VAE level')
    ap.add_argument('--jagged', type=int, default=1,
                    help='token-wise step over each sequence\'s span only (jagged.py; padding rows are dead in the '
                         'reference); 0 = the padded [B, T] step')
    ap.add_argument('--step-times', type=int, default=0,
                    help='diagnostic: per-step device intervals (events) and host issue times to stderr')
    ap.add_argument('--fp8', type=int, default=0,
                    help='config C5: HSTU layers with fp8 (e4m3) q/k/v on the chunked attention kernels '
                         '(padded layout; e.g. --fp8 1 --hidden 1024 --maxlen 1024 --batch 16)')
    ap.add_argument('--jagged-quantum', type=int, default=512,
                    help='jagged capacity granularity (rows): one GEMM plan set and one HIP graph per capacity '
                         '(512: 6 capacities at C2, +0.7 %% over 1024 at 32 steps, gpurun_out r4v)')
    return ap.parse_args()


def _time(fn, reps):
    """Average duration (ms) of fn's launches, HIP events on the stream grk launches on."""
    stream = torch.cuda.current_stream()
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


PMC_TAG = 'r6'  # round tag of the committed PMC summaries (scripts/pmc_rooflines.py)


def _pmc(name, match):
    """HBM bytes per launch from a committed rocprofv3 PMC summary of the same workload (or None)."""
    path = os.path.join(REPO, 'profiles', name)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        p = json.load(f)
    if any(p.get('workload', {}).get(k) != v for k, v in match.items()):
        return None
    return p


def attention_rooflines(a, key_valid, reps, jagged=False):
    """The attention kernels of one layer at the bench shape and the batch's own
    ragged lengths, timed alone (HIP events on their stream).

    Algorithmic bytes count the rows a kernel must move for VALID tokens
    (padding rows are skipped by the kernels): fwd reads q, k, v and writes o;
    dq reads q, k, v, dO and writes dq; dk/dv reads q, k, v, dO and writes dk,
    dv (bf16, D = H*hd per token; + the fp32 rab row / softmax lse, delta).
    FLOPs count causal valid pairs P = H * sum_b L_b (L_b + 1) / 2, 2*hd per
    pair per matmul: fwd 2 matmuls, dq 3 (S, dP, dQ), dk/dv 4 (S, dV, dP, dK).
    At T = 201, hd = 64 the intensity (~45-65 FLOP/B) is far below the MI355X
    ridge (2.5 PF / 8 TB/s = 312 FLOP/B): HBM is the bound."""
    from tencent_recommendation_2025_amd import _lib as L
    from tencent_recommendation_2025_amd import kernels as K
    B, T = key_valid.shape
    H, D = a.heads, a.hidden
    hd = D // H
    dev = key_valid.device
    g = torch.Generator(device=dev).manual_seed(7)
    pre = torch.randn(B * T, 4 * D, device=dev, generator=g).bfloat16()    # [u | v | q | k] as HSTUAttention
    kv = key_valid.to(torch.uint8).contiguous()
    row_base, seq_range = None, K.seq_ranges(kv)
    if jagged:   # the rows the jagged step holds: each sequence's span only (jagged.py)
        from tencent_recommendation_2025_amd import jagged as J
        jag = J.layout(kv, J.capacity_for(J.span_rows(kv), a.jagged_quantum))
        jpre = torch.empty(jag.capacity, 4 * D, dtype=torch.bfloat16, device=dev)
        K.gather_rows([(pre, jpre)], jag.row_map)
        pre, row_base, seq_range = jpre, jag.row_base, jag.seq_range
    N = pre.shape[0]
    hstu = a.block == 'hstu'
    fp8 = bool(getattr(a, 'fp8', 0))
    kind = L.ATTN_HSTU if hstu else L.ATTN_SOFTMAX
    extra = dict(rab=0.1 * torch.randn(H, T, device=dev, generator=g), inv_n=1.0 / T, act='silu') if hstu else {}
    if fp8:   # config C5: the layer's e4m3(SiLU(v|q|k)) as HSTUAttention(fp8=True) feeds the chunked kernels
        x8 = K.silu_fp8(pre[:, D:])
        extra.pop('act', None)
        args = K.attn_args(kind, x8[:, D:2 * D], x8[:, 2 * D:], x8[:, :D], B, T, H, hd, key_valid=kv,
                           scale=hd ** -0.5, out_dtype=torch.bfloat16, seq_range=seq_range, precise=1, **extra)
    else:
        args = K.attn_args(kind, pre[:, 2 * D:3 * D], pre[:, 3 * D:], pre[:, D:2 * D], B, T, H, hd, key_valid=kv,
                           scale=hd ** -0.5, out_dtype=torch.bfloat16, seq_range=seq_range, row_base=row_base,
                           **extra)
    o = torch.empty(N, D, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(B, H, T, device=dev)
    do = torch.randn(N, D, device=dev, generator=g).bfloat16()
    dpre = torch.empty(N, 4 * D, dtype=torch.bfloat16, device=dev)
    delta = torch.empty(B, H, T, device=dev)
    drab = torch.zeros(H, T, device=dev) if hstu else None
    K.attention_fwd(args, o, lse)
    K.attention_bwd(args, o, do, lse, delta, dpre[:, 2 * D:3 * D], dpre[:, 3 * D:], dpre[:, D:2 * D], drab)
    t_fwd = _time(lambda: K.attention_fwd(args, o, lse), reps)
    t_dq = _time(lambda: K.attention_bwd(args, o, do, lse, delta, dpre[:, 2 * D:3 * D], None, None, drab,
                                         parts=L.ATTN_BWD_DQ), reps)
    t_dkdv = _time(lambda: K.attention_bwd(args, o, do, lse, delta, None, dpre[:, 3 * D:], dpre[:, D:2 * D], None,
                                           parts=L.ATTN_BWD_DKDV), reps)
    lens = kv.sum(1).double()
    n_valid = int(lens.sum().item())
    pairs = float((lens * (lens + 1) / 2).sum().item()) * H
    row = D * 2
    qkv_row = D if fp8 else D * 2                              # bytes of one token's q (k, v) row
    side = H * T * 4 if hstu else n_valid * H * 4            # rab row / lse (+ delta) per kernel
    ridge = BF16_PEAK_TFLOPS * 1e12 / (HBM_PEAK_GBPS * 1e9)
    name = ('hstu' if hstu else 'softmax') + ('_fp8' if fp8 else '')
    workload = {'B': B, 'T': T, 'D': D, 'H': H, 'kind': name, 'valid_tokens': n_valid,
                'layout': 'jagged' if jagged else 'padded'}
    # whole-sequence kernels at the C2 shape; the chunked ones for fp8 q/k/v or long sequences
    seq = not fp8 and (T + 31) // 32 * 32 + 32 <= 512 and hd <= 128
    kn = {'fwd': 'k_attn_fwd_seq', 'dq': 'k_attn_dq_seq', 'dkdv': 'k_attn_dkdv_seq'} if seq else \
        {'fwd': 'k_attn_fwd', 'dq': 'k_attn_bwd_dq', 'dkdv': 'k_attn_bwd_dkdv'}

    def entry(kernel, ms, nbytes, flops, pmc_name):
        gbps = nbytes / (ms * 1e-3) / 1e9
        tfs = flops / (ms * 1e-3) / 1e12
        ai = flops / nbytes
        bound = 'hbm' if ai < ridge else 'mfma'
        res = {'bound': bound, 'kernel': kernel,
               'achieved': round(gbps if bound == 'hbm' else tfs, 1),
               'peak': HBM_PEAK_GBPS if bound == 'hbm' else BF16_PEAK_TFLOPS,
               'unit': 'GB/s' if bound == 'hbm' else 'TFLOP/s',
               'frac': round(gbps / HBM_PEAK_GBPS if bound == 'hbm' else tfs / BF16_PEAK_TFLOPS, 4),
               'traffic': None, 'alg_bytes_per_launch': int(nbytes), 'flops_per_launch': int(flops),
               'tflops': round(tfs, 1), 'mfma_frac': round(tfs / BF16_PEAK_TFLOPS, 4),
               'arith_intensity': round(ai, 1), 'ridge': round(ridge, 1), 'avg_launch_us': round(ms * 1e3, 2),
               'calls_per_step': a.blocks, 'ms_per_step': round(ms * a.blocks, 4), 'workload': workload}
        p = _pmc(pmc_name, workload)
        if p is not None:
            res['traffic'] = int(p['traffic_bytes_per_launch'])
            res['traffic_note'] = (f'rocprofv3 PMC (profiles/{pmc_name}): FETCH_SIZE x2 + WRITE_SIZE '
                                   '(MI355X_MICROARCH.md gfx950 corrections)')
        return res

    dkdv = entry(f'grk::{kn["dkdv"]} ({name} attention dK/dV, one layer)', t_dkdv,
                 3 * n_valid * qkv_row + 3 * n_valid * row + side, 8 * hd * pairs,
                 f'{PMC_TAG}_pmc_attn_dkdv_{name}.json')
    fwd = entry(f'grk::{kn["fwd"]} ({name} attention forward, one layer)', t_fwd,
                3 * n_valid * qkv_row + n_valid * row + side, 4 * hd * pairs, f'{PMC_TAG}_pmc_attn_fwd_{name}.json')
    dq = entry(f'grk::{kn["dq"]} ({name} attention dQ{" + drab" if hstu else ""}, one layer)', t_dq,
               3 * n_valid * qkv_row + 2 * n_valid * row + side, 6 * hd * pairs,
               f'{PMC_TAG}_pmc_attn_dq_{name}.json')
    for e, k in ((fwd, 'fwd'), (dq, 'dq'), (dkdv, 'dkdv')):
        e['pmc_kernel'] = kn[k] + '<'
        e['pmc_name'] = f'{PMC_TAG}_pmc_attn_{k}_{name}.json'
    if fp8:
        for e in (fwd, dq, dkdv):
            e['peak_note'] = 'bf16 MFMA peak (QK^T runs on the fp8 MFMA, the other products on bf16)'

    fwd['survey_formula_flops'] = int(2 * B * D * T * (T + 1))  # 2*B*D*T(T+1) per layer fwd
    return dkdv, [fwd, dq]


def gather_roofline(trace, reps):
    """The seq-side fused gather alone (HIP events on its stream).

    Algorithmic bytes per SURVEY.md 8(d): rows x D x elem read + output rows
    written + index bytes.  Most rows are projected feature-table rows and the
    padding row, which stay resident in L2 / the Infinity Cache, so this rate
    is a cache-served gather rate, not an HBM rate: no HBM fraction is given
    (MI355X_MICROARCH.md measures ~17-19 TB/s for L2-resident and ~8.6 TB/s for
    Infinity-Cache-resident row gathers)."""
    from tencent_recommendation_2025_amd import kernels as K
    lookups, out, n, tt, T = max(trace, key=lambda r: r[1].shape[1])  # widest = seq side
    ms = _time(lambda: K.embedding_gather(lookups, out, n, tt, T), reps)
    D = lookups[0].table.shape[1]
    es = lookups[0].table.element_size()
    rows = n * sum(lk.bag for lk in lookups)
    idx_bytes = sum(lk.idx.numel() * lk.idx.element_size() for lk in lookups)
    tt_bytes = n * 4 if tt is not None else 0
    alg = rows * D * es + n * D * len(lookups) * es + idx_bytes + tt_bytes
    res = {'bound': 'l2/infinity-cache', 'kernel': 'grk::k_gather (seq-side fused lookup)',
           'achieved': round(alg / (ms * 1e-3) / 1e9, 1), 'peak': None, 'unit': 'GB/s', 'frac': None,
           'traffic': None, 'alg_bytes_per_launch': int(alg), 'avg_launch_us': round(ms * 1e3, 2),
           'calls_per_step': 1, 'ms_per_step': round(ms, 4),
           'rows_per_launch': int(rows), 'features': len(lookups),
           'workload': {'tokens': int(n), 'rows': int(rows), 'features': len(lookups)}}
    p = _pmc(f'{PMC_TAG}_pmc_gather.json', res['workload'])
    if p is not None:
        res['traffic'] = int(p['traffic_bytes_per_launch'])
        res['traffic_gbps'] = round(p['traffic_bytes_per_launch'] / (ms * 1e-3) / 1e9, 1)
    return res


def item_gather_roofline(table, batch, reps):
    """The item-table lookups of one bench batch (item tokens of seq, pos, neg;
    padding dropped) through grk_embedding_gather from the 1M-row bf16 table:
    random 1-KiB rows of a 1 GB table, read cold (the Infinity Cache is evicted
    before every timed launch), so every row comes from HBM -- the north
    star's "HBM-roofline on embedding gather" figure.  Algorithmic bytes =
    rows x D x 2 read + rows x D x 2 written + 8 B of index per row."""
    from tencent_recommendation_2025_amd import kernels as K
    seq, pos, neg, tt = batch[0], batch[1], batch[2], batch[3]
    ids = torch.cat([torch.where(tt == 1, seq, 0).reshape(-1), pos.reshape(-1), neg.reshape(-1)]).long()
    ids = ids[ids > 0].contiguous()
    n, D = ids.numel(), table.shape[1]
    out = torch.empty(n, D, dtype=table.dtype, device=table.device)
    lk = [K.Lookup(table, ids, 0)]
    K.embedding_gather(lk, out, n)
    # cold rows every launch: READING a 512 MiB buffer (twice the Infinity Cache)
    # evicts the table between the timed launches; a read leaves clean lines, so
    # the timed launch pays no write-back of the evicting buffer (a fill would:
    # it halves even a contiguous copy's rate, scripts/microbench/gather.hip).
    # Each launch timed alone with HIP events.
    flush = torch.ones(128 << 20, dtype=torch.int32, device=table.device)
    sink = torch.empty((), dtype=torch.int64, device=table.device)
    stream = torch.cuda.current_stream()
    total = 0.0
    for _ in range(reps):
        torch.sum(flush, dim=0, out=sink)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        K.embedding_gather(lk, out, n)
        e1.record(stream)
        e1.synchronize()
        total += e0.elapsed_time(e1)
    ms = total / reps
    del flush, sink
    warm = _time(lambda: K.embedding_gather(lk, out, n), reps)  # same rows again: Infinity-Cache served
    alg = 2 * n * D * table.element_size() + 8 * n
    gbps = alg / (ms * 1e-3) / 1e9
    # context for the fraction: a contiguous copy of the same bytes in one launch, timed
    # the same way (cold, alone) -- at ~84 MB a launch's ramp and drain cap even that
    # near 0.62 of the HBM peak (scripts/microbench/gather.hip sweeps)
    src = torch.empty(n, D, dtype=table.dtype, device=table.device)
    flush = torch.ones(128 << 20, dtype=torch.int32, device=table.device)
    sink = torch.empty((), dtype=torch.int64, device=table.device)
    ctot = 0.0
    for _ in range(reps):
        torch.sum(flush, dim=0, out=sink)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        out.copy_(src)
        e1.record(stream)
        e1.synchronize()
        ctot += e0.elapsed_time(e1)
    cms = ctot / reps
    del flush, sink, src
    res = {'bound': 'hbm', 'kernel': 'grk::k_gather (item-table rows, 1M x 512 bf16)', 'achieved': round(gbps, 1),
           'peak': HBM_PEAK_GBPS, 'unit': 'GB/s', 'frac': round(gbps / HBM_PEAK_GBPS, 4), 'traffic': None,
           'alg_bytes_per_launch': int(alg), 'avg_launch_us': round(ms * 1e3, 2), 'rows_per_launch': int(n),
           'warm_cache_gbps': round(alg / (warm * 1e-3) / 1e9, 1),
           'copy_same_bytes_us': round(cms * 1e3, 2),
           'copy_same_bytes_frac': round((2 * n * D * table.element_size()) / (cms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
           'frac_of_copy': round(cms / ms, 4),
           'workload': {'rows': int(n), 'table_rows': int(table.shape[0]), 'D': int(D)}}
    p = _pmc(f'{PMC_TAG}_pmc_gather_item.json', res['workload'])
    if p is not None:
        res['traffic'] = int(p['traffic_bytes_per_launch'])
    return res


def _source_rows_read(s, token_type):
    """Distinct upstream gradient rows one lookup reads: its tokens with at least
    one non-padding row in the bag (a bag's slots share one gradient row)."""
    idx = s.idx.reshape(s.grad.shape[0], -1)
    live = (idx != 0).any(1)
    if s.mode in (1, 2) and token_type is not None:          # IDX_ITEM_MASK / IDX_USER_MASK
        live &= token_type.reshape(-1)[:live.numel()] == s.mode
    return int(live.sum().item())


def backward_rooflines(trace, reps):
    """grk_embedding_backward (key build, stable radix sort, segment bounds,
    segmented reduction: every launch of the call), timed alone with HIP
    events on the step's own arguments, for two calls of one step:

    * the item-table group (1M rows, row-sparse output): seq / pos / neg item
      rows -- the HBM-bound one;
    * the projected feature rows P (dense output, GRK_BWD_CHUNKED), the call
      with the most occurrences.

    Algorithmic bytes count DISTINCT data: each distinct upstream
    gradient row read once (a bag's slots and a row's repeated lookups re-read
    the same row, from cache), 8-B / 4-B indices per occurrence, and the output
    written once (dense: the whole [rows, D] fp32 gradient; sparse: unique
    rows x (D x 4 + 8 B id)).  The replays run last in bench.py, item call
    first (scripts/pmc_rooflines.py attributes the PMC windows by that order)."""
    from tencent_recommendation_2025_amd import kernels as K
    out = []
    item = [c for c in trace if c['sparse'] and not c.get('chunked')]
    proj = [c for c in trace if c.get('chunked')]
    picks = []
    if item:
        picks.append(('item', max(item, key=lambda c: c['num_rows']), 1))
    if proj:
        picks.append(('projected', max(proj, key=lambda c: sum(s.idx.numel() for s in c['sources'])), len(proj)))
    for kind, call, per_step in picks:
        def run(call=call):
            kw = dict(call)
            rs = kw.pop('row_slot')
            return K.embedding_backward(row_slot=None if rs is None else rs.clone(), **kw)

        res = run()
        srcs = call['sources']
        occ = sum(s.idx.numel() for s in srcs)
        D = call['dim']
        es = srcs[0].grad.element_size()
        isz = srcs[0].idx.element_size()
        uniq = int(res.count.item())
        seen, rows_read = set(), 0
        for s in srcs:
            key = (s.grad.data_ptr(), s.grad_col, s.grad.shape[0])
            if key not in seen:
                seen.add(key)
                rows_read += _source_rows_read(s, call['token_type'])
        dsz = 2 if call.get('dense_dtype') == torch.bfloat16 else 4
        written = call['num_rows'] * D * dsz if call['dense'] else uniq * (D * 4 + 8)
        alg = rows_read * D * es + occ * isz + written
        ms = _time(run, reps)
        gbps = alg / (ms * 1e-3) / 1e9
        res = {'bound': 'hbm',
               'kernel': f'grk_embedding_backward ({kind} '
                         + ('item-table group, row-sparse' if kind == 'item' else 'feature rows P, dense, chunked')
                         + ' gradient: all launches of the call)',
               'achieved': round(gbps, 1), 'peak': HBM_PEAK_GBPS, 'unit': 'GB/s',
               'frac': round(gbps / HBM_PEAK_GBPS, 4), 'traffic': None, 'alg_bytes_per_launch': int(alg),
               'avg_launch_us': round(ms * 1e3, 2), 'calls_per_step': per_step,
               'ms_per_step': round(ms * per_step, 4), 'pmc_calls': reps + 2,   # run() + _time's 1 + reps
               'alg_bytes_note': 'distinct upstream gradient rows read once + indices + output written once',
               'workload': {'table': kind, 'occurrences': int(occ), 'distinct_grad_rows': int(rows_read),
                            'unique_rows': uniq, 'table_rows': int(call['num_rows']), 'D': D,
                            'grad_dtype': str(srcs[0].grad.dtype), 'lookups': len(srcs)}}
        p = _pmc(f'{PMC_TAG}_pmc_emb_bwd_{kind}.json', res['workload'])
        if p is not None:
            res['traffic'] = int(p['traffic_bytes_per_launch'])
            res['traffic_note'] = (f'rocprofv3 PMC (profiles/{PMC_TAG}_pmc_emb_bwd_{kind}.json): FETCH_SIZE x2 + '
                                   'WRITE_SIZE summed over the launches of one call')
        out.append(res)
    return out


def ss_rooflines(batch, a, reps):
    """The in-batch sampled softmax of the bench batch (north star; grk_sampled_
    softmax_fwd / _bwd, every launch of each call), bf16 h / e of the valid
    positions, timed alone with HIP events.  MFMA-bound: nv valid positions,
    algorithmic FLOPs fwd 2 nv^2 D (the logits; the LSE is fused), bwd 6 nv^2 D
    (logits recomputed + dH = P E + dE = P^T H).  calls_per_step: 1 with
    --loss sampled_softmax, else 0 (the BCE step does not run it)."""
    from tencent_recommendation_2025_amd import kernels as K
    seq, pos, ntt = batch[0], batch[1], batch[4]
    B, T = seq.shape
    D = a.hidden
    if D not in (32, 64, 128, 256, 512):     # the kernel's head widths (C5's d = 1024 runs BCE only)
        return []
    dev = seq.device
    g = torch.Generator(device=dev).manual_seed(11)
    h = (0.1 * torch.randn(B * T, D, device=dev, generator=g)).bfloat16()
    e = (0.1 * torch.randn(B * T, D, device=dev, generator=g)).bfloat16()
    ids = pos.reshape(-1).long().contiguous()
    valid = (ntt.reshape(-1) == 1).to(torch.uint8).contiguous()
    nv = int(valid.sum().item())
    loss, lse2, _ = K.sampled_softmax_fwd(h, e, ids, valid, 0.05)
    t_f = _time(lambda: K.sampled_softmax_fwd(h, e, ids, valid, 0.05), reps)
    t_b = _time(lambda: K.sampled_softmax_bwd(h, e, ids, valid, 0.05, lse2), reps)
    per_step = 1 if a.loss == 'sampled_softmax' else 0
    out = []
    for name, ms, flops, alg, calls in (('fwd', t_f, 2.0 * nv * nv * D, 2 * nv * D * 2 + 8 * nv, reps + 2),
                                        ('bwd', t_b, 6.0 * nv * nv * D, 2 * nv * D * 2 + 2 * nv * D * 4 + 12 * nv,
                                         reps + 1)):
        tfs = flops / (ms * 1e-3) / 1e12
        res = {'bound': 'mfma', 'kernel': f'grk::k_ss_{name} (in-batch sampled softmax {name}, all launches)',
               'achieved': round(tfs, 1), 'peak': BF16_PEAK_TFLOPS, 'unit': 'TFLOP/s',
               'frac': round(tfs / BF16_PEAK_TFLOPS, 4), 'traffic': None, 'flops_per_launch': int(flops),
               'alg_bytes_per_launch': int(alg), 'avg_launch_us': round(ms * 1e3, 2), 'calls_per_step': per_step,
               'ms_per_step': round(ms * per_step, 4), 'pmc_calls': calls,
               'workload': {'valid_positions': nv, 'D': D, 'pass': name}}
        p = _pmc(f'{PMC_TAG}_pmc_ss_{name}.json', res['workload'])
        if p is not None:
            res['traffic'] = int(p['traffic_bytes_per_launch'])
        out.append(res)
    return out


def _wgrad_time(k, m, n, reps, out_dtype=torch.float32, want_db=True):
    from tencent_recommendation_2025_amd import kernels as K
    g = torch.Generator(device='cuda').manual_seed(0)
    dy = torch.randn(k, m, device='cuda', generator=g).bfloat16()
    x = torch.randn(k, n, device='cuda', generator=g).bfloat16()
    return _time(lambda: K.wgrad(dy, x, out_dtype=out_dtype, want_db=want_db), reps)


def wgrad_roofline(a, reps, k, wtrace=None):
    """grk_wgrad, the whole kernel family of one step (every k_wgrad
    instantiation counts toward the headline ranking): every weight gradient the
    step computes on grk_wgrad (recorded from one eager step: the HSTU uvqk and
    output projections, the item / user dnn weights ...), each shape timed alone
    (HIP events; k_wgrad + its in-order slice reduction).  MFMA bound: algorithmic
    FLOPs 2*K*M*N per call.  ``shapes`` lists each distinct shape; the uvqk one
    (dW [4D, D] over the K token rows of the step + bias gradient) carries the
    PMC traffic."""
    m, n = 4 * a.hidden, a.hidden
    calls = {}
    for kk, mm, nn, odt, db in (wtrace or [(k, m, n, torch.float32, True)] * a.blocks):
        key = (int(kk), int(mm), int(nn), odt, bool(db))
        calls[key] = calls.get(key, 0) + 1
    shapes, tot_ms, tot_flops, launches = [], 0.0, 0, 0
    for (kk, mm, nn, odt, db), cnt in sorted(calls.items(), key=lambda kv: -kv[0][0] * kv[0][1] * kv[0][2]):
        ms = _wgrad_time(kk, mm, nn, reps, odt, db)
        fl = 2 * kk * mm * nn
        tot_ms += ms * cnt
        tot_flops += fl * cnt
        launches += cnt
        shapes.append({'K': kk, 'M': mm, 'N': nn, 'calls_per_step': cnt, 'avg_launch_us': round(ms * 1e3, 2),
                       'tflops': round(fl / (ms * 1e-3) / 1e12, 1),
                       'frac': round(fl / (ms * 1e-3) / 1e12 / BF16_PEAK_TFLOPS, 4)})
    tf = tot_flops / (tot_ms * 1e-3) / 1e12
    uvqk = next((s for s in shapes if s['M'] == m and s['N'] == n), None)
    res = {'bound': 'mfma', 'kernel': 'grk::k_wgrad* + k_wgrad_reduce (every weight + bias gradient of the step)',
           'achieved': round(tf, 1), 'peak': BF16_PEAK_TFLOPS, 'unit': 'TFLOP/s',
           'frac': round(tf / BF16_PEAK_TFLOPS, 4), 'traffic': None, 'flops_per_step': int(tot_flops),
           'avg_launch_us': round(tot_ms / launches * 1e3, 2), 'calls_per_step': launches,
           'ms_per_step': round(tot_ms, 4), 'shapes': shapes,
           'workload': {'K': int(k), 'M': int(m), 'N': int(n)}}
    p = _pmc(f'{PMC_TAG}_pmc_wgrad.json', res['workload'])
    if p is not None and uvqk is not None:
        uvqk['traffic'] = int(p['traffic_bytes_per_launch'])
        uvqk['alg_bytes_per_launch'] = int(2 * k * (m + n) + 4 * m * (n + 1))
        # the family's traffic field: its largest launch's (uvqk: ring kernel + slice reduction)
        res['traffic'] = uvqk['traffic']
        res['traffic_note'] = ('rocprofv3 PMC (profiles/%s_pmc_wgrad.json) of the uvqk shape (dW [4D, D] + db, '
                               'the largest launch): FETCH_SIZE x2 + WRITE_SIZE; algorithmic %d B'
                               % (PMC_TAG, uvqk['alg_bytes_per_launch']))
    return res


def catchup_roofline(opt, reps, batch=None):
    """The deferred dense-parity table AdamW's replays (FusedAdamW rolling, round 5),
    every k_adamw_catchup launch of a step: per deferred table the
    batch rows' catch-up at the head of the step (the rows the step reads, brought to
    the current step) and the rolling flush slice (a 1/period slice of its rows, each
    row replaying the g = 0 steps it lags).  Timed on copies of the item table's state
    as the timed region left it (the slice the clock points at, its real lags), last[]
    restored before every launch; the batch-row launch on the first pool batch's ids.
    Algorithmic bytes: moved rows x D x (2 + 4 + 4) B read and written + 8 B of last[]
    per row; the kernel is VALU-bound (~100 instructions, 16 of them sqrt / rcp, per
    replayed step of 8 elements), reported against HBM."""
    from tencent_recommendation_2025_amd import kernels as K
    if not getattr(opt, 'rolling', False):
        return None
    g = opt._deferred.get('item') or next(iter(opt._deferred.values()))
    period = opt._period
    p, m, v = g.flat.clone(), g.exp_avg.clone(), g.exp_avg_sq.clone()
    last0 = g.last.clone()
    last = last0.clone()
    t = int(opt.clock.t.item())
    rows, D = p.shape
    per = -(-rows // period)
    s = t % period
    lo, hi = s * per, min(rows, (s + 1) * per)
    lag = (t - last0[lo:hi].long()).clamp(min=0)
    stream = torch.cuda.current_stream()

    def timed(fn):
        total = 0.0
        for _ in range(reps):
            last.copy_(last0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            fn()
            e1.record(stream)
            e1.synchronize()
            total += e0.elapsed_time(e1)
        return total / reps

    # the batch rows' catch-up first: rows the batch reads, from the state the timed region
    # left (their lag since they were last read or flushed, at most one period); then the
    # slice, whose launches end the run's catch-ups (scripts/pmc_rooflines.py takes the
    # PMC traffic of the last launches)
    b_ms = b_alg = 0.0
    if batch is not None:
        ids = K.batch_row_ids(*batch[:4], with_user=False)[0]
        b_ms = timed(lambda: K.table_adamw_catchup(p, m, v, last, None, opt.clock, ids))
        u = ids[ids > 0].unique()
        b_moved = int(((t - last0[u].long()) > 0).sum().item())
        b_alg = b_moved * D * (p.element_size() + 8) * 2 + ids.numel() * 8 + u.numel() * 8
    ms = timed(lambda: K.table_adamw_catchup_slice(p, m, v, last, opt.clock, period))
    n = hi - lo
    moved = int((lag > 0).sum().item())
    alg = moved * D * (p.element_size() + 8) * 2 + n * 8
    calls = len(opt._deferred)
    launches = calls * (2 if batch is not None else 1)
    tot_ms = calls * (ms + b_ms)
    tot_alg = calls * (alg + b_alg)
    gbps = tot_alg / (tot_ms * 1e-3) / 1e9
    res = {'bound': 'hbm', 'kernel': 'grk::k_adamw_catchup (every launch of a step: per deferred table the batch '
                                     'rows\' catch-up + the rolling flush slice, 1/%d of a 1M-row table)' % period,
           'achieved': round(gbps, 1), 'peak': HBM_PEAK_GBPS, 'unit': 'GB/s', 'frac': round(gbps / HBM_PEAK_GBPS, 4),
           'traffic': None, 'alg_bytes_per_launch': int(tot_alg / launches),
           'avg_launch_us': round(tot_ms / launches * 1e3, 2), 'calls_per_step': launches,
           'ms_per_step': round(tot_ms, 4),
           'slice': {'avg_launch_us': round(ms * 1e3, 2), 'alg_bytes_per_launch': int(alg),
                     'replayed_steps_per_launch': int(lag.sum().item()), 'rows_moved_per_launch': moved,
                     'mean_lag_steps': round(float(lag.float().mean().item()), 2)},
           'batch_rows': {'avg_launch_us': round(b_ms * 1e3, 2), 'alg_bytes_per_launch': int(b_alg)},
           'note': 'VALU-bound: the g = 0 AdamW replay is ~100 VALU instructions (16 of them 8-cycle '
                   'sqrt / rcp) per replayed step of 8 elements',
           'workload': {'table_rows': int(rows), 'D': int(D), 'slice_rows': int(n), 'period': int(period)}}
    p_ = _pmc(f'{PMC_TAG}_pmc_catchup.json', {k: res['workload'][k] for k in ('table_rows', 'D', 'period')})
    if p_ is not None:
        res['slice']['traffic'] = int(p_['traffic_bytes_per_launch'])
        res['traffic_note'] = f'PMC of the slice launch only: slice.traffic (profiles/{PMC_TAG}_pmc_catchup.json)'
    del p, m, v, last, last0
    return res


def family_entry(name, members):
    """One kernel family (the headline is ONE rule -- the family with
    the most device time per step): every launch of the family in one step, i.e. its
    members' ms_per_step summed, and its rate = the members' algorithmic bytes (HBM
    bound) or FLOPs (MFMA bound) per step over that time.  ``traffic`` is the PMC HBM
    bytes per launch averaged over the members that carry one (None if none does)."""
    members = [r for r in members if r and r.get('peak') and r.get('ms_per_step')]
    if not members:
        return None
    bound = members[0]['bound']
    ms = sum(r['ms_per_step'] for r in members)
    calls = sum(r.get('calls_per_step', 1) for r in members)
    if bound == 'mfma':
        work = sum(r.get('flops_per_launch', 0) * r.get('calls_per_step', 1) for r in members) \
            or sum(r.get('flops_per_step', 0) for r in members)
        achieved, peak, unit = work / (ms * 1e-3) / 1e12, BF16_PEAK_TFLOPS, 'TFLOP/s'
    else:
        work = sum(r.get('alg_bytes_per_launch', 0) * r.get('calls_per_step', 1) for r in members)
        achieved, peak, unit = work / (ms * 1e-3) / 1e9, HBM_PEAK_GBPS, 'GB/s'
    with_t = [r for r in members if r.get('traffic')]
    traffic = alg = None
    if with_t:
        c = sum(r.get('calls_per_step', 1) for r in with_t)
        traffic = int(sum(r['traffic'] * r.get('calls_per_step', 1) for r in with_t) / c)
        alg = int(sum(r.get('alg_bytes_per_launch', 0) * r.get('calls_per_step', 1) for r in with_t) / c)
    return {'family': name, 'bound': bound, 'kernel': name + ': ' + ' + '.join(r['kernel'] for r in members),
            'achieved': round(achieved, 1), 'peak': peak, 'unit': unit, 'frac': round(achieved / peak, 4),
            'traffic': traffic, 'traffic_alg_bytes_per_launch': alg,
            'avg_launch_us': round(ms / calls * 1e3, 2), 'calls_per_step': calls, 'ms_per_step': round(ms, 4),
            'members': [r['kernel'] for r in members]}


_T0 = time.perf_counter()


def progress(msg):
    """One stderr line per phase (stdout keeps the single JSON line): a run whose
    phases take minutes in total -- model build, capture, rooflines, the CPU
    baseline -- always shows it is alive."""
    print(f'# bench {time.perf_counter() - _T0:7.1f} s: {msg}', file=sys.stderr, flush=True)


def cpu_baseline(a, stats, types):
    """fp32 torch-CPU restatement (oracle/model_ref.py) of the same model + step, bounded sample."""
    from oracle import model_ref
    from tencent_recommendation_2025_amd import synthetic as S
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        cores = os.cpu_count() or 1
    cores = max(1, min(cores, 16))   # the GPU box's CPU share is 16 threads per GPU
    torch.set_num_threads(cores)
    model_name = 'unknown CPU'
    try:
        with open('/proc/cpuinfo') as f:
            model_name = next((ln.split(':', 1)[1].strip() for ln in f if ln.startswith('model name')), model_name)
    except OSError:  # pragma: no cover
        pass
    cfg = S.SyntheticConfig(batch_size=a.cpu_batch, maxlen=a.maxlen, num_items=a.items, num_users=a.users,
                            zipf=a.zipf)
    margs = S.make_args(hidden_units=a.hidden, maxlen=a.maxlen, num_blocks=a.blocks, num_heads=a.heads,
                        block=a.block, device='cpu', dropout_rate=a.dropout)
    ref = model_ref.RefBaselineModel(a.users, a.items, stats, types, margs, variant='o1', block=a.block)
    model_ref.init_params(ref, seed=0)
    opt = torch.optim.AdamW(ref.parameters(), lr=1e-3, betas=(0.9, 0.98), weight_decay=0.01)
    g = torch.Generator().manual_seed(0)
    batches = [S.make_batch(cfg, g, 'cpu') for _ in range(a.cpu_steps + 1)]

    def step(b):
        seq, pos, neg, tt, ntt, _nat, sf, pf, nf = b
        opt.zero_grad()
        if a.loss == 'bce':
            pl, nl = ref(seq, pos, neg, tt, ntt, sf, pf, nf)
            loss = model_ref.bce_loss(pl, nl, ntt)
        else:
            h = ref.log2feats(seq, tt, sf)
            pe = ref.feat2emb(pos, pf, include_user=False)
            loss = model_ref.sampled_softmax_loss(h, pe, pos, ntt, 0.05)
        loss.backward()
        opt.step()

    step(batches[0])
    progress(f'cpu baseline: warm-up step done ({cores} threads)')
    times = []
    for i, b in enumerate(batches[1:]):
        t0 = time.perf_counter()
        step(b)
        times.append(time.perf_counter() - t0)
        progress(f'cpu baseline: step {i + 1}/{len(batches) - 1} {times[-1]:.1f} s')
    dt = sum(times)
    n = a.cpu_batch * a.cpu_steps
    rates = sorted(a.cpu_batch / t for t in times)
    mean = n / dt
    sd = (sum((r - mean) ** 2 for r in rates) / max(len(rates) - 1, 1)) ** 0.5
    return {'value': round(mean, 3), 'unit': 'seq/s', 'cores': cores, 'kind': 'port', 'cpu_model': model_name,
            'per_step_seq_s': {'min': round(rates[0], 3), 'median': round(rates[len(rates) // 2], 3),
                               'max': round(rates[-1], 3), 'stdev': round(sd, 3), 'steps': len(rates)},
            'sample': f'{a.cpu_steps} timed steps x B={a.cpu_batch} of the same model/config/loss '
                      f'(fp32 CPU, full {a.items}-row item table, dense AdamW, dropout {a.dropout}), after 1 warmup step, '
                      f'{cores} threads on {model_name}; {dt:.1f} s (BASELINE.md 3 asks 10 warmup + 50 timed steps: '
                      f'bounded to keep the bench within minutes)'}


FP32_VALU_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 vector (packed FMA)


def semantic_id_setup(a, dev, reps):
    """Config 4: train an RQ-VAE briefly on the items' mm rows (feature 81,
    [items, 32] -> latent 64 -> levels x sid_codes codes; k-means init, 30 Adam
    steps of 16384 rows, timed), tokenise the whole item table and return the
    per-item semantic-id rows plus the code search's roofline entry.

    grk_rq_assign is VALU-bound: per row levels * codes * latent * 3 FLOP (one
    difference, square and add per element; no FMA so the codes are exact).  A
    packed v_pk_add/v_pk_mul issue does 2 FLOP per lane, half a packed FMA's
    4, so the FMA-free ceiling is 0.5 of the 157.3 TFLOP/s vector peak."""
    from tencent_recommendation_2025_amd.rqvae import RQVAE, rq_assign, semantic_id_table
    g = torch.Generator(device=dev).manual_seed(81)
    mm = torch.randn(a.items, 32, device=dev, generator=g)
    torch.manual_seed(4)
    tok = RQVAE(32, hidden=(256, 128), latent_dim=64, levels=a.semantic_ids, codebook_size=a.sid_codes).to(dev)
    tok.init_codebooks(mm[:65536], iters=5)
    # a short tokenizer training run (MSE + codebook + commitment, Adam), timed
    opt = torch.optim.Adam(tok.parameters(), lr=1e-3)
    tb = 16384
    train_steps = 30
    for i in range(train_steps + 3):
        if i == 3:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        x = mm[(i * tb) % (a.items - tb):][:tb]
        opt.zero_grad(set_to_none=True)
        loss = tok(x)[2]['loss']
        loss.backward()
        opt.step()
    torch.cuda.synchronize()
    train_rows_s = train_steps * tb / (time.perf_counter() - t0)
    t0 = time.perf_counter()
    codes = tok.tokenize(mm)
    torch.cuda.synchronize()
    tok_s = time.perf_counter() - t0
    with torch.no_grad():
        z = tok.encode(mm)
    cb = tok.codebooks.detach().contiguous()
    ms = _time(lambda: rq_assign(z, cb, want_quant=False), reps)
    flops = 3.0 * a.items * a.semantic_ids * a.sid_codes * 64
    tfs = flops / (ms * 1e-3) / 1e12
    roof = {'bound': 'valu', 'kernel': 'grk::k_rq_assign<64> (RQ-VAE code search, whole item table)',
            'achieved': round(tfs, 1), 'peak': FP32_VALU_PEAK_TFLOPS, 'unit': 'TFLOP/s',
            'frac': round(tfs / FP32_VALU_PEAK_TFLOPS, 4), 'fma_free_ceiling_frac': 0.5, 'traffic': None,
            'avg_launch_us': round(ms * 1e3, 1), 'flops_per_launch': int(flops),
            'alg_bytes_per_launch': int(a.items * (64 * 4 + a.semantic_ids * 4)),
            'tokenize_items_per_s': round(a.items / tok_s, 1),
            'tokenizer_train_rows_per_s': round(train_rows_s, 1), 'tokenizer_train_batch': tb,
            'tokenizer_final_loss': round(float(loss.item()), 5),
            'workload': {'rows': a.items, 'latent': 64, 'levels': a.semantic_ids, 'codes': a.sid_codes}}
    p = _pmc('r2s7_pmc_rq_assign.json', roof['workload'])
    if p is not None:
        roof['traffic'] = int(p['traffic_bytes_per_launch'])
        roof['traffic_note'] = ('rocprofv3 PMC (profiles/r2s7_pmc_rq_assign.json): FETCH_SIZE x2 + WRITE_SIZE '
                                '(MI355X_MICROARCH.md gfx950 corrections)')
    sid = semantic_id_table(codes, a.items)
    del mm, z, tok
    return sid, roof


def _rooflines(a, kv, jagged, rows, trace, btrace, model, pool, sid_roof, wtrace=None, opt=None):
    """Every measured kernel (after the timed region): (headline roofline, the others).

    The headline is the kernel FAMILY with the most device time per step (every launch
    of the family in one step; one rule for all of them): the attention kernels of every
    layer (forward, dQ, dK/dV), the weight gradients, the table AdamW replays, the
    embedding backward calls, the sampled softmax (with --loss sampled_softmax).  The
    family entries head ``rooflines``, followed by every member and the unranked
    entries (cold item gather, seq-side gather, RQ-VAE code search)."""
    from tencent_recommendation_2025_amd import jagged as J
    dkdv, (fwd, dq) = attention_rooflines(a, kv, a.roofline_reps, jagged=jagged)
    progress('rooflines: attention')
    others = [gather_roofline(trace, a.roofline_reps)]
    item_table = model.item_emb.weight if model.item_emb.weight.numel() else None
    if item_table is not None:
        others.append(item_gather_roofline(item_table.detach(), pool[0], a.roofline_reps))
    progress('rooflines: gathers')
    wk = J.capacity_for(rows[0], a.jagged_quantum) if jagged else a.batch * (a.maxlen + 1)
    wg = wgrad_roofline(a, a.roofline_reps, wk, wtrace)
    ss = ss_rooflines(pool[0], a, a.roofline_reps)
    progress('rooflines: wgrad, sampled softmax')
    cu = catchup_roofline(opt, a.roofline_reps, pool[0]) if opt is not None else None
    if cu is not None:
        progress('rooflines: table AdamW replays')
    eb = []
    if btrace:   # last: scripts/pmc_rooflines.py finds these calls' PMC windows at the end of the run
        eb = backward_rooflines(btrace, a.roofline_reps)
        progress('rooflines: embedding backward')
    if sid_roof is not None:
        others.append(sid_roof)
    fams = [family_entry('HSTU attention (fwd + dQ + dK/dV, every layer)' if a.block == 'hstu'
                         else 'softmax attention (fwd + dQ + dK/dV, every layer)', [fwd, dq, dkdv]),
            family_entry('weight gradients (grk_wgrad, every dense layer)', [wg]),
            family_entry('table AdamW replays (k_adamw_catchup)', [cu]),
            family_entry('embedding backward (grk_embedding_backward calls)', eb),
            family_entry('in-batch sampled softmax (fwd + bwd)', ss)]
    fams = sorted((f for f in fams if f is not None), key=lambda f: -f['ms_per_step'])
    roof = fams[0]
    members = [fwd, dq, dkdv, wg] + ([cu] if cu else []) + eb + ss
    return roof, fams[1:] + members + others


def main():
    a = parse()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    ndev = torch.cuda.device_count()
    dev = torch.device('cuda', local % max(ndev, 1))
    torch.cuda.set_device(dev)
    sharded = (world > 1) if a.sharded is None else bool(a.sharded)
    if world > 1 or sharded:
        for k, v in (('RANK', '0'), ('WORLD_SIZE', '1'), ('MASTER_ADDR', '127.0.0.1'), ('MASTER_PORT', '29533')):
            os.environ.setdefault(k, v)      # --sharded 1 without a launcher: a world of one
        if a.backend == 'nccl':
            dist.init_process_group('nccl', device_id=dev)
        else:
            dist.init_process_group('gloo')

    from tencent_recommendation_2025_amd import functional as G
    from tencent_recommendation_2025_amd import synthetic as S
    from tencent_recommendation_2025_amd.model import BaselineModel, init_reference_
    from tencent_recommendation_2025_amd.optim import FusedAdamW
    from tencent_recommendation_2025_amd.train import Trainer

    sid, sid_roof = (semantic_id_setup(a, dev, a.roofline_reps) if a.semantic_ids else (None, None))
    cfg = S.SyntheticConfig(batch_size=a.batch, maxlen=a.maxlen, num_items=a.items, num_users=a.users, zipf=a.zipf,
                            timestamps=a.time_buckets > 0, sid_table=sid, sid_codes=a.sid_codes)
    stats, types = S.feature_schema(cfg)
    if a.fp8 and (a.block != 'hstu' or a.time_buckets):
        raise SystemExit('--fp8 takes HSTU blocks without the time bias (chunked fp8 kernels)')
    margs = S.make_args(hidden_units=a.hidden, maxlen=a.maxlen, num_blocks=a.blocks, num_heads=a.heads,
                        block=a.block, dropout_rate=a.dropout, hstu_time_buckets=a.time_buckets,
                        hstu_fp8=bool(a.fp8))
    shard_tables = sharded and (a.shard_tables if a.shard_tables is not None else a.items >= 10_000_000)
    margs.shard_tables = bool(shard_tables)
    margs.merge_proj_backward = bool(a.merge_proj)
    margs.grouped_proj = bool(a.grouped_proj)
    progress(f'rank {rank}/{world}: building the model')
    torch.manual_seed(0)
    model = BaselineModel(a.users, a.items, stats, types, margs).to(dev)
    model.train()
    init_reference_(model, seed=0, live_norms=True)
    if sharded:
        from tencent_recommendation_2025_amd.sharding import ShardedFusedAdamW
        opt = ShardedFusedAdamW(model, lr=1e-3, weight_decay=0.01, table_mode=a.table_mode)
    else:
        opt = FusedAdamW(model, lr=1e-3, weight_decay=0.01, table_mode=a.table_mode, dense_flat=bool(a.dense_flat))
    # the jagged layout runs on the whole-sequence attention kernels (T <= 256 at hd <= 128, not fp8)
    jagged = (bool(a.jagged) and (not sharded or bool(a.sharded_jagged)) and not a.fp8 and a.maxlen + 1 <= 256
              and a.hidden // a.heads <= 128)
    trainer = Trainer(model, opt, loss=a.loss, graph=bool(a.graph), jagged=jagged, jagged_quantum=a.jagged_quantum)
    gen = torch.Generator(device=dev).manual_seed(1234 + rank)
    # each pooled batch in one device arena (train.pack_batch): a graph replay copies it in one launch
    from tencent_recommendation_2025_amd.train import pack_batch
    pool = [pack_batch(S.make_batch(cfg, gen, dev)) for _ in range(max(2, a.pool))]
    from tencent_recommendation_2025_amd import jagged as J
    # the data loader knows its batches' lengths: the span-row counts are host
    # metadata of the pool, computed once here (not inside the timed steps)
    rows = [J.span_rows(b[3]) if jagged else None for b in pool]
    caps = sorted({J.capacity_for(r, a.jagged_quantum) for r in rows}) if jagged else []

    from tencent_recommendation_2025_amd import kernels as K
    trace = btrace = wtrace = None
    def step(i):
        return trainer.step(pool[i % len(pool)], next_batch=pool[(i + 1) % len(pool)], rows=rows[i % len(pool)])

    progress('warm-up steps')
    for i in range(a.warmup):
        if i == 0:
            G.GATHER_TRACE = []          # record the fused-gather launches of one real (eager) step
            K.BACKWARD_TRACE = []        # ... its embedding-table gradients
            K.WGRAD_TRACE = []           # ... and its weight gradients
        step(i)
        if i == 0:
            trace, G.GATHER_TRACE = G.GATHER_TRACE, None
            btrace, K.BACKWARD_TRACE = K.BACKWARD_TRACE, None
            wtrace, K.WGRAD_TRACE = K.WGRAD_TRACE, None
    # jagged + graph: one captured graph per capacity of the pool, captured before the
    # timed region (extra untimed steps on the batches of a capacity not captured yet)
    # Every rank takes the same number of steps (each one's collectives: the row
    # exchange and the all-reduces); a rank whose pool has its capacities captured
    # keeps stepping until every rank's are.  The batch sequence continues from the
    # warm-up, so every prefetch is the batch of the step after it.
    prewarm = 0
    if jagged and trainer.graph:
        k = a.warmup
        while True:
            done = all(c in trainer._graphs for c in caps)
            if world > 1:
                flag = torch.tensor([0 if done else 1], dtype=torch.int32, device=dev)
                dist.all_reduce(flag, op=dist.ReduceOp.MAX)
                done = int(flag.item()) == 0
            if done:
                break
            step(k)
            k += 1
            prewarm += 1
    first = a.warmup + prewarm
    torch.cuda.synchronize()
    progress(f'timed region: {a.steps} steps ({prewarm} prewarm steps captured the remaining capacities)')
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    evs, host = [], []
    for i in range(a.steps):
        th = time.perf_counter()
        loss = step(first + i)
        if a.step_times:
            host.append(time.perf_counter() - th)
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            evs.append(e)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    final_loss = float(loss.float().item())
    if a.step_times and rank == 0:
        dev_ms = [evs[i].elapsed_time(evs[i + 1]) for i in range(len(evs) - 1)]
        caps_i = [J.capacity_for(rows[(first + i) % len(pool)], a.jagged_quantum) if jagged else 0
                  for i in range(a.steps)]
        print('# step device intervals (ms) / host issue (ms) / capacity:', file=sys.stderr)
        for i, d in enumerate(dev_ms):
            print(f'  {i + 1:3d} {d:7.3f} {1e3 * host[i + 1]:7.3f} {caps_i[i + 1]}', file=sys.stderr)

    if not trace:  # --warmup 0: trace one extra, untimed eager step after the timed region
        G.GATHER_TRACE, K.BACKWARD_TRACE, K.WGRAD_TRACE = [], [], []
        trainer.eager_step(pool[0])
        trace, G.GATHER_TRACE = G.GATHER_TRACE, None
        btrace, K.BACKWARD_TRACE = K.BACKWARD_TRACE, None
        wtrace, K.WGRAD_TRACE = K.WGRAD_TRACE, None
    kv = (pool[0][3] != 0).to(torch.uint8)        # the first bench batch's key validity (token_type != 0)
    roof, more = None, []
    progress(f'timed region done: {elapsed / a.steps * 1e3:.3f} ms/step')
    if a.rooflines:
        roof, more = _rooflines(a, kv, jagged, rows, trace, btrace, model, pool, sid_roof, wtrace,
                                None if sharded else opt)
        progress('rooflines done')

    cpu = None
    if rank == 0 and world == 1 and a.cpu_baseline and not a.semantic_ids and not a.fp8:   # config 2's CPU model only
        cpu = cpu_baseline(a, stats, types)

    if rank == 0:
        value = a.batch * world * a.steps / elapsed
        line = {
            'metric': 'seq/sec training throughput, TencentGR HSTU d=512 L=200, at 1/2/4/8 MI355X',
            'value': round(value, 2), 'unit': 'seq/s', 'n_gpus': world, 'steps': a.steps, 'warmup': a.warmup,
            'ms_per_step': round(elapsed / a.steps * 1e3, 3), 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': None, 'dtype': 'bf16+fp8' if a.fp8 else 'bf16', 'data': 'synthetic (device-resident TencentGR-shaped batches)',
            'config': {'workload': f'BASELINE config {5 if a.fp8 else 4 if a.semantic_ids else 3 if shard_tables else 2}: '
                                   + (f'O1 + RQ-VAE semantic ids ({a.semantic_ids} levels x {a.sid_codes} codes '
                                      f'as item_sparse features), ' if a.semantic_ids else '')
                                   + f'{a.block.upper()} d={a.hidden} L={a.maxlen} '
                                   f'({a.blocks} blocks x {a.heads} heads), {a.items}-item bf16 table, '
                                   f'{a.users} users, loss={a.loss}, table AdamW={a.table_mode}, '
                                   f'dropout={a.dropout}'
                                   + (f', rab_time buckets={a.time_buckets}' if a.time_buckets else '')
                                   + (', fp8 (e4m3) q/k/v attention' if a.fp8 else '')
                                   + (', merged projected-row backward' if a.merge_proj else '')
                                   + (', grouped MFMA projections' if a.grouped_proj else '')
                                   + (', flat dense AdamW' if a.dense_flat else ''),
                       'global_batch': a.batch * world, 'per_gpu_batch': a.batch, 'seq_len': a.maxlen + 1,
                       'parallelism': f'dp{world}' + ('+rowshard' if sharded else '') + ('(shard-built tables)' if shard_tables else ''),
                       'step_launch': 'hip-graph replay' if trainer.graph else 'eager',
                       'batch_pool': len(pool),
                       'layout': (f'jagged (span rows only, capacity quantum {a.jagged_quantum}: '
                                  f'{len(caps)} capacities {caps}, span rows {min(rows)}-{max(rows)} of '
                                  f'{a.batch * (a.maxlen + 1)})') if jagged else 'padded [B, T]',
                       'prewarm_steps': prewarm},
            'final_loss': round(final_loss, 5),
            'roofline': roof,
            'rooflines': more,
            'cpu_baseline': cpu,
        }
        print(json.dumps(line), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
