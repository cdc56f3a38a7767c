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
dominant hand-written kernel (the fused seq-side embedding gather, HBM-bound)
and the CPU baseline (oracle/model_ref.py, the fp32 torch-CPU restatement of
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
    ap.add_argument('--steps', type=int, default=20)
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
    ap.add_argument('--cpu-baseline', type=int, default=1)
    ap.add_argument('--cpu-batch', type=int, default=8)
    ap.add_argument('--cpu-steps', type=int, default=2)
    ap.add_argument('--roofline-reps', type=int, default=20)
    ap.add_argument('--backend', default='nccl', choices=['nccl', 'gloo'],
                    help='gloo: rehearse N ranks on fewer GPUs (collectives staged via host)')
    ap.add_argument('--sharded', type=int, default=None, help='force the row-sharded optimizer (default: N > 1)')
    return ap.parse_args()


def gather_roofline(trace, reps):
    """Time the seq-side fused gather alone with HIP events on its stream."""
    from tencent_recommendation_2025_amd import kernels as K
    lookups, out, n, tt, T = max(trace, key=lambda r: r[1].shape[1])  # widest = seq side
    stream = torch.cuda.current_stream()
    K.embedding_gather(lookups, out, n, tt, T)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        K.embedding_gather(lookups, out, n, tt, T)
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    D = lookups[0].table.shape[1]
    es = lookups[0].table.element_size()
    rows = n * sum(lk.bag for lk in lookups)
    idx_bytes = sum(lk.idx.numel() * lk.idx.element_size() for lk in lookups)
    tt_bytes = n * 4 if tt is not None else 0
    alg = rows * D * es + n * D * len(lookups) * es + idx_bytes + tt_bytes
    gbps = alg / (ms * 1e-3) / 1e9
    res = {'bound': 'hbm', 'kernel': 'grk::k_gather (seq-side fused lookup)', 'achieved': round(gbps, 1),
           'peak': HBM_PEAK_GBPS, 'unit': 'GB/s', 'frac': round(gbps / HBM_PEAK_GBPS, 4), 'traffic': None,
           'alg_bytes_per_launch': int(alg), 'avg_launch_us': round(ms * 1e3, 2),
           'rows_per_launch': int(rows), 'features': len(lookups)}
    # HBM bytes per launch from the committed rocprofv3 PMC passes of this same workload
    pmc = os.path.join(REPO, 'profiles', 'r1_pmc_gather.json')
    if os.path.exists(pmc):
        with open(pmc) as f:
            p = json.load(f)
        if abs(p['write_bytes_per_launch'] - n * D * len(lookups) * es) < 1e6:  # same output bytes => same workload
            res['traffic'] = int(p['traffic_bytes_per_launch'])
            res['traffic_note'] = ('rocprofv3 PMC (profiles/r1_pmc_gather.json): FETCH_SIZE x2 + WRITE_SIZE; '
                                   'reads of small/padding rows hit L2, so traffic < algorithmic bytes')
            res['traffic_gbps'] = round(p['traffic_bytes_per_launch'] / (ms * 1e-3) / 1e9, 1)
    return res


def cpu_baseline(a, stats, types):
    """fp32 torch-CPU restatement (oracle/model_ref.py) of the same model + step, bounded sample."""
    from oracle import model_ref
    from tencent_recommendation_2025_amd import synthetic as S
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        cores = os.cpu_count() or 1
    cores = max(1, min(cores, 16))
    torch.set_num_threads(cores)
    cfg = S.SyntheticConfig(batch_size=a.cpu_batch, maxlen=a.maxlen, num_items=a.items, num_users=a.users,
                            zipf=a.zipf)
    margs = S.make_args(hidden_units=a.hidden, maxlen=a.maxlen, num_blocks=a.blocks, num_heads=a.heads,
                        block=a.block, device='cpu')
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
    t0 = time.perf_counter()
    for b in batches[1:]:
        step(b)
    dt = time.perf_counter() - t0
    n = a.cpu_batch * a.cpu_steps
    return {'value': round(n / dt, 3), 'unit': 'seq/s', 'cores': cores, 'kind': 'port',
            'sample': f'{a.cpu_steps} timed steps x B={a.cpu_batch} of the same model/config/loss '
                      f'(fp32 CPU, full {a.items}-row item table, dense AdamW), after 1 warmup step; '
                      f'{dt:.1f} s'}


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
        if a.backend == 'nccl':
            dist.init_process_group('nccl', device_id=dev)
        else:
            dist.init_process_group('gloo')

    from tencent_recommendation_2025_amd import functional as G
    from tencent_recommendation_2025_amd import synthetic as S
    from tencent_recommendation_2025_amd.model import BaselineModel, init_reference_
    from tencent_recommendation_2025_amd.optim import FusedAdamW
    from tencent_recommendation_2025_amd.train import Trainer

    cfg = S.SyntheticConfig(batch_size=a.batch, maxlen=a.maxlen, num_items=a.items, num_users=a.users, zipf=a.zipf)
    stats, types = S.feature_schema(cfg)
    margs = S.make_args(hidden_units=a.hidden, maxlen=a.maxlen, num_blocks=a.blocks, num_heads=a.heads,
                        block=a.block)
    torch.manual_seed(0)
    model = BaselineModel(a.users, a.items, stats, types, margs).to(dev)
    init_reference_(model, seed=0, live_norms=True)
    if sharded:
        from tencent_recommendation_2025_amd.sharding import ShardedFusedAdamW
        opt = ShardedFusedAdamW(model, lr=1e-3, weight_decay=0.01, table_mode=a.table_mode)
    else:
        opt = FusedAdamW(model, lr=1e-3, weight_decay=0.01, table_mode=a.table_mode)
    trainer = Trainer(model, opt, loss=a.loss)
    gen = torch.Generator(device=dev).manual_seed(1234 + rank)
    pool = [S.make_batch(cfg, gen, dev) for _ in range(4)]

    for i in range(a.warmup):
        if i == a.warmup - 1:
            G.GATHER_TRACE = []          # capture the fused-gather launches of one real step
        trainer.step(pool[i % len(pool)])
    trace, G.GATHER_TRACE = G.GATHER_TRACE, None
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(a.steps):
        loss = trainer.step(pool[i % len(pool)])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    final_loss = float(loss.float().item())

    if not trace:  # --warmup 0: trace one extra, untimed step after the timed region
        G.GATHER_TRACE = []
        trainer.step(pool[0])
        trace, G.GATHER_TRACE = G.GATHER_TRACE, None
    roof = gather_roofline(trace, a.roofline_reps)

    cpu = None
    if rank == 0 and world == 1 and a.cpu_baseline:
        cpu = cpu_baseline(a, stats, types)

    if rank == 0:
        value = a.batch * world * a.steps / elapsed
        line = {
            'metric': 'seq/sec training throughput, TencentGR HSTU d=512 L=200, at 1/2/4/8 MI355X',
            'value': round(value, 2), 'unit': 'seq/s', 'n_gpus': world, 'steps': a.steps, 'warmup': a.warmup,
            'ms_per_step': round(elapsed / a.steps * 1e3, 3), 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': None, 'dtype': 'bf16', 'data': 'synthetic (device-resident TencentGR-shaped batches)',
            'config': {'workload': f'BASELINE config 2: {a.block.upper()} d={a.hidden} L={a.maxlen} '
                                   f'({a.blocks} blocks x {a.heads} heads), {a.items}-item bf16 table, '
                                   f'{a.users} users, loss={a.loss}, table AdamW={a.table_mode}',
                       'global_batch': a.batch * world, 'per_gpu_batch': a.batch, 'seq_len': a.maxlen + 1,
                       'parallelism': f'dp{world}' + ('+rowshard' if sharded else '')},
            'final_loss': round(final_loss, 5),
            'roofline': roof,
            'cpu_baseline': cpu,
        }
        print(json.dumps(line), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
