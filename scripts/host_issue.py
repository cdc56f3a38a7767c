"""Host issue time vs device time of the bench training step.

    python scripts/host_issue.py [--sharded 1] [--steps 20]

Times the host side of Trainer.step (no synchronize inside the loop) and the
wall time with a final synchronize: host issue >= wall means the step is
host-bound (the GPU waits on Python), and the per-phase host times (prepare /
replay / optimizer step for the sharded path) say where.
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--sharded', type=int, default=0)
    ap.add_argument('--steps', type=int, default=20)
    a = ap.parse_args()
    if a.sharded:
        import torch.distributed as dist
        for k, v in (('RANK', '0'), ('WORLD_SIZE', '1'), ('MASTER_ADDR', '127.0.0.1'), ('MASTER_PORT', '29536')):
            os.environ.setdefault(k, v)
        dist.init_process_group('nccl', device_id=torch.device('cuda', 0))
    from tencent_recommendation_2025_amd import synthetic as S
    from tencent_recommendation_2025_amd.model import BaselineModel, init_reference_
    from tencent_recommendation_2025_amd.optim import FusedAdamW
    from tencent_recommendation_2025_amd.train import Trainer
    cfg = S.SyntheticConfig(batch_size=128)
    stats, types = S.feature_schema(cfg)
    torch.manual_seed(0)
    m = BaselineModel(cfg.num_users, cfg.num_items, stats, types, S.make_args()).cuda()
    init_reference_(m, seed=0, live_norms=True)
    if a.sharded:
        from tencent_recommendation_2025_amd.sharding import ShardedFusedAdamW
        opt = ShardedFusedAdamW(m, lr=1e-3, weight_decay=0.01)
    else:
        opt = FusedAdamW(m, lr=1e-3)
    tr = Trainer(m, opt, loss='bce', graph=True)
    g = torch.Generator(device='cuda').manual_seed(0)
    batches = [S.make_batch(cfg, g, 'cuda') for _ in range(4)]
    phases = {}
    if a.sharded:  # per-phase host time
        for name in ('prepare', 'prefetch', 'restore_captured', 'step'):
            fn = getattr(opt, name)

            def wrap(*x, fn=fn, name=name, **kw):
                t = time.perf_counter()
                r = fn(*x, **kw)
                phases[name] = phases.get(name, 0.0) + time.perf_counter() - t
                return r
            setattr(opt, name, wrap)
    if a.sharded:  # host time inside prepare(): event waits, exchanges, segment flushes
        from tencent_recommendation_2025_amd import sharding as SH

        def timed(obj, name, label):
            fn = getattr(obj, name)

            def w(*x, **kw):
                t = time.perf_counter()
                r = fn(*x, **kw)
                phases[label] = phases.get(label, 0.0) + time.perf_counter() - t
                return r
            setattr(obj, name, w)
        timed(torch.cuda.Event, 'synchronize', '  event.synchronize')
        timed(SH.ShardExchange, 'fetch', '  exchange.fetch')
        timed(SH.ShardExchange, 'route', '  exchange.route')
        timed(opt, 'maybe_segment', '  maybe_segment')
    for i in range(8):
        tr.step(batches[i % 4], batches[(i + 1) % 4])
    torch.cuda.synchronize()
    phases.clear()
    if a.sharded:
        opt.trace = []
    t0 = time.perf_counter()
    for i in range(a.steps):
        tr.step(batches[i % 4], batches[(i + 1) % 4])
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    n = a.steps
    print(f'host issue {1e3 * (t1 - t0) / n:.3f} ms/step, wall {1e3 * (t2 - t0) / n:.3f} ms/step')
    for k, v in phases.items():
        print(f'  {k:18s} {1e3 * v / n:.3f} ms/step (host)')
    if a.sharded:
        done = sum(1 for k, v in opt.trace if v)
        print(f'route already complete at prepare: {done} of {len(opt.trace)} steps')
        torch.distributed.destroy_process_group()


if __name__ == '__main__':
    main()
