"""Which Python call sites launch the torch (non-grk) kernels of one eager step?

    python scripts/glue_ops.py [--batch 128] [--loss bce] > gpurun_out/glue_ops.txt

torch.profiler with CPU + device activities and Python stacks over two eager
steps of the bench model; prints the aten ops by self device time grouped by
their top model-code frames, so each glue kernel of
profiles/*_step_breakdown.txt can be traced to the line that issues it.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=128)
    ap.add_argument('--loss', default='bce')
    ap.add_argument('--rows', type=int, default=60)
    a = ap.parse_args()
    from torch.profiler import ProfilerActivity, profile
    from tencent_recommendation_2025_amd import synthetic as S
    from tencent_recommendation_2025_amd.model import BaselineModel, init_reference_
    from tencent_recommendation_2025_amd.optim import FusedAdamW
    from tencent_recommendation_2025_amd.train import Trainer
    cfg = S.SyntheticConfig(batch_size=a.batch)
    stats, types = S.feature_schema(cfg)
    torch.manual_seed(0)
    m = BaselineModel(cfg.num_users, cfg.num_items, stats, types, S.make_args()).cuda()
    init_reference_(m, seed=0, live_norms=True)
    opt = FusedAdamW(m, lr=1e-3)
    tr = Trainer(m, opt, loss=a.loss)
    g = torch.Generator(device='cuda').manual_seed(0)
    batches = [S.make_batch(cfg, g, 'cuda') for _ in range(3)]
    for i in range(3):
        tr.eager_step(batches[i % 3], next_batch=batches[(i + 1) % 3])
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True,
                 record_shapes=True) as prof:
        for i in range(2):
            tr.eager_step(batches[i % 3], next_batch=batches[(i + 1) % 3])
        torch.cuda.synchronize()
    ka = prof.key_averages(group_by_input_shape=True)
    rows = [e for e in ka if e.self_device_time_total > 0 and e.key.startswith('aten::')]
    rows.sort(key=lambda e: -e.self_device_time_total)
    tot = sum(e.self_device_time_total for e in ka if e.self_device_time_total > 0)
    print(f'device time over 2 steps: {tot / 1e3:.3f} ms (all kernels incl. grk)')
    for e in rows[:a.rows]:
        print(f'{e.self_device_time_total / 2e3:8.3f} ms/step {e.count / 2:5.1f}x  {e.key}  {e.input_shapes}')
    print('\n# by call site (model-code frames)')
    ks = prof.key_averages(group_by_stack_n=8)
    rows = [e for e in ks if e.self_device_time_total > 0 and e.key.startswith('aten::')]
    rows.sort(key=lambda e: -e.self_device_time_total)
    for e in rows[:a.rows]:
        fr = [f for f in e.stack if 'tencent_recommendation_2025_amd' in f or 'bench' in f][:3]
        print(f'{e.self_device_time_total / 2e3:8.3f} ms/step {e.count / 2:5.1f}x  {e.key}  | ' + ' <- '.join(
            f.split('/')[-1] for f in fr))


if __name__ == '__main__':
    main()
