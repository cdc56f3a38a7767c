"""Which model-code lines issue the torch (non-grk) ops of one eager training step?

    python scripts/op_sites.py [--batch 128] > gpurun_out/op_sites.txt

A TorchDispatchMode records every aten op of one eager step (forward, backward
and optimizer) with the innermost frame in this package; ops are grouped by
(op, call site) with their count, so the glue kernels of the step breakdown
can be traced to the lines that issue them.  grk ops are listed too (their
launches are ours; the rest is glue)."""
import argparse
import collections
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PKG = os.path.join(REPO, 'tencent_recommendation_2025_amd')


class Sites(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.count = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        site = '?'
        for fr in reversed(traceback.extract_stack(limit=40)):
            if fr.filename.startswith(PKG):
                site = f'{os.path.basename(fr.filename)}:{fr.lineno} {fr.name}'
                break
        shapes = tuple(tuple(a.shape) for a in args if isinstance(a, torch.Tensor))[:3]
        self.count[(str(func.overloadpacket), site, shapes)] += 1
        return func(*args, **(kwargs or {}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=128)
    ap.add_argument('--jagged', type=int, default=1)
    a = ap.parse_args()
    from tencent_recommendation_2025_amd import synthetic as S
    from tencent_recommendation_2025_amd.model import BaselineModel, init_reference_
    from tencent_recommendation_2025_amd.optim import FusedAdamW
    from tencent_recommendation_2025_amd.train import Trainer
    cfg = S.SyntheticConfig(batch_size=a.batch)
    stats, types = S.feature_schema(cfg)
    torch.manual_seed(0)
    m = BaselineModel(cfg.num_users, cfg.num_items, stats, types, S.make_args()).cuda()
    init_reference_(m, seed=0, live_norms=True)
    tr = Trainer(m, FusedAdamW(m, lr=1e-3), loss='bce', jagged=bool(a.jagged))
    g = torch.Generator(device='cuda').manual_seed(0)
    batches = [S.make_batch(cfg, g, 'cuda') for _ in range(3)]
    for i in range(3):
        tr.eager_step(batches[i % 3], next_batch=batches[(i + 1) % 3])
    torch.cuda.synchronize()
    mode = Sites()
    with mode:
        tr.eager_step(batches[0], next_batch=batches[1])
    torch.cuda.synchronize()
    skip = ('aten.view', 'aten._unsafe_view', 'aten.t', 'aten.transpose', 'aten.permute', 'aten.expand',
            'aten.slice', 'aten.select', 'aten.reshape', 'aten.as_strided', 'aten.detach', 'aten.alias',
            'aten.unsqueeze', 'aten.squeeze', 'aten.split', 'aten.split_with_sizes', 'aten.unbind',
            'aten.empty', 'aten.empty_like', 'aten.empty_strided', 'aten.new_empty', 'aten.sym_size',
            'aten.is_same_size', 'aten._to_copy' if False else '', 'aten.lift_fresh')
    rows = [(k, v) for k, v in mode.count.items() if k[0] not in skip]
    print(f'{sum(v for _, v in rows)} non-view ops in one eager step')
    for (op, site, shapes), v in sorted(rows, key=lambda kv: (kv[0][1], kv[0][0])):
        print(f'{v:4d}  {op:32s} {site:48s} {shapes}')


if __name__ == '__main__':
    main()
