"""Dump the captured training step (HIP graph) as DOT and list its non-kernel nodes."""
import re
import sys
from collections import Counter

import torch

sys.path.insert(0, '/root/repo')
from tencent_recommendation_2025_amd import synthetic as S  # noqa: E402
from tencent_recommendation_2025_amd.model import BaselineModel  # noqa: E402
from tencent_recommendation_2025_amd.optim import FusedAdamW  # noqa: E402
from tencent_recommendation_2025_amd.train import Trainer  # noqa: E402

DEV = 'cuda'
cfg = S.SyntheticConfig(batch_size=8, maxlen=30, num_items=5000, num_users=700, min_len=4)
stats, types = S.feature_schema(cfg)
block = sys.argv[1] if len(sys.argv) > 1 else 'hstu'
out = sys.argv[2] if len(sys.argv) > 2 else 'gpurun_out/step_graph.dot'
args = S.make_args(hidden_units=64, maxlen=30, num_blocks=2, num_heads=2, dropout_rate=0.1, block=block)
m = BaselineModel(cfg.num_users, cfg.num_items, stats, types, args).to(DEV)
tr = Trainer(m, FusedAdamW(m, lr=1e-3, defer_period=4), loss='bce', graph=True, graph_warmup=2, graph_dump=out)
g = torch.Generator(device=DEV).manual_seed(0)
for i in range(4):
    tr.step(S.make_batch(cfg, g, DEV))
torch.cuda.synchronize()
text = open(out).read()
kinds = Counter(re.findall(r'\b(MEMSET|MEMCPY|KERNEL|EVENT_RECORD|WAIT_EVENT|HOST|EMPTY)\w*', text, re.I))
print('node kinds:', dict(kinds))
for line in text.splitlines():
    if re.search('memset|memcpy', line, re.I):
        print(line[:300])
