"""Helper of tests/test_gpu_knobs.py (not a test module): three fused training steps
of a small HSTU model on cuda:0 under whatever GRK_* environment the parent set,
printed as one JSON line {"loss": [...], "lib": path, "host_times": bool}.

The sequence length (T = 151) takes the whole-sequence attention kernels by default
and the chunked ones under GRK_ATTN_CHUNKED; the dnn layers' K = d + 40 GEMMs go to
grk_mgemm by default and to hipBLASLt under GRK_GEMM_BACKEND=hipblaslt."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from tencent_recommendation_2025_amd import _lib as L
    from tencent_recommendation_2025_amd import streams
    from tencent_recommendation_2025_amd import synthetic as S
    from tencent_recommendation_2025_amd.model import BaselineModel, init_reference_
    from tencent_recommendation_2025_amd.optim import FusedAdamW
    from tencent_recommendation_2025_amd.train import Trainer

    dev = torch.device('cuda', 0)
    cfg = S.SyntheticConfig(batch_size=6, maxlen=150, num_items=4000, num_users=500, min_len=20)
    stats, types = S.feature_schema(cfg)
    torch.manual_seed(0)
    m = BaselineModel(cfg.num_users, cfg.num_items, stats, types,
                      S.make_args(hidden_units=128, maxlen=150, num_blocks=2, num_heads=2, block='hstu')).to(dev)
    init_reference_(m, seed=0, live_norms=True)
    tr = Trainer(m, FusedAdamW(m, lr=1e-3), loss='bce')
    g = torch.Generator(device=dev).manual_seed(1)
    losses = [float(tr.step(S.make_batch(cfg, g, dev))) for _ in range(3)]
    torch.cuda.synchronize()
    print(json.dumps({'loss': losses, 'lib': str(L.loaded_path()), 'host_times': streams.HOST_TIMES}))


if __name__ == '__main__':
    main()
