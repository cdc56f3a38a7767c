"""Data-path throughput: sequences/s of assembling
tensorised C2-shaped batches (B = 128, maxlen 200) from a TencentGR-format
directory, one host process:

  reference path -- MyDataset.__getitem__ (seek + json.loads + per-token
                    feature dicts + np.random negatives) + collate_tensor_fn
                    (the reference's collate_fn + feat2tensor, vectorised);
  SeqStore path  -- columnar cache (built once) + array-indexed batch assembly;
                    negatives then drawn on the device (--device: adds
                    DeviceNegatives.attach and the H2D copy, timed with a sync).

    python scripts/bench_datapath.py [--users 2048] [--events 300] [--device cuda]
"""
import argparse
import json
import os
import sys
import tempfile
import time
from types import SimpleNamespace

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
from tencent_recommendation_2025_amd.dataset import MyDataset, write_synthetic_tencentgr  # noqa: E402
from tencent_recommendation_2025_amd.seqstore import DeviceNegatives, SeqStore, to_device  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--users', type=int, default=2048)
    ap.add_argument('--events', type=int, default=300)
    ap.add_argument('--items', type=int, default=100000)
    ap.add_argument('--batch', type=int, default=128)
    ap.add_argument('--maxlen', type=int, default=200)
    ap.add_argument('--ref-batches', type=int, default=4)
    ap.add_argument('--device', default=None)
    a = ap.parse_args()
    torch.set_num_threads(1)
    with tempfile.TemporaryDirectory() as d:
        t0 = time.perf_counter()
        write_synthetic_tencentgr(d, num_users=a.users, num_items=a.items, max_events=a.events, seed=0)
        t_write = time.perf_counter() - t0
        ds = MyDataset(d, SimpleNamespace(maxlen=a.maxlen, mm_emb_id=['81']))
        rng = np.random.default_rng(0)
        batches = [rng.choice(a.users, a.batch, replace=False) for _ in range(max(a.ref_batches, 8))]
        t0 = time.perf_counter()
        for uids in batches[:a.ref_batches]:
            ds.collate_tensor_fn([ds[int(u)] for u in uids])
        ref = a.batch * a.ref_batches / (time.perf_counter() - t0)
        t0 = time.perf_counter()
        st = SeqStore(d, maxlen=a.maxlen)
        t_build = time.perf_counter() - t0
        st.batch(batches[0])
        t0 = time.perf_counter()
        for uids in batches:
            st.batch(uids)
        store = a.batch * len(batches) / (time.perf_counter() - t0)
        res = {'metric': 'data-path seq/s (one host process, tensorised C2 batches)', 'batch': a.batch,
               'maxlen': a.maxlen, 'users': a.users, 'max_events': a.events,
               'reference_getitem_collate_seq_per_s': round(ref, 1), 'seqstore_seq_per_s': round(store, 1),
               'speedup': round(store / ref, 1), 'seqstore_build_s': round(t_build, 2),
               'synthetic_write_s': round(t_write, 2), 'tokens': int(st.off[-1])}
        if a.device:
            dn = DeviceNegatives(st, a.device)
            dn.attach(to_device(st.batch(batches[0]), a.device), batches[0], 0)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i, uids in enumerate(batches):
                dn.attach(to_device(st.batch(uids), a.device), uids, i)
            torch.cuda.synchronize()
            res['seqstore_plus_device_negatives_seq_per_s'] = round(a.batch * len(batches) / (time.perf_counter() - t0), 1)
        print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
