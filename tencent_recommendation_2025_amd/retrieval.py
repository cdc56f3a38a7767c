"""Retrieval step of inference on the GPU: exact inner-product top-k
(grk_mips_topk) in place of the reference's external faiss HNSW binary.

The reference (model/BaseLine/infer.py:205-225) writes ``query.fbin`` next to
the ``embedding.fbin`` / ``id.u64bin`` of save_item_emb (model/BaseLine/
model.py:402-433), runs ``faiss_demo --dataset_vector_file_path=...
--dataset_id_file_path=... --query_vector_file_path=...
--result_id_file_path=... --query_ann_top_k=10 ... --faiss_metric_type=0``
and reads the result with ``read_result_ids`` (infer.py:51-65).  ``ann_search``
takes the same four paths and top-k and writes the same result file;
``python -m tencent_recommendation_2025_amd.retrieval`` accepts faiss_demo's
command line (the HNSW build/search knobs are accepted and ignored: the
search is exhaustive, so its recall is 1).

File formats (dataset.save_emb, model/BaseLine/dataset.py:421-434):
``uint32 n, uint32 d`` then n x d rows (float32 vectors, uint64 ids); the
result file is ``uint32 num_queries, uint32 top_k`` then uint64 ids.
"""
import argparse
import struct
import sys

import numpy as np
import torch

from . import kernels as K


def read_bin(path, dtype=np.float32):
    """[n, d] array of an .fbin (float32) / .u64bin (uint64) file written by save_emb."""
    with open(path, 'rb') as f:
        n, d = struct.unpack('II', f.read(8))
        return np.fromfile(f, dtype=dtype, count=n * d).reshape(n, d)


def write_result_ids(ids, path):
    """[num_queries, top_k] ids (int64 -1 = no item, stored as its uint64 bits, as faiss)."""
    ids = np.asarray(ids)
    with open(path, 'wb') as f:
        f.write(struct.pack('II', ids.shape[0], ids.shape[1]))
        ids.astype(np.int64).view(np.uint64).tofile(f)


def read_result_ids(path):
    """model/BaseLine/infer.py:51-65: the [num_queries, top_k] uint64 result ids."""
    with open(path, 'rb') as f:
        nq, k = struct.unpack('II', f.read(8))
        return np.fromfile(f, dtype=np.uint64, count=nq * k).reshape(nq, k)


def mips_topk(queries, items, k=10, item_ids=None, query_batch=1 << 16):
    """Exact top-k by inner product on the GPU.

    queries [Q, D], items [N, D]: device tensors, both fp32 or both bf16;
    item_ids: optional [N] int64 / uint64 device tensor (retrieval ids).
    Returns (scores fp32 [Q, k], ids int64 [Q, k]) on the device, score
    descending, ties by item row ascending; -inf / -1 past N items.  Queries
    run in batches of ``query_batch`` (bounds the candidate workspace)."""
    if queries.shape[0] <= query_batch:
        return K.mips_topk(queries, items, k, item_ids)
    outs = [K.mips_topk(queries[i:i + query_batch], items, k, item_ids)
            for i in range(0, queries.shape[0], query_batch)]
    return torch.cat([o[0] for o in outs]), torch.cat([o[1] for o in outs])


def ann_search(dataset_vector_file_path, dataset_id_file_path, query_vector_file_path, result_id_file_path,
               query_ann_top_k=10, device='cuda', dtype=torch.float32):
    """The faiss_demo step of infer.py:213-225 on the GPU: reads the three
    inputs, writes ``result_id_file_path``; returns the uint64 ids [Q, k]."""
    dev = torch.device(device)
    items = torch.from_numpy(read_bin(dataset_vector_file_path)).to(dev, dtype)
    ids = torch.from_numpy(read_bin(dataset_id_file_path, np.uint64).reshape(-1).view(np.int64)).to(dev)
    queries = torch.from_numpy(read_bin(query_vector_file_path)).to(dev, dtype)
    if ids.numel() != items.shape[0]:
        raise ValueError(f'{dataset_id_file_path}: {ids.numel()} ids for {items.shape[0]} vectors')
    _, top = mips_topk(queries, items, query_ann_top_k, ids)
    out = top.cpu().numpy()
    write_result_ids(out, result_id_file_path)
    return out.view(np.uint64)


def main(argv=None):
    ap = argparse.ArgumentParser(description='exact inner-product top-k (faiss_demo command line)')
    ap.add_argument('--dataset_vector_file_path', required=True)
    ap.add_argument('--dataset_id_file_path', required=True)
    ap.add_argument('--query_vector_file_path', required=True)
    ap.add_argument('--result_id_file_path', required=True)
    ap.add_argument('--query_ann_top_k', type=int, default=10)
    ap.add_argument('--faiss_metric_type', type=int, default=0)
    for knob in ('--faiss_M', '--faiss_ef_construction', '--query_ef_search'):
        ap.add_argument(knob, type=int, default=None, help='HNSW knob: accepted, unused (exhaustive search)')
    ap.add_argument('--dtype', default='float32', choices=['float32', 'bfloat16'])
    a = ap.parse_args(argv)
    if a.faiss_metric_type != 0:
        ap.error('only --faiss_metric_type=0 (inner product) is supported, as the reference uses')
    ann_search(a.dataset_vector_file_path, a.dataset_id_file_path, a.query_vector_file_path, a.result_id_file_path,
               a.query_ann_top_k, dtype=getattr(torch, a.dtype))
    return 0


if __name__ == '__main__':
    sys.exit(main())
