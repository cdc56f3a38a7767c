"""CPU oracle for the retrieval step -- TEST INFRASTRUCTURE ONLY (imported by
tests/ and never by the product path).

The reference's inference (model/BaseLine/infer.py:213-225) shells out to an
external faiss HNSW binary (``/workspace/faiss-based-ann/faiss_demo``: not in
the reference repository, so not runnable here) with
``--faiss_metric_type=0`` (faiss METRIC_INNER_PRODUCT) and
``--query_ann_top_k=10`` over ``embedding.fbin`` / ``id.u64bin``
(save_item_emb, model/BaseLine/model.py:402-433) and ``query.fbin``, and reads
``id100.u64bin`` back with ``read_result_ids`` (infer.py:51-65).  HNSW is
approximate; the exact answer it approximates is restated here: for each
query, the k items of largest inner product, score descending, ties by item
row ascending, in float64.  Parity of the GPU kernel is against this exact
answer (the HNSW graph's recall is not a reference behaviour to reproduce).
The file formats are pinned by tests/golden/retrieval.npz, written through
the reference's own ``save_emb`` / ``read_result_ids``.
"""
import struct

import numpy as np


def mips_topk(queries, items, k, item_ids=None):
    """(scores float64 [Q, k], ids int64 [Q, k]); past the item count: -inf / -1."""
    q = np.asarray(queries, dtype=np.float64)
    x = np.asarray(items, dtype=np.float64)
    nq, n = q.shape[0], x.shape[0]
    scores = np.full((nq, k), -np.inf)
    ids = np.full((nq, k), -1, dtype=np.int64)
    if n == 0:
        return scores, ids
    s = q @ x.T
    idx = np.arange(n)
    for i in range(nq):
        order = np.lexsort((idx, -s[i]))[:k]
        scores[i, :len(order)] = s[i, order]
        ids[i, :len(order)] = order if item_ids is None else np.asarray(item_ids, dtype=np.int64)[order]
    return scores, ids


def write_result_ids(ids, path):
    """``uint32 num_queries, uint32 top_k`` then uint64 ids row-major: the
    layout read_result_ids parses (model/BaseLine/infer.py:51-65)."""
    ids = np.asarray(ids)
    with open(path, 'wb') as f:
        f.write(struct.pack('II', ids.shape[0], ids.shape[1]))
        ids.astype(np.int64).view(np.uint64).tofile(f)


def read_result_ids(path):
    """model/BaseLine/infer.py:51-65: header then [num_queries, top_k] uint64."""
    with open(path, 'rb') as f:
        nq, k = struct.unpack('II', f.read(8))
        return np.fromfile(f, dtype=np.uint64, count=nq * k).reshape(nq, k)
