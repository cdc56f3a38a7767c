"""Microbench of grk_embedding_backward (run under rocprofv3 --kernel-trace --stats
for the per-kernel split): D=512 bf16 gradients, C2-sized occurrence counts,
(a) uniform ids over 1M rows (item-table shape), (b) a feature-table mix with
cardinality-10 hot rows (thousands of occurrences each, k_seg_hot), (c) the
projected-feature-row call of the bench step (its headline roofline entry).
GRK_LIB=abtest/libgrk_<variant>.so times a build variant (scripts/build_variant.sh).

    python scripts/microbench/emb_bwd.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
from tencent_recommendation_2025_amd import kernels as K  # noqa: E402


def time_call(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    dev = torch.device('cuda', 0)
    g = torch.Generator(device=dev).manual_seed(0)
    D, N = 512, 25728
    grad = torch.randn(N, 3 * D, device=dev, generator=g).bfloat16()
    # (a) item table: 3 lookups of 25.7k tokens over 1M rows
    idx = torch.randint(1, 1_000_001, (3, N), device=dev, generator=g)
    src = [K.GradSource(idx[f], grad, f * D) for f in range(3)]
    us = time_call(lambda: K.embedding_backward(src, 1_000_001, D, dense=False, sparse=True))
    print(f'uniform 1M rows, {3 * N} occurrences: {us:.1f} us')
    # (b) feature tables: cardinalities 10 / 100 / 1000 stacked in one group
    offs, cards, srcs = 0, (10, 10, 100, 1000, 10000), []
    for f, c in enumerate(cards):
        i = torch.randint(1, c + 1, (N,), device=dev, generator=g)
        srcs.append(K.GradSource(i, grad, (f % 3) * D, row_offset=offs, table_rows=c + 1))
        offs += c + 1
    us = time_call(lambda: K.embedding_backward(srcs, offs, D, dense=False, sparse=True))
    res = K.embedding_backward(srcs, offs, D, dense=False, sparse=True)
    print(f'feature tables {cards}, {len(cards) * N} occurrences ({int(res.count.item())} unique): {us:.1f} us')
    # (c) the headline call: the seq side's projected feature rows P (bench.py's first
    # roofline entry) -- 14,336 jagged rows, 14 item features (cardinalities 10 / 100 /
    # 1k / 10k cycled) as one bag of 14 and 20 user slots (4 sparse + 4 arrays x 4) as a
    # bag of 20 that only the user token of each sequence fills, stacked P rows,
    # GRK_BWD_CHUNKED with a dense fp32 output
    n, B = 14336, 128
    card_i = [(10, 100, 1000, 10000)[f % 4] for f in range(14)]
    card_u = [1000] * 20
    offs, col = [], 1
    for c in card_i + card_u:
        offs.append(col)
        col += c
    rows = col
    gi = torch.randn(n, 2 * D, device=dev, generator=g).bfloat16()
    ii = torch.stack([offs[f] + torch.randint(0, card_i[f], (n,), device=dev, generator=g) for f in range(14)], 1)
    iu = torch.zeros(n, 20, dtype=torch.int64, device=dev)
    users = torch.arange(0, n, n // B, device=dev)[:B]
    iu[users] = torch.stack([offs[14 + f] + torch.randint(0, 1000, (B,), device=dev, generator=g)
                             for f in range(20)], 1)
    srcs = [K.GradSource(ii, gi, 0, bag=14), K.GradSource(iu, gi, D, bag=20)]
    us = time_call(lambda: K.embedding_backward(srcs, rows, D, dense=True, chunked=True))
    print(f'projected P rows ({rows} rows, {34 * n} occurrences, chunk {K.chunked_size()}): {us:.1f} us')


if __name__ == '__main__':
    main()
