"""Synthetic TencentGR-shaped training batches, generated on the device.

Shape contract: B sequences of T = maxlen + 1 slots, valid
length ~ U{min_len..T}, left-padded; the user token sits at the first valid
slot (token_type 2), items fill the rest (token_type 1); next_token_type = 1
on valid slots; pos = next item; neg ~ U[1, N] (uniform, or Zipf(s) over item
popularity).  Feature schema of the TencentGR data
(model/BaseLine/dataset.py:191-212): 14 item-sparse features with
cardinalities {10, 100, 1k, 10k} cycled, 4 user-sparse (1k), 4 user-array
(1k, lengths U{1..4}), mm feature 81 = N(0, 1) [32].  Like the reference's
``fill_missing_feat``, item features are 0 on the user token and user
features are 0 on item tokens.  Item features are a fixed hash of the item
id, so pos/neg features agree with the seq-side ones for the same item.
The layout is exactly ``MyDataset.collate_tensor_fn``'s.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import torch

from .dataset import ITEM_SPARSE, USER_ARRAY, USER_SPARSE


@dataclass
class SyntheticConfig:
    batch_size: int = 128
    maxlen: int = 200
    num_items: int = 1_000_000
    num_users: int = 1_000_000
    item_sparse_card: tuple = (10, 100, 1000, 10000)
    user_sparse_card: int = 1000
    user_array_card: int = 1000
    array_len: int = 4
    min_len: int = 32
    zipf: float | None = None
    mm_ids: list = field(default_factory=lambda: ['81'])
    timestamps: bool = False   # append int64 [B, T] event times (the HSTU time bias input)
    # config 4: RQ-VAE semantic ids as extra item_sparse features 'sid0'..;
    # sid_table int64 [num_items + 1, levels] (rqvae.semantic_id_table), values 1..sid_codes
    sid_table: object = None
    sid_codes: int = 256


def feature_schema(cfg: SyntheticConfig):
    """(feat_statistics, feat_types) as MyDataset exposes them."""
    stats = {}
    for k, f in enumerate(ITEM_SPARSE):
        stats[f] = cfg.item_sparse_card[k % len(cfg.item_sparse_card)]
    for f in USER_SPARSE:
        stats[f] = cfg.user_sparse_card
    for f in USER_ARRAY:
        stats[f] = cfg.user_array_card
    item_sparse = list(ITEM_SPARSE)
    if cfg.sid_table is not None:
        from .rqvae import semantic_id_schema
        names, sid_stats = semantic_id_schema(cfg.sid_table.shape[1], cfg.sid_codes)
        item_sparse += names
        stats.update(sid_stats)
    types = {'user_sparse': list(USER_SPARSE), 'item_sparse': item_sparse, 'item_array': [],
             'user_array': list(USER_ARRAY), 'item_emb': list(cfg.mm_ids), 'user_continual': [],
             'item_continual': []}
    return stats, types


def _hash_feat(ids, k, card):
    return torch.where(ids > 0, (ids * (2654435761 + 2 * k) + 97 * k) % card + 1, torch.zeros_like(ids))


def _items(cfg, shape, g, dev):
    if cfg.zipf:
        # inverse-CDF Zipf(s) over ranks 1..N, ranks mapped to ids by a fixed permutation-like hash
        u = torch.rand(shape, generator=g, device=dev, dtype=torch.float64)
        s = cfg.zipf
        n = cfg.num_items
        r = ((1 - u) * (n ** (1 - s) - 1) + 1) ** (1 / (1 - s))
        r = r.clamp(1, n).long()
        return (r * 7919) % n + 1
    return torch.randint(1, cfg.num_items + 1, shape, generator=g, device=dev)


def make_batch(cfg: SyntheticConfig, generator: torch.Generator, device='cuda'):
    B, T = cfg.batch_size, cfg.maxlen + 1
    g, dev = generator, device
    lens = torch.randint(cfg.min_len, T + 1, (B, 1), generator=g, device=dev)
    t = torch.arange(T, device=dev).unsqueeze(0)
    start = T - lens
    valid = t >= start
    is_user = t == start
    is_item = valid & ~is_user
    uid = torch.randint(1, cfg.num_users + 1, (B, 1), generator=g, device=dev)
    items = _items(cfg, (B, T + 1), g, dev)
    seq = torch.where(is_user, uid, torch.where(is_item, items[:, :T], torch.zeros_like(items[:, :T])))
    nxt = torch.cat([seq[:, 1:], items[:, T:]], 1)          # next item (last slot: a fresh item)
    pos = torch.where(valid, nxt, torch.zeros_like(nxt))
    neg = torch.where(valid, _items(cfg, (B, T), g, dev), torch.zeros_like(pos))
    token_type = torch.where(is_user, 2, torch.where(is_item, 1, 0)).to(torch.int64)
    next_token_type = valid.to(torch.int64)
    next_action_type = torch.where(valid, torch.randint(0, 2, (B, T), generator=g, device=dev), 0)

    def item_feats(ids, mask):
        out = {}
        for k, f in enumerate(ITEM_SPARSE):
            card = cfg.item_sparse_card[k % len(cfg.item_sparse_card)]
            out[f] = torch.where(mask, _hash_feat(ids, k, card), torch.zeros_like(ids))
        if cfg.sid_table is not None:
            rows = cfg.sid_table[ids]
            for lvl in range(rows.shape[-1]):
                out[f'sid{lvl}'] = torch.where(mask, rows[..., lvl], torch.zeros_like(ids))
        for f in cfg.mm_ids:
            mm = torch.randn(B, T, 32 if f == '81' else 1024, generator=g, device=dev)
            out[f] = mm * mask.unsqueeze(-1)
        return out

    seq_feat = item_feats(seq, is_item)
    uvals = uid.expand(B, T)
    for k, f in enumerate(USER_SPARSE):
        seq_feat[f] = torch.where(is_user, _hash_feat(uvals, 20 + k, cfg.user_sparse_card), 0)
    alen = torch.randint(1, cfg.array_len + 1, (B, 1, 1), generator=g, device=dev)
    slot = torch.arange(cfg.array_len, device=dev).view(1, 1, -1)
    for k, f in enumerate(USER_ARRAY):
        vals = (uvals.unsqueeze(-1) * (40503 + 2 * k) + 131 * slot + 7 * k) % cfg.user_array_card + 1
        seq_feat[f] = torch.where(is_user.unsqueeze(-1) & (slot < alen), vals, 0)
    pos_feat = item_feats(pos, pos > 0)
    neg_feat = item_feats(neg, neg > 0)
    batch = (seq, pos, neg, token_type, next_token_type, next_action_type, seq_feat, pos_feat, neg_feat)
    if cfg.timestamps:
        # unix seconds, log-uniform gaps of 1 s .. ~1 month; 0 on padding slots (the
        # kernels take times relative to each sequence's first valid event)
        gaps = torch.exp(torch.rand(B, T, generator=g, device=dev) * 15.0).to(torch.int64)
        ts = 1_720_000_000 + torch.cumsum(torch.where(valid, gaps, 0), 1)
        batch += (torch.where(valid, ts, 0),)
    return batch


def make_args(hidden_units=512, maxlen=200, num_blocks=4, num_heads=8, dropout_rate=0.0, block='hstu',
              variant='o1', norm_first=False, device='cuda', hstu_time_buckets=0, hstu_fp8=False,
              merge_proj_backward=True, grouped_proj=True):
    from types import SimpleNamespace
    return SimpleNamespace(hidden_units=hidden_units, maxlen=maxlen, num_blocks=num_blocks, num_heads=num_heads,
                           dropout_rate=dropout_rate, block=block, variant=variant, norm_first=norm_first,
                           device=device, mm_emb_id=['81'], hstu_time_buckets=hstu_time_buckets, hstu_fp8=hstu_fp8,
                           merge_proj_backward=merge_proj_backward, grouped_proj=grouped_proj)
