"""CPU oracle for the device negative sampler -- TEST INFRASTRUCTURE ONLY
(imported by tests/ and never by the product path).

Reference: MyDataset.__getitem__ (model/BaseLine/dataset.py:136-162) draws, for
every position whose next token is an item with a non-zero positive, a
negative ``_random_neq(1, itemnum + 1, ts)`` (dataset.py:79-95): uniform over
[1, itemnum], redrawn while it is in ts (the user's item ids, :136-139) or has
no feature row.  Other positions stay 0.

The device kernel (grk_sample_negatives) keeps those semantics with a
counter-based generator instead of np.random's stream; this file restates the
kernel's arithmetic exactly (splitmix64 and the 64x64-bit high-word range
map), so the GPU result is checked bit-exactly against it.  The reference's
own random stream cannot be matched -- the draws are pinned by the
distributional properties the reference guarantees (range, exclusion,
positions) in tests/test_sampler.py: parity of the *values* is unpinned.
"""
import numpy as np

M64 = (1 << 64) - 1


def splitmix64(x):
    x = (x + 0x9E3779B97F4A7C15) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return x ^ (x >> 31)


def draw(seed, b, t, a, num_items):
    """Attempt a of position (b, t): an id in [1, num_items]."""
    x = splitmix64((seed ^ splitmix64(((b << 32) ^ (t << 16) ^ a) & M64)) & M64)
    return ((x * num_items) >> 64) + 1


def sample_negatives(pos, next_token_type, excl, num_items, seed, max_tries=1000, item_feat=None, item_ok=None):
    """(neg int32 [B, T], neg_feat or None, all_excluded flag) -- grk_sample_negatives' contract.

    item_ok (bool [num_items + 1], optional): ids with a feature row; a draw
    without one is redrawn, as ``str(t) not in self.item_feat_dict`` in
    _random_neq (model/BaseLine/dataset.py:92)."""
    pos = np.asarray(pos)
    ntt = np.asarray(next_token_type)
    B, T = pos.shape
    neg = np.zeros((B, T), np.int32)
    flag = False
    for b in range(B):
        ts = set(int(v) for v in np.asarray(excl)[b] if v != 0)
        for t in range(T):
            if ntt[b, t] != 1 or pos[b, t] == 0:
                continue
            v, hit = 0, True
            for a in range(max_tries):
                v = draw(seed, b, t, a, num_items)
                hit = v in ts or (item_ok is not None and not item_ok[v])
                if not hit:
                    break
            flag |= hit
            neg[b, t] = v
    feat = None if item_feat is None else np.asarray(item_feat)[neg]
    return neg, feat, flag
