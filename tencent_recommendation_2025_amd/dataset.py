"""DataLoader surface of the reference, kept as the drop-in contract.

Mirrors ``model/BaseLine/dataset.py`` (BaseLineO1's ``dataset.py`` differs only
in file preloading and orjson parsing):

* ``MyDataset(data_dir, args)`` -- ``__getitem__(uid)`` returns the 9-tuple
  ``(seq, pos, neg, token_type, next_token_type, next_action_type,
  seq_feat, pos_feat, neg_feat)`` with the same left padding, negative
  sampling (same ``np.random`` draws) and missing-feature defaults
  (``model/BaseLine/dataset.py:96-169,237-265``);
* ``MyDataset.collate_fn`` -- stacks the six id arrays, keeps the three
  feature columns as lists (``:267-293``);
* ``MyDataset.collate_tensor_fn`` -- the tensorised format the hot path eats
  (SURVEY.md §8(f) #1): features become ``{fid: LongTensor[B,T] |
  LongTensor[B,T,A] | FloatTensor[B,T,E]}`` with exactly ``feat2tensor``'s
  padding (``model/BaseLine/model.py:186-224``);
* ``MyTestDataset``, ``save_emb``, ``load_mm_emb`` (``:296-472``).

``write_synthetic_tencentgr`` writes a TencentGR-format directory
(``seq.jsonl`` + ``seq_offsets.pkl``, ``item_feat_dict.json``,
``indexer.pkl``, ``creative_emb/emb_81_32.pkl``) with the feature schema of
``_init_feat_info`` (``:180-235``) for tests and demos; there is no network to
fetch the real data.
"""
from __future__ import annotations

import json
import pickle
import struct
from pathlib import Path

import numpy as np
import torch

# Feature schema of the TencentGR data (model/BaseLine/dataset.py:191-212).
USER_SPARSE = ['103', '104', '105', '109']
ITEM_SPARSE = ['100', '117', '111', '118', '101', '102', '119', '120', '114', '112', '121', '115', '122', '116']
ITEM_ARRAY: list = []
USER_ARRAY = ['106', '107', '108', '110']
MM_SHAPE = {"81": 32, "82": 1024, "83": 3584, "84": 4096, "85": 3584, "86": 3584}


def save_emb(emb, save_path):
    """``uint32 n, uint32 d`` header then raw rows (model/BaseLine/dataset.py:421-434)."""
    n, d = emb.shape[0], emb.shape[1]
    with open(Path(save_path), 'wb') as f:
        f.write(struct.pack('II', n, d))
        emb.tofile(f)


def load_mm_emb(mm_path, feat_ids):
    """Multimodal embedding dicts (model/BaseLine/dataset.py:437-472).

    Feature 81 is a pickle written by the data producer (trusted local data,
    as in the reference); 82-86 are JSON-lines shards.
    """
    out = {}
    for fid in feat_ids:
        shape = MM_SHAPE[fid]
        d = {}
        if fid == '81':
            with open(Path(mm_path, f'emb_{fid}_{shape}.pkl'), 'rb') as f:
                d = pickle.load(f)
        else:
            for js in Path(mm_path, f'emb_{fid}_{shape}').glob('*.json'):
                with open(js, 'r', encoding='utf-8') as f:
                    for line in f:
                        rec = json.loads(line.strip())
                        e = rec['emb']
                        d[rec['anonymous_cid']] = np.array(e, dtype=np.float32) if isinstance(e, list) else e
        out[fid] = d
    return out


class MyDataset(torch.utils.data.Dataset):
    """Training sequences, one per user (model/BaseLine/dataset.py:10-293)."""

    def __init__(self, data_dir, args):
        super().__init__()
        self.data_dir = Path(data_dir)
        self._load_data_and_offsets()
        self.maxlen = args.maxlen
        self.mm_emb_ids = list(getattr(args, 'mm_emb_id', ['81']))
        # args.timestamps: samples carry the records' event times as a tenth field
        # (int64 [maxlen + 1], 0 on padding) for the HSTU time bias; off = the reference's nine
        self.with_timestamps = bool(getattr(args, 'timestamps', False))
        with open(self.data_dir / 'item_feat_dict.json', 'r') as f:
            self.item_feat_dict = json.load(f)
        self.mm_emb_dict = load_mm_emb(self.data_dir / 'creative_emb', self.mm_emb_ids)
        with open(self.data_dir / 'indexer.pkl', 'rb') as f:
            indexer = pickle.load(f)
        self.itemnum = len(indexer['i'])
        self.usernum = len(indexer['u'])
        self.indexer_i_rev = {v: k for k, v in indexer['i'].items()}
        self.indexer_u_rev = {v: k for k, v in indexer['u'].items()}
        self.indexer = indexer
        self.feature_default_value, self.feature_types, self.feat_statistics = self._init_feat_info()
        self._all_fids = [f for group in self.feature_types.values() for f in group]

    def _load_data_and_offsets(self):
        self.data_file = open(self.data_dir / 'seq.jsonl', 'rb')
        with open(self.data_dir / 'seq_offsets.pkl', 'rb') as f:
            self.seq_offsets = pickle.load(f)

    def _load_user_data(self, uid):
        self.data_file.seek(self.seq_offsets[uid])
        return json.loads(self.data_file.readline())

    def _random_neq(self, l, r, s):
        """Uniform rejection sampler; same RNG draws as dataset.py:79-94."""
        t = np.random.randint(l, r)
        while t in s or str(t) not in self.item_feat_dict:
            t = np.random.randint(l, r)
        return t

    def _init_feat_info(self):
        ftypes = {
            'user_sparse': list(USER_SPARSE), 'item_sparse': list(ITEM_SPARSE),
            'item_array': list(ITEM_ARRAY), 'user_array': list(USER_ARRAY),
            'item_emb': list(self.mm_emb_ids), 'user_continual': [], 'item_continual': [],
        }
        default, stats = {}, {}
        for fid in ftypes['user_sparse'] + ftypes['item_sparse']:
            default[fid] = 0
            stats[fid] = len(self.indexer['f'][fid])
        for fid in ftypes['item_array'] + ftypes['user_array']:
            default[fid] = [0]
            stats[fid] = len(self.indexer['f'][fid])
        for fid in ftypes['item_emb']:
            default[fid] = np.zeros(next(iter(self.mm_emb_dict[fid].values())).shape[0], dtype=np.float32)
        return default, ftypes, stats

    def fill_missing_feat(self, feat, item_id):
        """Defaults for absent features + mm embedding (dataset.py:237-265)."""
        feat = {} if feat is None else feat
        filled = dict(feat)
        for fid in set(self._all_fids) - set(feat.keys()):
            filled[fid] = self.feature_default_value[fid]
        for fid in self.feature_types['item_emb']:
            if item_id != 0:
                cid = self.indexer_i_rev[item_id]
                e = self.mm_emb_dict[fid].get(cid)
                if type(e) == np.ndarray:
                    filled[fid] = e
        return filled

    def __len__(self):
        return len(self.seq_offsets)

    def __getitem__(self, uid):
        records = self._load_user_data(uid)
        ext, ext_ts = [], []
        for u, i, ufeat, ifeat, act, when in records:
            if u and ufeat:
                ext.insert(0, (u, ufeat, 2, act))
                ext_ts.insert(0, when or 0)
            if i and ifeat:
                ext.append((i, ifeat, 1, act))
                ext_ts.append(when or 0)
        times = np.zeros([self.maxlen + 1], np.int64)
        n = self.maxlen + 1
        seq, pos, neg = (np.zeros([n], np.int32) for _ in range(3))
        token_type, next_token_type, next_action_type = (np.zeros([n], np.int32) for _ in range(3))
        seq_feat, pos_feat, neg_feat = (np.empty([n], dtype=object) for _ in range(3))
        nxt = ext[-1]
        idx = self.maxlen
        ts = {r[0] for r in ext if r[2] == 1 and r[0]}
        for rec, when in zip(reversed(ext[:-1]), reversed(ext_ts[:-1])):
            i, feat, type_, _ = rec
            times[idx] = when
            next_i, next_feat, next_type, next_act = nxt
            feat = self.fill_missing_feat(feat, i)
            next_feat = self.fill_missing_feat(next_feat, next_i)
            seq[idx] = i
            token_type[idx] = type_
            next_token_type[idx] = next_type
            if next_act is not None:
                next_action_type[idx] = next_act
            seq_feat[idx] = feat
            if next_type == 1 and next_i != 0:
                pos[idx] = next_i
                pos_feat[idx] = next_feat
                neg_id = self._random_neq(1, self.itemnum + 1, ts)
                neg[idx] = neg_id
                neg_feat[idx] = self.fill_missing_feat(self.item_feat_dict[str(neg_id)], neg_id)
            nxt = rec
            idx -= 1
            if idx == -1:
                break
        dflt = self.feature_default_value
        seq_feat = np.where(seq_feat == None, dflt, seq_feat)  # noqa: E711  (object-array compare, as the reference)
        pos_feat = np.where(pos_feat == None, dflt, pos_feat)  # noqa: E711
        neg_feat = np.where(neg_feat == None, dflt, neg_feat)  # noqa: E711
        out = seq, pos, neg, token_type, next_token_type, next_action_type, seq_feat, pos_feat, neg_feat
        return out + (times,) if self.with_timestamps else out

    @staticmethod
    def collate_fn(batch):
        """Reference collate (dataset.py:267-293); a tenth field (event times) is stacked too."""
        fields = list(zip(*batch))
        seq, pos, neg, tt, ntt, nat, sf, pf, nf = fields[:9]
        t = lambda x: torch.from_numpy(np.array(x))
        return (t(seq), t(pos), t(neg), t(tt), t(ntt), t(nat), list(sf), list(pf), list(nf)) \
            + tuple(t(x) for x in fields[9:])

    def collate_tensor_fn(self, batch):
        """Tensorised collate: the six id tensors + three feature dicts of tensors
        (+ the event times when the dataset carries them)."""
        seq, pos, neg, tt, ntt, nat, sf, pf, nf, *rest = self.collate_fn(batch)
        ft = self.feature_types
        item = ft['item_sparse'] + ft['item_array'] + ft['item_emb']
        user = ft['user_sparse'] + ft['user_array']
        arr = set(ft['item_array'] + ft['user_array'])
        emb = set(ft['item_emb'])
        return (seq, pos, neg, tt, ntt, nat,
                tensorize(sf, item + user, arr, emb), tensorize(pf, item, arr, emb),
                tensorize(nf, item, arr, emb)) + tuple(rest)


def tensorize(feat_list, fids, array_fids=(), emb_fids=()):
    """Vectorised ``feat2tensor`` (model/BaseLine/model.py:186-224) + mm loop (:281-296).

    Array features are right-padded with 0 to the batch's longest array (the
    reference's ``max_array_len``); mm features default to zeros.
    """
    B = len(feat_list)
    T = max(len(s) for s in feat_list)
    out = {}
    for k in fids:
        if k in array_fids:
            vals = [[d[k] for d in s] for s in feat_list]
            A = max(max(len(v) for v in row) for row in vals)
            arr = np.zeros((B, T, A), np.int64)
            for i, row in enumerate(vals):
                for j, v in enumerate(row):
                    arr[i, j, :len(v)] = v[:A]
            out[k] = torch.from_numpy(arr)
        elif k in emb_fids:
            arr = np.zeros((B, T, MM_SHAPE[k]), np.float32)
            for i, s in enumerate(feat_list):
                for j, d in enumerate(s):
                    if k in d:
                        arr[i, j] = d[k]
            out[k] = torch.from_numpy(arr)
        else:
            out[k] = torch.from_numpy(np.array([[d[k] for d in s] for s in feat_list], dtype=np.int64))
    return out


def sample_negatives(seq, pos, token_type, next_token_type, num_items, seed, item_feat=None, max_tries=1000,
                     item_ok=None):
    """Negatives of a tensorised batch drawn on the device (grk_sample_negatives):
    the neg / neg_feat of MyDataset.__getitem__ (model/BaseLine/dataset.py:136-162)
    for every sequence at once, so DataLoader workers need not draw them.

    The exclusion set of sequence b (the reference's ts, dataset.py:136-139) is
    the item tokens of its window plus its positives -- every item of the user
    the batch holds (items older than the maxlen window are not in the batch and
    are not excluded).  item_feat: int32 [num_items + 1, F] item feature ids, row
    0 = the default values (fill_missing_feat); item_ok: bool [num_items + 1], the
    ids that have a feature row (the reference redraws the others,
    dataset.py:92); returns (neg [B, T], neg_feat [B, T, F] or None), int32 on the
    batch's device."""
    from . import kernels as K
    excl = torch.cat([torch.where(token_type == 1, seq, 0), pos], 1)
    return K.sample_negatives(pos, next_token_type, excl, num_items, seed, max_tries=max_tries,
                              item_feat=item_feat, item_ok=item_ok)


class MyTestDataset(MyDataset):
    """Inference sequences (model/BaseLine/dataset.py:296-419)."""

    def _load_data_and_offsets(self):
        self.data_file = open(self.data_dir / 'predict_seq.jsonl', 'rb')
        with open(self.data_dir / 'predict_seq_offsets.pkl', 'rb') as f:
            self.seq_offsets = pickle.load(f)

    @staticmethod
    def _process_cold_start_feat(feat):
        out = {}
        for k, v in feat.items():
            if type(v) == list:
                out[k] = [0 if type(x) == str else x for x in v]
            elif type(v) == str:
                out[k] = 0
            else:
                out[k] = v
        return out

    def __getitem__(self, uid):
        records = self._load_user_data(uid)
        ext = []
        user_id = None
        for u, i, ufeat, ifeat, _, _ in records:
            if u:
                user_id = u if type(u) == str else self.indexer_u_rev[u]
            if u and ufeat:
                if type(u) == str:
                    u = 0
                ext.insert(0, (u, self._process_cold_start_feat(ufeat), 2))
            if i and ifeat:
                if i > self.itemnum:
                    i = 0
                ext.append((i, self._process_cold_start_feat(ifeat), 1))
        n = self.maxlen + 1
        seq = np.zeros([n], np.int32)
        token_type = np.zeros([n], np.int32)
        seq_feat = np.empty([n], dtype=object)
        idx = self.maxlen
        for i, feat, type_ in reversed(ext[:-1]):
            seq[idx] = i
            token_type[idx] = type_
            seq_feat[idx] = self.fill_missing_feat(feat, i)
            idx -= 1
            if idx == -1:
                break
        seq_feat = np.where(seq_feat == None, self.feature_default_value, seq_feat)  # noqa: E711
        return seq, token_type, seq_feat, user_id

    @staticmethod
    def collate_fn(batch):
        seq, tt, sf, uid = zip(*batch)
        return torch.from_numpy(np.array(seq)), torch.from_numpy(np.array(tt)), list(sf), uid


def write_synthetic_tencentgr(data_dir, num_users=64, num_items=500, max_events=60, seed=0,
                              sparse_card=(10, 100, 1000, 10000), user_card=1000, array_len=4,
                              missing_rate=0.05, mm_rate=0.8):
    """Write a small TencentGR-format directory (schema of dataset.py:180-235)."""
    rng = np.random.default_rng(seed)
    d = Path(data_dir)
    (d / 'creative_emb').mkdir(parents=True, exist_ok=True)
    item_card = {f: int(sparse_card[k % len(sparse_card)]) for k, f in enumerate(ITEM_SPARSE)}
    ucard = {f: user_card for f in USER_SPARSE + USER_ARRAY}
    indexer = {
        'i': {f'c{n}': n for n in range(1, num_items + 1)},
        'u': {f'user_{n}': n for n in range(1, num_users + 1)},
        'f': {f: {f'v{v}': v for v in range(1, c + 1)} for f, c in {**item_card, **ucard}.items()},
    }
    item_feat = {}
    for n in range(1, num_items + 1):
        item_feat[str(n)] = {f: int(rng.integers(1, c + 1)) for f, c in item_card.items()
                             if rng.random() >= missing_rate}
    mm = {f'c{n}': rng.standard_normal(32).astype(np.float32)
          for n in range(1, num_items + 1) if rng.random() < mm_rate}
    offsets = []
    with open(d / 'seq.jsonl', 'wb') as f:
        for u in range(1, num_users + 1):
            ufeat = {k: int(rng.integers(1, user_card + 1)) for k in USER_SPARSE if rng.random() >= missing_rate}
            for k in USER_ARRAY:
                if rng.random() >= missing_rate:
                    ufeat[k] = [int(x) for x in rng.integers(1, user_card + 1, int(rng.integers(1, array_len + 1)))]
            recs = [[u, None, ufeat, None, None, 0]]
            for t in range(int(rng.integers(3, max_events + 1))):
                i = int(rng.integers(1, num_items + 1))
                recs.append([None, i, None, item_feat[str(i)], int(rng.integers(0, 2)), t + 1])
            offsets.append(f.tell())
            f.write((json.dumps(recs) + '\n').encode())
    with open(d / 'seq_offsets.pkl', 'wb') as f:
        pickle.dump(offsets, f)
    with open(d / 'item_feat_dict.json', 'w') as f:
        json.dump(item_feat, f)
    with open(d / 'indexer.pkl', 'wb') as f:
        pickle.dump(indexer, f)
    with open(d / 'creative_emb' / 'emb_81_32.pkl', 'wb') as f:
        pickle.dump(mm, f)
    return d
