"""Tensorised TencentGR data path.

The reference builds every training sample in a DataLoader worker:
``MyDataset.__getitem__`` seeks, ``json.loads`` the user's line, fills a
feature dict per token and draws one negative per position with np.random
(``model/BaseLine/dataset.py:96-169``); ``collate_fn`` stacks the ids and
the model's ``feat2tensor`` turns the dict lists into tensors on the host
(``model/BaseLine/model.py:186-224``).  Here:

* ``SeqStore`` parses ``seq.jsonl`` ONCE into columnar token arrays (ids,
  types, actions, the feature ids of every token after ``fill_missing_feat``,
  a row index into the multimodal-embedding table) and caches them as ``.npy``
  files; ``SeqStore.batch(uids)`` then assembles a whole batch with array
  indexing -- the same ``(seq, pos, neg, token_type, next_token_type,
  next_action_type, seq_feat, pos_feat, neg_feat)`` as
  ``MyDataset.collate_tensor_fn`` (bit-identical; the negatives excepted);
* ``DeviceNegatives`` draws the negatives of a device-resident batch with
  ``grk_sample_negatives`` (uniform over the items, redrawn while in the
  user's history or without a feature row, as ``_random_neq``) and gathers
  their feature ids and mm embeddings on the device.

The negative ids come from a counter-based generator, not np.random's stream:
their values are parity-unpinned (the contract they satisfy is tested).
"""
from __future__ import annotations

import ctypes as C
import json
import pickle
from pathlib import Path

import numpy as np
import torch

from .dataset import ITEM_ARRAY, ITEM_SPARSE, MM_SHAPE, USER_ARRAY, USER_SPARSE, load_mm_emb

CACHE_VERSION = 3   # 2: per-token event times (ts); 3: per-user distinct item histories


class SeqStore:
    """Columnar token store of a TencentGR data directory.

    Tokens of user line ``u`` are ``[off[u], off[u + 1])``, in the order
    ``MyDataset.__getitem__`` lays out its ``ext`` list (user tokens first,
    most recent user record first, then the item tokens in record order).
    Per token: ``tid`` (item or user id), ``ttype`` (1 item, 2 user), ``act``
    (action type, 0 when absent), ``ts`` (the record's timestamp, int64, 0 when
    absent -- the HSTU time-bias input; the reference drops it,
    model/BaseLine/dataset.py:117), ``sparse`` int32 [F_sparse] (user then item
    sparse fids, default 0), ``arr`` int32 [F_array, A_cap] + ``arr_len``
    (default ``[0]``), ``mm`` int32 per mm fid (row of that fid's embedding
    table, 0 = the zero row)."""

    def __init__(self, data_dir, maxlen, mm_emb_ids=('81',), cache_dir=None, rebuild=False):
        self.data_dir = Path(data_dir)
        self.maxlen = int(maxlen)
        self.mm_ids = list(mm_emb_ids)
        self.sparse_fids = USER_SPARSE + ITEM_SPARSE
        self.array_fids = USER_ARRAY + ITEM_ARRAY
        self.item_fids = ITEM_SPARSE + ITEM_ARRAY + self.mm_ids    # MyDataset.collate_tensor_fn's order
        self.user_fids = USER_SPARSE + USER_ARRAY
        self.cache_dir = Path(cache_dir) if cache_dir else self.data_dir / 'grk_seqstore'
        with open(self.data_dir / 'indexer.pkl', 'rb') as f:
            indexer = pickle.load(f)
        self.itemnum = len(indexer['i'])
        self.usernum = len(indexer['u'])
        meta = self.cache_dir / 'meta.json'
        if rebuild or not meta.exists() or json.loads(meta.read_text()).get('version') != CACHE_VERSION \
                or json.loads(meta.read_text()).get('mm_ids') != self.mm_ids:
            self._build(indexer)
        self._load()

    # ------------------------------------------------------------ build ----
    def _build(self, indexer):
        rev_i = {v: k for k, v in indexer['i'].items()}
        mm = load_mm_emb(self.data_dir / 'creative_emb', self.mm_ids)
        mm_rows = {}
        mm_tables = {}
        for fid in self.mm_ids:
            keys = [k for k, e in mm[fid].items() if type(e) == np.ndarray]  # noqa: E721 (reference test)
            mm_rows[fid] = {k: n + 1 for n, k in enumerate(keys)}
            tab = np.zeros((len(keys) + 1, MM_SHAPE[fid]), np.float32)
            for k, n in mm_rows[fid].items():
                tab[n] = mm[fid][k]
            mm_tables[fid] = tab
        with open(self.data_dir / 'seq_offsets.pkl', 'rb') as f:
            offsets = pickle.load(f)
        sp_col = {f: c for c, f in enumerate(self.sparse_fids)}
        ar_col = {f: c for c, f in enumerate(self.array_fids)}
        tid, ttype, act, tss, sparse, arrs, mmi, off = [], [], [], [], [], [], [], [0]
        a_cap = 1

        def mm_row(token_id, fid):
            # fill_missing_feat looks the token id up as an ITEM id for every token
            # (user tokens included, model/BaseLine/dataset.py:254-262)
            if token_id == 0 or token_id not in rev_i:
                return 0
            return mm_rows[fid].get(rev_i[token_id], 0)

        with open(self.data_dir / 'seq.jsonl', 'rb') as f:
            for o in offsets:
                f.seek(o)
                ext = []
                for u, i, ufeat, ifeat, a, ts in json.loads(f.readline()):
                    if u and ufeat:
                        ext.insert(0, (u, ufeat, 2, a, ts))
                    if i and ifeat:
                        ext.append((i, ifeat, 1, a, ts))
                for t_id, feat, t_type, a, ts in ext:
                    tid.append(t_id)
                    ttype.append(t_type)
                    act.append(0 if a is None else a)
                    tss.append(0 if ts is None else int(ts))
                    row = np.zeros(len(self.sparse_fids), np.int32)
                    ar = [[0] for _ in self.array_fids]
                    for k, v in feat.items():
                        if k in sp_col:
                            row[sp_col[k]] = v
                        elif k in ar_col:
                            ar[ar_col[k]] = list(v)
                    sparse.append(row)
                    arrs.append(ar)
                    a_cap = max(a_cap, max((len(x) for x in ar), default=1))
                    mmi.append([mm_row(t_id, fid) for fid in self.mm_ids])
                off.append(len(tid))
        n = len(tid)
        arr = np.zeros((n, len(self.array_fids), a_cap), np.int32)
        arr_len = np.zeros((n, len(self.array_fids)), np.int32)
        for t, ar in enumerate(arrs):
            for c, v in enumerate(ar):
                arr[t, c, :len(v)] = v
                arr_len[t, c] = len(v)
        # item feature table for the negatives: fill_missing_feat(item_feat_dict[str(i)], i)
        with open(self.data_dir / 'item_feat_dict.json', 'r') as f:
            item_feat = json.load(f)
        isp = np.zeros((self.itemnum + 1, len(ITEM_SPARSE)), np.int32)
        iok = np.zeros(self.itemnum + 1, np.uint8)
        imm = np.zeros((self.itemnum + 1, len(self.mm_ids)), np.int32)
        icol = {f: c for c, f in enumerate(ITEM_SPARSE)}
        for i in range(1, self.itemnum + 1):
            d = item_feat.get(str(i))
            if d is None:
                continue
            iok[i] = 1
            for k, v in d.items():
                if k in icol:
                    isp[i, icol[k]] = v
            imm[i] = [mm_row(i, fid) for fid in self.mm_ids]
        # per-user distinct item ids, ascending (the exclusion sets of the negatives,
        # DeviceNegatives / history_items), CSR over the users
        tid_a, tt_a, off_a = np.asarray(tid, np.int32), np.asarray(ttype, np.int8), np.asarray(off, np.int64)
        hist, hist_off = [], [0]
        for u in range(len(off_a) - 1):
            s_, e_ = off_a[u], off_a[u + 1]
            h = np.unique(tid_a[s_:e_][tt_a[s_:e_] == 1])
            h = h[h != 0]
            hist.append(h)
            hist_off.append(hist_off[-1] + len(h))
        hist_items = np.concatenate(hist).astype(np.int32) if hist else np.zeros(0, np.int32)
        self.cache_dir.mkdir(parents=True, exist_ok=True)
        arrays = dict(hist_items=hist_items, hist_off=np.asarray(hist_off, np.int64),off=np.asarray(off, np.int64), tid=np.asarray(tid, np.int32), ttype=np.asarray(ttype, np.int8),
                      act=np.asarray(act, np.int32), ts=np.asarray(tss, np.int64), sparse=np.asarray(sparse, np.int32).reshape(n, -1), arr=arr,
                      arr_len=arr_len, mm=np.asarray(mmi, np.int32).reshape(n, -1), item_sparse=isp, item_ok=iok,
                      item_mm=imm)
        for fid in self.mm_ids:
            arrays[f'mm_table_{fid}'] = mm_tables[fid]
        for k, v in arrays.items():
            np.save(self.cache_dir / f'{k}.npy', v)
        (self.cache_dir / 'meta.json').write_text(json.dumps({'version': CACHE_VERSION, 'mm_ids': self.mm_ids,
                                                             'tokens': n, 'users': len(offsets)}))

    def _load(self):
        ld = lambda k: np.load(self.cache_dir / f'{k}.npy', mmap_mode='r')
        self.off, self.tid, self.ttype, self.act, self.ts = ld('off'), ld('tid'), ld('ttype'), ld('act'), ld('ts')
        self.sparse, self.arr, self.arr_len, self.mm = ld('sparse'), ld('arr'), ld('arr_len'), ld('mm')
        self.item_sparse, self.item_ok, self.item_mm = ld('item_sparse'), ld('item_ok'), ld('item_mm')
        self.hist_items, self.hist_off = ld('hist_items'), ld('hist_off')
        self.mm_tables = {fid: np.load(self.cache_dir / f'mm_table_{fid}.npy') for fid in self.mm_ids}

    _MAPPED = ('off', 'tid', 'ttype', 'act', 'ts', 'sparse', 'arr', 'arr_len', 'mm', 'item_sparse', 'item_ok',
               'item_mm', 'mm_tables', 'hist_items', 'hist_off')

    def __getstate__(self):
        """Pickled (DataLoader workers under spawn / forkserver) as the cache's path
        only: np.memmap pickles its whole contents, which would copy the token
        store into every worker; the worker maps the same files again."""
        return {k: v for k, v in self.__dict__.items() if k not in self._MAPPED}

    def __setstate__(self, state):
        self.__dict__.update(state)
        self._load()

    def __len__(self):
        return len(self.off) - 1

    # ------------------------------------------------------------ batch ----
    def batch(self, uids, timestamps=False):
        """The tensorised batch of users ``uids`` (= MyDataset.collate_tensor_fn of
        ``[ds[u] for u in uids]``), with ``neg`` all zero and ``neg_feat`` None:
        the negatives are drawn on the device (DeviceNegatives).  timestamps=True
        appends int64 [B, T] event times (0 on padding) as a tenth field -- the
        input of the HSTU time bias (Trainer / model ``timestamps``)."""
        uids = np.asarray(uids, np.int64)
        B, T = len(uids), self.maxlen + 1
        start, end = self.off[uids], self.off[uids + 1]
        n = end - start                                   # ext length (>= 1, as the reference needs)
        m = np.minimum(n - 1, T)                          # filled positions: the last m of T
        p = np.arange(T)[None, :]
        valid = p >= (T - m)[:, None]
        g = np.where(valid, (start + n - 1 - T)[:, None] + p, 0)  # token at position p; its next is g + 1
        gn = np.where(valid, g + 1, 0)
        seq = np.where(valid, self.tid[g], 0).astype(np.int32)
        tt = np.where(valid, self.ttype[g], 0).astype(np.int32)
        ntt = np.where(valid, self.ttype[gn], 0).astype(np.int32)
        nat = np.where(valid, self.act[gn], 0).astype(np.int32)
        nid = np.where(valid, self.tid[gn], 0)
        has_pos = valid & (ntt == 1) & (nid != 0)
        pos = np.where(has_pos, nid, 0).astype(np.int32)
        seq_feat = self._features(g, valid, self.item_fids + self.user_fids)
        pos_feat = self._features(gn, has_pos, self.item_fids)
        t = torch.from_numpy
        out = (t(seq), t(pos), torch.zeros(B, T, dtype=torch.int32), t(tt), t(ntt), t(nat), seq_feat, pos_feat, None)
        if timestamps:
            out += (t(np.where(valid, self.ts[g], 0).astype(np.int64)),)
        return out

    def _features(self, g, sel, fids):
        """{fid: tensor} of the tokens g where sel, the defaults elsewhere (tensorize's layout).
        One gather per feature kind (sparse block, array block, mm rows), then per-fid columns."""
        # grk_store_features (host code in libgrk, no GPU): one pass per output
        # column, straight into the int64 / fp32 tensors feat2tensor would build
        from . import _lib as L
        B, T = g.shape
        N = B * T
        sp_col = {f: c for c, f in enumerate(self.sparse_fids)}
        ar_col = {f: c for c, f in enumerate(self.array_fids)}
        tok = np.ascontiguousarray(g.reshape(-1), dtype=np.int64)
        sl = np.ascontiguousarray(sel.reshape(-1), dtype=np.uint8)
        view = self._view()
        widths = np.ones(max(1, len(self.array_fids)), np.int32)
        if any(k in ar_col for k in fids):
            L.check(L.lib().grk_store_array_widths(C.byref(view), tok.ctypes.data, sl.ctypes.data, N,
                                                   widths.ctypes.data), 'grk_store_array_widths')
        out, cols = {}, []
        for k in fids:
            if k in ar_col:
                c, A = ar_col[k], int(widths[ar_col[k]])       # the batch's longest array
                t = torch.empty((B, T, A), dtype=torch.int64)
                cols.append(L.GrkStoreCol(L.STORE_ARRAY, c, A, 0, 0, None, t.data_ptr()))
            elif k in self.mm_ids:
                tab = self.mm_tables[k]
                if tab.dtype != np.float32 or not tab.flags['C_CONTIGUOUS']:
                    raise L.GrkError(f'mm table {k} must be C-contiguous float32')
                t = torch.empty((B, T, tab.shape[1]), dtype=torch.float32)
                cols.append(L.GrkStoreCol(L.STORE_MM, self.mm_ids.index(k), tab.shape[1], 0, tab.shape[0],
                                          tab.ctypes.data, t.data_ptr()))
            else:
                t = torch.empty((B, T), dtype=torch.int64)
                cols.append(L.GrkStoreCol(L.STORE_SPARSE, sp_col[k], 1, 0, 0, None, t.data_ptr()))
            out[k] = t
        arr = (L.GrkStoreCol * max(1, len(cols)))(*cols)
        L.check(L.lib().grk_store_features(C.byref(view), tok.ctypes.data, sl.ctypes.data, N, arr, len(cols)),
                'grk_store_features')
        return out

    def _view(self):
        """grk_store_view over the memory-mapped token blocks.  Built per call, never
        cached on the store: a cached struct's raw pointers would travel with a
        pickled store into a spawned DataLoader worker and point into the parent."""
        from . import _lib as L
        for a in (self.sparse, self.arr, self.arr_len, self.mm):
            if not a.flags['C_CONTIGUOUS'] or a.dtype != np.int32:
                raise L.GrkError('SeqStore blocks must be C-contiguous int32')
        return L.GrkStoreView(self.sparse.ctypes.data, self.arr.ctypes.data, self.arr_len.ctypes.data,
                              self.mm.ctypes.data, len(self.tid), self.sparse.shape[1], self.arr.shape[1],
                              self.arr.shape[2], self.mm.shape[1])

    def history_items(self, uids):
        """int32 [B, L]: each user's distinct item ids over the whole history,
        ascending, 0-padded (L = the largest distinct count in the batch) --
        _random_neq's exclusion set ts (model/BaseLine/dataset.py:136-139).  No
        truncation: grk_sample_negatives takes exclusion lists of any length.
        One gather from the per-user lists the cache holds (no per-user work)."""
        uids = np.asarray(uids, np.int64)
        start, n = self.hist_off[uids], self.hist_off[uids + 1] - self.hist_off[uids]
        L = max(1, int(n.max()) if len(n) else 1)
        col = np.arange(L)[None, :]
        keep = col < n[:, None]
        src = np.where(keep, start[:, None] + col, 0)
        out = np.where(keep, self.hist_items[src] if len(self.hist_items) else 0, 0).astype(np.int32)
        return torch.from_numpy(np.ascontiguousarray(out))


class DeviceNegatives:
    """Negatives of device-resident SeqStore batches: ``grk_sample_negatives``
    with the users' whole-history exclusion sets and the ids without a feature
    row redrawn (``_random_neq``), then the negatives' feature ids and mm
    embeddings gathered on the device (``fill_missing_feat(item_feat_dict[neg])``)."""

    def __init__(self, store: SeqStore, device):
        self.store = store
        self.device = torch.device(device)
        self.item_sparse = torch.from_numpy(np.ascontiguousarray(store.item_sparse)).to(self.device)
        self.item_ok = torch.from_numpy(np.ascontiguousarray(store.item_ok)).to(self.device)
        self.item_mm = torch.from_numpy(np.ascontiguousarray(store.item_mm)).to(self.device).long()
        self.mm_tables = {k: torch.from_numpy(v).to(self.device) for k, v in store.mm_tables.items()}

    def attach(self, batch, uids, seed):
        """The batch (on the device) with neg and neg_feat filled."""
        from . import kernels as K
        seq, pos, _neg, tt, ntt, nat, sf, pf, _nf = batch[:9]
        # the whole history holds every positive of the window (pos are the users' own next items)
        excl = self.store.history_items(uids).to(self.device)
        neg, nfeat = K.sample_negatives(pos, ntt, excl, self.store.itemnum, seed, item_feat=self.item_sparse,
                                        item_ok=self.item_ok)
        neg_feat = {}
        for k in self.store.item_fids:
            if k in ITEM_SPARSE:
                neg_feat[k] = nfeat[..., ITEM_SPARSE.index(k)].long()
            elif k in self.mm_tables:
                neg_feat[k] = self.mm_tables[k][self.item_mm[neg.long(), self.store.mm_ids.index(k)]]
        return (seq, pos, neg, tt, ntt, nat, sf, pf, neg_feat) + tuple(batch[9:])


def to_device(batch, device):
    """Every tensor of a (SeqStore / collate_tensor_fn) batch on `device` (non-blocking from pinned memory)."""
    dev = torch.device(device)
    mv = lambda x: x.to(dev, non_blocking=True) if torch.is_tensor(x) else x
    return tuple({k: mv(v) for k, v in x.items()} if isinstance(x, dict) else mv(x) for x in batch)


class StoreBatches(torch.utils.data.Dataset):
    """Whole shuffled batches of a SeqStore, for a ``DataLoader(..., batch_size=None,
    num_workers=k, pin_memory=True)``: workers share the memory-mapped cache, and
    each yields ``(uids, batch)`` (the reference shuffles users every epoch,
    model/BaseLine/main.py:58-70; ``set_epoch`` reshuffles)."""

    def __init__(self, store: SeqStore, batch_size, seed=0, drop_last=True, timestamps=False):
        self.store, self.batch_size, self.seed, self.drop_last = store, int(batch_size), int(seed), drop_last
        self.timestamps = bool(timestamps)
        self.set_epoch(0)

    def set_epoch(self, epoch):
        self.perm = np.random.default_rng((self.seed, int(epoch))).permutation(len(self.store))

    def __len__(self):
        n = len(self.perm)
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def __getitem__(self, i):
        uids = self.perm[i * self.batch_size:(i + 1) * self.batch_size]
        return torch.from_numpy(uids), self.store.batch(uids, self.timestamps)
