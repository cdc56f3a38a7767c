"""Retrieval file formats and host logic (no GPU): the reference's own
save_emb bytes and read_result_ids reading (tests/golden/retrieval.npz,
model/BaseLine/dataset.py:421-434, infer.py:51-65), the oracle's exact top-k,
and the faiss_demo command line."""
import numpy as np
import pytest

from conftest import GOLDEN
from oracle import retrieval as oret
from tencent_recommendation_2025_amd import retrieval as R

G = np.load(GOLDEN / 'retrieval.npz')


def test_read_bin_parses_reference_save_emb(tmp_path):
    for name, dtype in (('items', np.float32), ('queries', np.float32), ('ids', np.uint64)):
        p = tmp_path / name
        p.write_bytes(G[f'{name}_bytes'].tobytes())
        got = R.read_bin(p, dtype)
        assert got.dtype == dtype and np.array_equal(got, G[name])


def test_result_file_matches_reference_reader(tmp_path):
    p = tmp_path / 'id100.u64bin'
    R.write_result_ids(G['top10_ids'], p)
    assert p.read_bytes() == G['result_bytes'].tobytes()
    assert np.array_equal(R.read_result_ids(p), G['result_read_by_reference'])
    assert np.array_equal(oret.read_result_ids(p), G['result_read_by_reference'])
    oret.write_result_ids(G['top10_ids'], tmp_path / 'o')
    assert (tmp_path / 'o').read_bytes() == p.read_bytes()


def test_missing_ids_written_as_faiss_minus_one(tmp_path):
    R.write_result_ids(np.array([[5, -1]]), tmp_path / 'r')
    assert R.read_result_ids(tmp_path / 'r').tolist() == [[5, 2 ** 64 - 1]]


def test_oracle_topk_order_and_fill():
    q = np.array([[1.0, 0.0]])
    x = np.array([[1.0, 0.0], [2.0, 0.0], [1.0, 5.0], [2.0, 1.0]])
    s, i = oret.mips_topk(q, x, 6)
    # scores 1, 2, 1, 2: ties broken by the lower item row; past 4 items -> -1 / -inf
    assert i.tolist() == [[1, 3, 0, 2, -1, -1]]
    assert s[0, :4].tolist() == [2.0, 2.0, 1.0, 1.0] and np.isneginf(s[0, 4:]).all()
    s2, i2 = oret.mips_topk(q, x, 2, item_ids=[10, 11, 12, 13])
    assert i2.tolist() == [[11, 13]]
    assert np.array_equal(oret.mips_topk(q, x[:0], 3)[1], [[-1, -1, -1]])


def test_oracle_golden_top10_is_exact():
    s = G['queries'].astype(np.float64) @ G['items'].astype(np.float64).T
    ref = G['ids'].reshape(-1)[np.argsort(-s, axis=1, kind='stable')[:, :10]]
    assert np.array_equal(G['top10_ids'], ref.astype(np.int64))


def test_cli_rejects_other_metrics(tmp_path):
    with pytest.raises(SystemExit):
        R.main(['--dataset_vector_file_path=a', '--dataset_id_file_path=b', '--query_vector_file_path=c',
                '--result_id_file_path=d', '--faiss_metric_type=1'])
