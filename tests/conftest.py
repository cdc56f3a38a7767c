"""Test configuration: `gpu` marks tests that need an MI355X (they call libgrk.so)."""
import os
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
GOLDEN = REPO / 'tests' / 'golden'

# Synthetic TencentGR directory used by make_golden.py (regenerated identically by the tests).
GOLDEN_DATA_KW = dict(num_users=24, num_items=300, max_events=40, seed=0, sparse_card=(10, 50, 100), user_card=100)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a HIP device (MI355X) and the built libgrk.so')


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason='no HIP device in this container')
    for item in items:
        if 'gpu' in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope='session')
def golden():
    import numpy as np

    def load(name):
        return np.load(GOLDEN / name, allow_pickle=False)
    return load
