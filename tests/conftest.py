import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, 'radar-slam_amd'), os.path.join(ROOT, 'oracle'), os.path.join(ROOT, 'tests')):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, 'tests', 'golden')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (HIP) device; run with -m gpu')


@pytest.fixture(scope='session')
def golden():
    cache = {}

    def load(name):
        if name not in cache:
            z = np.load(os.path.join(GOLDEN, f'golden_{name}.npz'), allow_pickle=False)
            cache[name] = {k: z[k] for k in z.files}
        return cache[name]
    return load


@pytest.fixture(scope='session')
def ctx():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    import rsl
    return rsl.get_context(0)
