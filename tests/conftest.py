import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, 'tests', 'golden')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a real MI355X (HIP device); run with -m gpu')
    config.addinivalue_line('markers', 'slow: long-running case')


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope='session')
def simple_golden():
    return load_golden('simple.npz')


@pytest.fixture(scope='session')
def sphere_inputs():
    return load_golden('sphere_inputs.npz')


@pytest.fixture(scope='session')
def sphere_naive():
    return load_golden('sphere_raster_naive.npz')


@pytest.fixture(scope='session')
def sphere_softmask():
    return load_golden('sphere_softmask.npz')


@pytest.fixture(scope='session')
def soup_naive():
    return load_golden('soup_raster_naive.npz')
