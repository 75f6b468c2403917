import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "ml-amg_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden", "reference_vectors.npz")
GOLDEN_SINGULAR = os.path.join(ROOT, "tests", "golden", "reference_singular.npz")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and libmlamg_hip.so")
    config.addinivalue_line("markers", "slow: full-size (BASELINE) configurations")


@pytest.fixture(scope="session")
def golden():
    return dict(np.load(GOLDEN, allow_pickle=False))


@pytest.fixture(scope="session")
def golden_singular():
    return dict(np.load(GOLDEN_SINGULAR, allow_pickle=False))


def golden_csr(g, key):
    import scipy.sparse as sp
    shape = tuple(g[f"{key}_shape"]) if f"{key}_shape" in g else None
    return sp.csr_matrix((g[f"{key}_data"], g[f"{key}_indices"], g[f"{key}_indptr"]), shape=shape)


@pytest.fixture(scope="session")
def oracle():
    from oracle import build, restated
    build.build()
    return restated
