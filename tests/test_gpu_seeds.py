"""GPU: the reference's seed selection `np.random.RandomState(seed).permutation(n)[:k]`
(ns/lib/graph.py:230-231, utils/evaluate_dataset.py:80-85) computed by mlamg.graph.
legacy_permutation (csrc/seeds.hip) equals numpy's, element for element, up to the C4 size."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def graph():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mlamg.graph
    return mlamg.graph


@pytest.mark.parametrize("seed,n,k", [(0, 1, 1), (0, 2, 2), (0, 5, 0), (3, 1000, 1000),
                                      (0, 4096, 410), (12345, 65537, 6554),
                                      (2 ** 32 - 1, 300000, 30000), (0, 1048576, 104858),
                                      (0, 10077696, 1007770)])
def test_legacy_permutation_matches_numpy(graph, seed, n, k):
    got = graph.legacy_permutation(seed, n, k).cpu().numpy()
    ref = np.random.RandomState(seed).permutation(n)[:k]
    assert got.shape == (k,) and np.array_equal(got, ref)


def test_legacy_permutation_leaves_global_generator(graph):
    np.random.seed(5)
    a = np.random.rand(3)
    np.random.seed(5)
    graph.legacy_permutation(0, 1000, 100)
    assert np.array_equal(np.random.rand(3), a)
    with pytest.raises(ValueError):
        graph.legacy_permutation(-1, 10, 1)
    with pytest.raises(ValueError):
        graph.legacy_permutation(0, 10, 11)
