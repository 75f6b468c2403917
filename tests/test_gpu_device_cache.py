"""GPU: the library's device allocation cache (csrc/runtime.cpp cached_malloc / cached_free).

A released buffer goes back to its size-class list and the next allocation of that class gets
it without a new hipMalloc; a trim really frees the cached blocks. Results must not depend on
whether a buffer came from the cache: a two-level amg_2_v repeated after the first call's
objects were released (so every buffer is a reused one) returns the same x and history."""
import gc

import ctypes
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch


def _stats(_lib):
    c, h, m = ctypes.c_size_t(), ctypes.c_int64(), ctypes.c_int64()
    _lib.call("mlamg_device_cache_stats", ctypes.byref(c), ctypes.byref(h), ctypes.byref(m))
    return c.value, h.value, m.value


def test_released_blocks_are_reused_and_trimmed(torch_cuda):
    from mlamg import _lib, problems
    from mlamg.sparse import as_device
    A = problems.poisson_2d_5pt(64)
    Ad = as_device(A)
    del Ad
    gc.collect()
    cached0, hits0, _ = _stats(_lib)
    assert cached0 > 0
    Ad = as_device(A)
    _, hits1, _ = _stats(_lib)
    assert hits1 > hits0
    np.testing.assert_array_equal(Ad.to_scipy().toarray(), A.toarray())
    del Ad
    gc.collect()
    freed = ctypes.c_size_t()
    _lib.call("mlamg_device_cache_trim", ctypes.byref(freed))
    assert freed.value > 0 and _stats(_lib)[0] == 0


def test_amg_2_v_same_result_on_reused_buffers(torch_cuda):
    """PCG coarse solve (n_c > TWO_LEVEL_DENSE_MAX) so the inner hierarchy, GS plan, PCG and
    dense buffers all come back from the cache on the second call."""
    from mlamg import multigrid, problems
    from mlamg.hierarchy import Hierarchy
    import oracle.restated as orc
    m = 96
    A = problems.poisson_2d_5pt(m)
    P, _ = orc.smoothed_aggregation_jacobi(A, problems.box_aggregates_2d(m, m, 3), omega=2.0 / 3.0)
    x0 = np.random.RandomState(1).randn(A.shape[0])
    b = np.zeros(A.shape[0])
    old = Hierarchy.TWO_LEVEL_DENSE_MAX
    Hierarchy.TWO_LEVEL_DENSE_MAX = 256
    try:
        first = multigrid.amg_2_v(A, P, b, x0, res_tol=1e-10, engine="hierarchy")
        gc.collect()
        second = multigrid.amg_2_v(A, P, b, x0, res_tol=1e-10, engine="hierarchy")
    finally:
        Hierarchy.TWO_LEVEL_DENSE_MAX = old
    np.testing.assert_array_equal(first[0], second[0])
    np.testing.assert_array_equal(first[2], second[2])
    assert first[3] == second[3]
