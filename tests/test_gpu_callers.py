"""GPU: the reference's caller loops run through mlamg.compat.install() alone (pyamg and
torch_sparse absent) and reproduce the reference's own results on the device
(tests/golden/reference_callers.npz, made by running the reference's utils/common.py and
utils/evaluate_dataset.py in the container: tests/golden/make_golden_callers.py).

The loop bodies are restated below line by line (the reference tree does not travel to the GPU
box); every call inside them goes through the aliased module names, as in the scripts.
Aggregate maps (the Agg each loop hands to smoothed_aggregation_jacobi) are compared bitwise,
conv factors to 1e-8 absolute (the coarse solve is the device's dense inverse
against SuperLU, and omega the device Lanczos against ARPACK, both at fp64 rounding)."""
import os
import sys

import numpy as np
import numpy.linalg as la
import pytest
import scipy.sparse as sp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
CONV_TOL = 1e-8


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(os.path.join(HERE, "golden", "reference_callers.npz"), allow_pickle=False))


@pytest.fixture(scope="module")
def aliases():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mlamg.compat
    saved = {k: v for k, v in sys.modules.items()
             if k == "pyamg" or k.startswith("pyamg.") or k == "ns" or k.startswith("ns.")}
    for k in saved:
        del sys.modules[k]
    installed = mlamg.compat.install(pyamg=True)
    yield installed
    mlamg.compat.uninstall(installed)
    sys.modules.update(saved)


class Grid:
    def __init__(self, A):
        self.A = A


def _dataset(g):
    out, i = [], 0
    while f"ds{i}_indptr" in g:
        out.append(Grid(sp.csr_matrix((g[f"ds{i}_data"], g[f"ds{i}_indices"], g[f"ds{i}_indptr"]))))
        i += 1
    return out


def _olson(A):
    """utils/common.py:30 (strength_measure_funcs['olson']) on the aliased pyamg."""
    import pyamg.strength
    return pyamg.strength.evolution_strength_of_connection(A) + \
        sp.csr_matrix((1. / np.abs(A.data), A.indices, A.indptr), A.shape)


def _conv(res):
    return 0.0 if np.isnan(res) else res


def evaluate_ref_conv(dataset, strength_measure_func, seen, alpha=0.3, omega=2. / 3.):
    """utils/common.py:84-111 (the exception branch only plots)."""
    import ns.lib.multigrid
    import pyamg.aggregation
    conv = np.zeros(len(dataset))
    for i in range(len(dataset)):
        A = dataset[i].A
        np.random.seed(0)
        C = strength_measure_func(A)
        Agg, _ = pyamg.aggregation.lloyd_aggregation(C, ratio=alpha, distance='same')
        seen.append(Agg)
        P = ns.lib.multigrid.smoothed_aggregation_jacobi(A, Agg)
        b = np.zeros(A.shape[1])
        np.random.seed(0)
        x = np.random.randn(A.shape[1])
        x /= la.norm(x, 2)
        np.random.seed()
        conv[i] = _conv(ns.lib.multigrid.amg_2_v(A, P, b, x, res_tol=1e-10, singular=False,
                                                 jacobi_weight=omega)[1])
    return conv


def evaluate_dataset_common(dataset, seen, alpha=0.3, omega=2. / 3.):
    """utils/common.py:40-82 with model=None, S=None."""
    import ns.lib.graph
    import ns.lib.multigrid
    conv = np.zeros(len(dataset))
    for i in range(len(dataset)):
        A = dataset[i].A
        n = A.shape[1]
        b = np.zeros(n)
        np.random.seed(0)
        C = _olson(A)
        L_Agg, L_Roots, L_Seeds = ns.lib.graph.lloyd_aggregation(C, ratio=alpha, distance='same',
                                                                 rand=0)
        seen.append(L_Agg)
        P = ns.lib.multigrid.smoothed_aggregation_jacobi(A, L_Agg)
        x = np.random.RandomState(0).randn(A.shape[1])
        x /= la.norm(x, 2)
        conv[i] = _conv(ns.lib.multigrid.amg_2_v(A, P, b, x, res_tol=1e-10, singular=False,
                                                 jacobi_weight=omega)[1])
    return conv


def evaluate_dataset_script(dataset, method, seen, alpha=0.1, omega=2. / 3.):
    """utils/evaluate_dataset.py:59-101, methods 'lloyd' and 'dumb' ('ml' needs weights)."""
    import torch
    import ns.lib.graph
    import ns.lib.multigrid
    import ns.lib.sparse
    import pyamg.aggregation
    conv = np.zeros(len(dataset))
    for i in range(len(dataset)):
        A = dataset[i].A
        np.random.seed(0)
        if method == 'lloyd':
            C = _olson(A)
            Agg, _ = pyamg.aggregation.lloyd_aggregation(C, ratio=alpha, distance='same')
        else:
            rand = np.random.RandomState(0)
            N = A.shape[0]
            num_seeds = int(np.ceil(alpha * N))
            seeds = rand.permutation(N)[:num_seeds]
            C = _olson(A)
            seeds_T = torch.Tensor(seeds).long()
            distance, nearest_center = ns.lib.graph.modified_bellman_ford(
                ns.lib.sparse.scipy_to_torch(C), seeds_T)
            Agg_T = ns.lib.graph.nearest_center_to_agg(seeds_T, nearest_center)
            Agg = ns.lib.sparse.torch_to_scipy(Agg_T)
        seen.append(Agg)
        P = ns.lib.multigrid.smoothed_aggregation_jacobi(A, Agg)
        b = np.zeros(A.shape[1])
        x = np.random.RandomState(0).randn(A.shape[1])
        x /= la.norm(x, 2)
        conv[i] = _conv(ns.lib.multigrid.amg_2_v(A, P, b, x, res_tol=1e-10, singular=False,
                                                 jacobi_weight=omega)[1])
    return conv


RUNS = {
    "ref_conv": lambda ds, seen: evaluate_ref_conv(ds, _olson, seen, alpha=0.1),
    "common_ed": lambda ds, seen: evaluate_dataset_common(ds, seen, alpha=0.1),
    "ed_lloyd": lambda ds, seen: evaluate_dataset_script(ds, 'lloyd', seen),
    "ed_dumb": lambda ds, seen: evaluate_dataset_script(ds, 'dumb', seen),
}


@pytest.mark.parametrize("name", tuple(RUNS))
def test_caller_loop_matches_reference(aliases, gold, name):
    ds = _dataset(gold)
    seen = []
    conv = RUNS[name](ds, seen)
    assert len(seen) == len(ds)
    for i, Agg in enumerate(seen):
        Agg = sp.csr_matrix(Agg)
        Agg.sort_indices()
        assert np.array_equal(Agg.indptr, gold[f"{name}{i}_agg_indptr"]), (name, i)
        assert np.array_equal(Agg.indices, gold[f"{name}{i}_agg_indices"]), (name, i)
    ref = gold[f"{name}_conv"]
    assert np.all(np.abs(conv - ref) <= CONV_TOL), (conv, ref)


def test_pyamg_lloyd_aggregation_global_rng(aliases, oracle):
    """pyamg.aggregation.lloyd_aggregation (aliased) vs the oracle's pyamg 4.x restatement:
    seed count int(min(max(ratio N, 1), N)), seeds from the global generator inside
    lloyd_cluster (generator state after the call identical), (AggOp, seeds) bitwise."""
    import pyamg.aggregation
    from mlamg import problems
    A = problems.poisson_2d_5pt(30)
    C = abs(A).tocsr()
    for ratio, distance in ((0.1, 'unit'), (0.05, 'same'), (1e-4, 'abs')):
        np.random.seed(11)
        Agg, seeds = pyamg.aggregation.lloyd_aggregation(C, ratio=ratio, distance=distance)
        st = np.random.get_state()
        np.random.seed(11)
        AggR, seedsR = oracle.pyamg_lloyd_aggregation(C, ratio=ratio, distance=distance)
        stR = np.random.get_state()
        assert np.array_equal(seeds, seedsR) and seeds.dtype == np.intc
        assert np.array_equal(Agg.indptr, AggR.indptr) and np.array_equal(Agg.indices, AggR.indices)
        assert Agg.dtype == np.int8 and Agg.shape == AggR.shape
        assert np.array_equal(st[1], stR[1]) and st[2] == stR[2]


def test_pyamg_gauss_seidel_in_place(aliases, oracle):
    """pyamg.relaxation.relaxation.gauss_seidel (aliased; ns/lib/multigrid.py:175,184 calls it
    with x updated in place) bitwise against the oracle's forward sweep."""
    import pyamg.relaxation.relaxation as rr
    from mlamg import problems
    A = problems.poisson_2d_5pt(17)
    rs = np.random.RandomState(3)
    x, b = rs.randn(A.shape[0]), rs.randn(A.shape[0])
    ref = oracle.gauss_seidel(A, x.copy(), b, iterations=3)
    xx = x.copy()
    assert rr.gauss_seidel(A, xx, b, iterations=3) is None
    assert np.array_equal(xx, ref)
