"""CPU: the oracle's restatement of pyamg's smoothed_aggregation_solver recipe (the hierarchy of
ns/preconditioner/PyAMG.py:94), pinned to pyamg's own docstring examples (pyamg is absent here,
so these known answers and the algorithm's invariants are what pin it)."""
import numpy as np
import pytest
import scipy.sparse as sp


def _poisson_2d(m):
    T = sp.diags([-np.ones(m - 1), 2 * np.ones(m), -np.ones(m - 1)], [-1, 0, 1])
    I = sp.identity(m)
    A = sp.csr_matrix(sp.kron(T, I) + sp.kron(I, T))
    A.sort_indices()
    return A


def test_standard_aggregation_docstring_examples(oracle):
    """pyamg.aggregation.standard_aggregation's examples: a 4-vertex 1D mesh gives two
    aggregates {0,1}, {2,3}; an isolated first vertex stays unaggregated."""
    A = sp.csr_matrix(sp.diags([-np.ones(3), 2 * np.ones(4), -np.ones(3)], [-1, 0, 1]))
    agg, cpts, k = oracle.pyamg_standard_aggregation(A)
    assert k == 2 and agg.tolist() == [0, 0, 1, 1] and cpts.tolist() == [0, 3]
    Agg = oracle.pyamg_aggop(agg, k).toarray()
    assert Agg.tolist() == [[1, 0], [1, 0], [0, 1], [0, 1]]
    B = sp.csr_matrix(np.array([[1, 0, 0], [0, 1, 1], [0, 1, 1.0]]))
    agg, cpts, k = oracle.pyamg_standard_aggregation(B)
    assert k == 1 and agg.tolist() == [-1, 0, 0]
    assert oracle.pyamg_aggop(agg, k).toarray().tolist() == [[0], [1], [1]]


def test_fit_candidates_docstring_example(oracle):
    """pyamg.aggregation.fit_candidates's example: the constant over two aggregates of two."""
    T, Bc = oracle.pyamg_fit_candidates(np.array([0, 0, 1, 1], dtype=np.int32), 2, np.ones(4))
    np.testing.assert_allclose(T.toarray(), [[0.70710678, 0], [0.70710678, 0], [0, 0.70710678],
                                             [0, 0.70710678]], rtol=1e-8)
    np.testing.assert_allclose(Bc, [1.41421356, 1.41421356], rtol=1e-8)
    # a zero candidate on an aggregate: T column and B_c zero (threshold tol * norm)
    T, Bc = oracle.pyamg_fit_candidates(np.array([0, 0, 1, 1], dtype=np.int32), 2,
                                        np.array([0.0, 0.0, 3.0, 4.0]))
    assert Bc.tolist() == [0.0, 5.0]
    np.testing.assert_allclose(T.toarray()[:, 1], [0.0, 0.0, 0.6, 0.8], rtol=1e-15)
    assert (T.toarray()[:, 0] == 0).all()


def test_symmetric_strength_rule(oracle):
    """Diagonal always kept; a_ij kept iff a_ij^2 >= theta^2 |a_ii a_jj|; |.| / row max."""
    A = sp.csr_matrix(np.array([[4.0, -1.0, -0.1], [-1.0, 4.0, -2.0], [-0.1, -2.0, 4.0]]))
    S = oracle.pyamg_symmetric_strength(A, 0.1)
    assert S.toarray().tolist() == [[1.0, 0.25, 0.0], [0.25, 1.0, 0.5], [0.0, 0.5, 1.0]]
    S0 = oracle.pyamg_symmetric_strength(A, 0.0)
    assert S0.nnz == A.nnz


def test_standard_aggregation_invariants(oracle):
    """On a symmetric pattern every vertex is aggregated, the roots are pairwise more than two
    edges apart, each root's aggregate holds its whole neighbourhood, and pass 3 adds no
    aggregate."""
    A = _poisson_2d(24)
    agg, cpts, k = oracle.pyamg_standard_aggregation(A)
    assert (agg >= 0).all() and k == len(cpts)
    G = (A != 0).astype(np.int8)
    G2 = (G @ G).tocsr()
    for a, r in enumerate(cpts):
        nb = A.indices[A.indptr[r]:A.indptr[r + 1]]
        assert (agg[nb] == a).all()
        reach = set(G2.indices[G2.indptr[r]:G2.indptr[r + 1]].tolist())
        assert not (reach & (set(cpts.tolist()) - {r}))


def test_block_gauss_seidel_sweeps(oracle):
    """block_gauss_seidel: forward = x_i <- (b_i - sum_j a_ij x_j) / a_ii in row order, backward
    in reverse order, symmetric = both; a symmetric sweep is an A-norm contraction on SPD A."""
    A = sp.csr_matrix(np.array([[2.0, -1.0], [-1.0, 2.0]]))
    b = np.array([1.0, 0.0])
    x = np.zeros(2)
    oracle.pyamg_block_gauss_seidel(A, x, b, 1, "forward")
    assert x.tolist() == [0.5, 0.25]
    x = np.zeros(2)
    oracle.pyamg_block_gauss_seidel(A, x, b, 1, "backward")
    assert x.tolist() == [0.5, 0.0]
    P = _poisson_2d(16)
    rng = np.random.default_rng(0)
    e = rng.standard_normal(P.shape[0])
    z = np.zeros_like(e)
    before = e @ (P @ e)
    oracle.pyamg_block_gauss_seidel(P, e, z, 1, "symmetric")
    assert e @ (P @ e) < 0.9 * before


def test_pyamg_sa_setup_and_cycle(oracle):
    """The restated smoothed_aggregation_solver on a 2D Poisson problem: levels down to <= 10
    rows, improved candidate still near constant on level 0, Galerkin operators symmetric, and
    the V-cycle a contraction with factor well below 0.5 (pyamg's SA on 2D Poisson)."""
    A = _poisson_2d(32)
    levels, Ac = oracle.pyamg_sa_setup(A)
    assert Ac.shape[0] <= 10 and len(levels) >= 2
    assert abs(levels[0]["rho"] - 2.0) < 0.01  # rho(D^-1 A) of the 5-point Laplacian -> 2
    for L in levels:
        assert abs(L["A"] - L["A"].T).max() <= 1e-12 * abs(L["A"]).max()
    import scipy.linalg
    pinv = scipy.linalg.pinv(Ac.toarray())
    rng = np.random.default_rng(1)
    b = rng.standard_normal(A.shape[0])
    x = np.zeros_like(b)
    norms = []
    for _ in range(6):
        oracle.pyamg_sa_vcycle(levels, pinv, b, x)
        norms.append(np.linalg.norm(b - A @ x))
    rates = np.array(norms[1:]) / np.array(norms[:-1])
    assert rates.max() < 0.5, rates


@pytest.mark.parametrize("m", [5, 9])
def test_pyamg_sa_tiny_is_coarse_only(oracle, m):
    """n <= max_coarse: no level, the cycle is the pinv solve."""
    A = sp.csr_matrix(sp.diags([-np.ones(m - 1), 2 * np.ones(m), -np.ones(m - 1)], [-1, 0, 1]))
    levels, Ac = oracle.pyamg_sa_setup(A)
    assert levels == [] and Ac.shape == (m, m)


def test_gmres_householder_docstring_example():
    """pyamg.krylov.gmres's docstring example (orthog='householder'): poisson((10, 10)),
    b = ones, maxiter=2, tol=1e-8 prints norm(b - A x) = 6.54282; the restatement's loop with
    an identity preconditioner reproduces it, and with an exact one stops after one step."""
    import mlamg.problems as P
    from oracle import restated as R
    A = P.poisson_2d_5pt(10)
    b = np.ones(100)
    x, info, it, res = R.pyamg_gmres_householder(A, b, lambda r: r, tol=1e-8, maxiter=2)
    assert f"{np.linalg.norm(b - A @ x):.6}" == "6.54282"
    assert it == 2 and info == 2 and len(res) == 3
    Ainv = np.linalg.inv(A.toarray())
    x, info, it, res = R.pyamg_gmres_householder(A, b, lambda r: Ainv @ r, tol=1e-10)
    assert it == 1 and info == 0
    np.testing.assert_allclose(A @ x, b, atol=1e-12)
