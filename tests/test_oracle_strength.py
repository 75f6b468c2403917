"""CPU: the oracle's restatement of pyamg's evolution strength of connection (the reference's
'evolution' / 'olson' measures, utils/common.py:27,30). pyamg is absent and no reference
fixture pins these values (parity unpinned): checked here against the measure's
defining properties and an independent dense computation of its first stage."""
import numpy as np
import pytest
import scipy.sparse as sp


def _mats():
    from mlamg import problems
    rs = np.random.RandomState(3)
    A2 = problems.poisson_2d_5pt(14)
    B = sp.random(150, 150, density=0.03, random_state=rs, format="csr")
    B = abs(B + B.T)
    A3 = (sp.diags(np.asarray(B.sum(axis=1)).ravel() + 1.0) - B).tocsr()  # SPD M-matrix
    A3.sort_indices()
    return {"poisson2d": A2, "random_m": A3}


@pytest.mark.parametrize("name", ("poisson2d", "random_m"))
def test_evolution_properties(oracle, name):
    A = _mats()[name]
    Dinv_A = sp.diags(1.0 / A.diagonal()) @ A
    lam = np.abs(np.linalg.eigvals(Dinv_A.toarray())).max()
    E = oracle.evolution_strength(A, rho=lam)
    n = A.shape[0]
    # pattern: inside A's pattern (+ diagonal), symmetric (0.5 (E + E^T)); the final row scaling
    # makes the values non-symmetric
    pat = (abs(E) > 0).astype(np.int8)
    assert ((pat - pat.multiply(abs(A) + sp.eye(n) > 0)) != 0).nnz == 0
    assert ((pat - pat.T) != 0).nnz == 0
    assert np.all(E.diagonal() > 0)
    # every row is scaled by its largest |entry| (maximum_row_value + scale_rows)
    Ed = abs(E).toarray()
    assert np.allclose(Ed.max(axis=1), 1.0, rtol=0, atol=1e-15)
    assert np.all(E.data > 0) and np.all(E.data <= 1.0)
    # the first stage against a dense computation: S = ((I - D^-1 A / rho)^T)^2 on A's pattern
    U = np.eye(n) - Dinv_A.toarray() / lam
    S = (U.T @ U.T) * (A.toarray() != 0)
    ref = oracle._incomplete_mat_mult(sp.csr_matrix(U.T), A)
    assert np.allclose(ref.toarray(), S, rtol=1e-13, atol=1e-15)


def test_evolution_isotropic_neighbours_equal(oracle):
    """Constant-coefficient 5-point Laplacian: an interior node's four neighbours are equally
    strong (the measure sees no direction)."""
    from mlamg import problems
    m = 16
    A = problems.poisson_2d_5pt(m)
    lam = np.abs(np.linalg.eigvals((sp.diags(1.0 / A.diagonal()) @ A).toarray())).max()
    E = oracle.evolution_strength(A, rho=lam)
    i = 7 * m + 7
    row = E[i]
    off = row.data[row.indices != i]
    assert len(off) == 4 and np.allclose(off, off[0], rtol=1e-12)


def test_arnoldi_estimate_within_its_tolerance(oracle):
    """approximate_spectral_radius (pyamg's estimate of rho(D^-1 A), seeded like
    utils/common.py:52) lands within its own 1e-2 relative tolerance of the exact value."""
    A = _mats()["random_m"]
    Dinv_A = sp.diags(1.0 / A.diagonal()) @ A
    lam = np.abs(np.linalg.eigvals(Dinv_A.toarray())).max()
    np.random.seed(0)
    rho = oracle.approximate_spectral_radius(Dinv_A.tocsr())
    assert abs(rho - lam) <= 1e-2 * lam


def test_arnoldi_consumes_n_global_draws(oracle):
    """pyamg draws its start vector as np.random.rand(n, 1) from the global generator and
    nothing else: after the estimate the state equals a seed(0) generator advanced by n
    doubles (what lloyd_aggregation(..., rand=None) then permutes from, ns/lib/graph.py:215)."""
    A = _mats()["random_m"]
    Dinv_A = (sp.diags(1.0 / A.diagonal()) @ A).tocsr()
    np.random.seed(0)
    oracle.approximate_spectral_radius(Dinv_A)
    after = np.random.get_state()
    rs = np.random.RandomState(0)
    rs.rand(A.shape[0], 1)
    want = rs.get_state()
    assert np.array_equal(after[1], want[1]) and after[2:] == want[2:]


@pytest.mark.parametrize("name", ("evolution", "olson"))
def test_measures_add_their_second_term(oracle, name):
    A = _mats()["poisson2d"]
    lam = np.abs(np.linalg.eigvals((sp.diags(1.0 / A.diagonal()) @ A).toarray())).max()
    E = oracle.evolution_strength(A, rho=lam)
    C = oracle.strength_measure(A, name, rho=lam)
    extra = (C - E).toarray()
    mask = A.toarray() != 0
    want = np.where(mask, 0.1 if name == "evolution" else 1.0 / np.abs(A.toarray() + ~mask), 0.0)
    assert np.allclose(extra, want, rtol=1e-12, atol=1e-15)
