"""GPU: coarsest solve without a size cap.

The reference factorises the Galerkin operator at any size (`spla.factorized(A_H)`,
ns/lib/multigrid.py:168; `splu`, MLAMG.py:122). Above Hierarchy.DENSE_MAX rows the device solves
the coarse system by PCG preconditioned with an inner SA hierarchy of A_H, to
||r_H|| <= 1e-12 ||b_H|| (csrc/pcg.hip). Parity is a tolerance: the outer residual histories must
match the oracle's SuperLU-based ones within rtol 1e-10 (SURVEY.md §8(d) history bound)."""
import numpy as np
import pytest
import scipy.sparse.linalg as spla

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch


@pytest.fixture(scope="module")
def ml(torch_cuda):
    import mlamg.hierarchy
    import mlamg.multigrid
    import mlamg.problems
    return mlamg


def _sa_P(ml, A):
    """P of the first level of the device's SA hierarchy (seeded Bellman-Ford, alpha = 0.1)."""
    H = ml.hierarchy.Hierarchy.build(A, alpha=0.1, max_levels=2, finalize=False)
    return H.levels[0].P.to_scipy()


def test_pcg_coarse_solve_accuracy(ml, torch_cuda):
    """PCG with the inner hierarchy solves A_c x = b to the requested relative residual; the
    solution matches SuperLU's within cond-scaled rounding."""
    torch = torch_cuda
    A = ml.problems.poisson_2d_5pt(128)
    P = _sa_P(ml, A)
    H = ml.hierarchy.Hierarchy.two_level(A, P)
    assert H.dense is not None  # n_c ~ 1.6k: dense
    Hp = ml.hierarchy.Hierarchy.build(A, alpha=0.1, max_levels=2, finalize=False)
    Hp._finalize(1, 1, dense_max=100)
    assert Hp.pcg is not None and Hp.inner is not None
    Ac = Hp.Ac.to_scipy()
    b = np.random.RandomState(3).randn(Ac.shape[0])
    ref = spla.spsolve(Ac.tocsc(), b)
    from mlamg._lib import call, ptr, stream_ptr
    bd = torch.as_tensor(b).cuda()
    xd = torch.zeros_like(bd)
    call("mlamg_pcg_solve", Hp.pcg, ptr(bd), ptr(xd), stream_ptr())
    x = xd.cpu().numpy()
    st = Hp.coarse_stats()
    assert st["not_converged"] == 0 and 1 <= st["last_iters"] <= 60, st
    assert np.linalg.norm(b - Ac @ x) <= 1.01e-12 * np.linalg.norm(b)
    assert np.abs(x - ref).max() <= 1e-9 * np.abs(ref).max()
    # zero right-hand side: x = 0 with no iteration
    xd.fill_(1.0)
    call("mlamg_pcg_solve", Hp.pcg, ptr(torch.zeros_like(bd)), ptr(xd), stream_ptr())
    assert not torch.any(xd).item()


def test_multilevel_pcg_coarse_matches_dense(ml, oracle, torch_cuda):
    """Two-level hierarchy (max_levels=2) with a PCG coarsest solve vs the oracle cycle with
    SuperLU on the same operators: residual histories within rtol 1e-10."""
    torch = torch_cuda
    from test_gpu_hierarchy import _oracle_levels_from_device
    A = ml.problems.poisson_2d_5pt(256)
    H = ml.hierarchy.Hierarchy.build(A, alpha=0.1, max_levels=2)
    assert H.Ac.shape[0] > H.DENSE_MAX and H.pcg is not None
    lv = _oracle_levels_from_device(H)
    n = A.shape[0]
    x0 = np.random.RandomState(0).randn(n)
    b = np.random.RandomState(1).randn(n)
    xo, ho = oracle.vcycle_solve(lv, H.Ac.to_scipy(), b, x0, 8)
    xd = torch.as_tensor(x0).cuda()
    hd = H.cycle(torch.as_tensor(b).cuda(), xd, 8)
    assert np.allclose(hd, ho, rtol=1e-10, atol=0), (hd, ho)
    assert np.allclose(xd.cpu().numpy(), xo, rtol=0, atol=1e-9 * np.abs(xo).max())
    st = H.coarse_stats()
    assert st["not_converged"] == 0 and st["max_rel_residual"] <= 1e-12


@pytest.mark.slow
def test_amg_2_v_large_coarse_1024(ml, oracle, torch_cuda):
    """The reference two-level solve at 1024^2 with alpha = 0.1 aggregates (n_c ~ 105k, beyond
    any dense inverse): the reference path factorises A_H with SuperLU; the device solves it by
    PCG. Gauss-Seidel smoother (the reference default) and the Jacobi form; histories within
    rtol 1e-10, conv factors within 1e-8."""
    A = ml.problems.poisson_2d_5pt(1024)
    P = _sa_P(ml, A)
    assert P.shape[1] > 100000
    n = A.shape[0]
    x0 = np.random.RandomState(0).randn(n)
    x0 /= np.linalg.norm(x0)
    b = np.zeros(n)
    for smoother in ("gauss_seidel", "jacobi"):
        xr, cr, er, ir = oracle.amg_2_v(A, P, b, x0, res_tol=1e-12, max_iter=30,
                                        smoother=smoother)
        x, c, e, it = ml.multigrid.amg_2_v(A, P, b, x0, res_tol=1e-12, max_iter=30,
                                           smoother=smoother)
        assert it == ir, (smoother, it, ir)
        assert np.allclose(e, er, rtol=1e-10, atol=0), (smoother, e, er)
        assert abs(c - cr) <= 1e-8
        assert np.abs(x - xr).max() <= 1e-8 * np.abs(xr).max()


def test_csr_symmetric_check(ml, torch_cuda):
    """mlamg_csr_symmetric: exact and to-rounding symmetry of unsorted Galerkin-like rows."""
    import scipy.sparse as sp
    from mlamg.hierarchy import csr_symmetric
    from mlamg.sparse import DeviceCSR
    A = ml.problems.poisson_2d_5pt(20).tocsr()
    assert csr_symmetric(DeviceCSR.from_scipy(A))
    B = A.copy()
    B.data = B.data.copy()
    B.data[5] *= 1 + 1e-14  # symmetric to rounding only
    assert not csr_symmetric(DeviceCSR.from_scipy(B), 0.0)
    assert csr_symmetric(DeviceCSR.from_scipy(B), 1e-12)
    C = A.tolil()
    C[0, 7] = 0.5  # no mirror entry: a_70 counts as 0
    assert not csr_symmetric(DeviceCSR.from_scipy(C.tocsr()), 1e-12)
    # unsorted rows (scipy's csr_matmat order) are fine
    A = ml.problems.poisson_2d_5pt(48).tocsr()
    P = _sa_P(ml, A)
    Ac = ml.sparse.galerkin(ml.sparse.DeviceCSR.from_scipy(P.T.tocsr()),
                            DeviceCSR.from_scipy(A), DeviceCSR.from_scipy(P))
    assert csr_symmetric(Ac, 1e-12)
    assert not csr_symmetric(DeviceCSR.from_scipy(sp.random(6, 7, 0.5, format="csr")), 1.0)


def test_nonsymmetric_coarse_takes_dense_or_gmres(ml, torch_cuda, monkeypatch):
    """A coarse operator that is not symmetric never goes to PCG: dense inverse up
    to DENSE_LIMIT rows, GMRES with an inner hierarchy above (VERDICT r05 Weak #9)."""
    import scipy.sparse as sp
    H_ = ml.hierarchy.Hierarchy
    A = ml.problems.poisson_2d_5pt(48).tocsr()
    n = A.shape[0]
    # upwind convection: A + c * (I - shift) is not symmetric
    A = (A + 0.5 * (sp.eye(n) - sp.eye(n, k=-1))).tocsr()
    P = _sa_P(ml, ml.problems.poisson_2d_5pt(48))
    monkeypatch.setattr(H_, "TWO_LEVEL_DENSE_MAX", 16)
    H = H_.two_level(A, P)
    assert H.pcg is None and H.dense is not None
    monkeypatch.setattr(H_, "DENSE_LIMIT", 64)
    H = H_.two_level(A, P)
    assert H.pcg is None and H.dense is None and H.coarse_gmres
    assert H.describe()[-1]["coarse"].startswith("GMRES")


def _upwind(ml, m, c=0.5):
    """2D 5-point Laplacian on m x m plus first-order upwind convection c (I - shift): an
    M-matrix whose Galerkin coarse operator is not symmetric."""
    import scipy.sparse as sp
    A = ml.problems.poisson_2d_5pt(m).tocsr()
    n = A.shape[0]
    return sp.csr_matrix(A + c * (sp.eye(n) - sp.eye(n, k=-1)))


@pytest.mark.parametrize("m,limit,inner_max", ((48, 64, 60), (128, 1000, 300)))
@pytest.mark.parametrize("smoother", ("gauss_seidel", "jacobi"))
def test_gmres_coarse_matches_superlu(ml, oracle, torch_cuda, monkeypatch, m, limit, inner_max,
                                      smoother):
    """A non-symmetric A_H beyond the dense solver's size (DENSE_LIMIT patched below n_c) is
    solved by GMRES preconditioned by an inner hierarchy (inner levels forced by patching its
    coarsest size) to 1e-14 relative: amg_2_v's residual history matches the oracle's SuperLU
    (spla.factorized, ns/lib/multigrid.py:168) within the SURVEY §8(d) history bound (1e-10
    relative + 1e-13 of the first residual) with the same iteration count and conv factor
    within 1e-8."""
    H_ = ml.hierarchy.Hierarchy
    A = _upwind(ml, m)
    n = A.shape[0]
    P = _sa_P(ml, ml.problems.poisson_2d_5pt(m))
    assert P.shape[1] > limit
    monkeypatch.setattr(H_, "TWO_LEVEL_DENSE_MAX", 16)
    monkeypatch.setattr(H_, "DENSE_LIMIT", limit)
    monkeypatch.setattr(H_, "PCG_INNER_MAX_COARSE", inner_max)
    H = H_.two_level(A, P, smoother=smoother)
    assert H.coarse_gmres and H.inner.n_levels >= 2
    x0 = np.random.RandomState(0).randn(n)
    b = np.random.RandomState(1).randn(n)
    # res_tol 1e-6 (7 decades below ||r_0|| ~ 20): deeper, the residual norms approach the
    # rounding floor of b - A x itself (eps ||A|| ||x|| ~ 1e-13 here), where any two coarse
    # solvers that differ in the last bits give histories that differ in their leading digits
    x, c, e, it = ml.multigrid.amg_2_v(A, P, b, x0, res_tol=1e-6, max_iter=100,
                                       smoother=smoother, engine="hierarchy")
    xr, cr, er, ir = oracle.amg_2_v(A, P, b, x0, res_tol=1e-6, max_iter=100, smoother=smoother)
    assert it == ir > 3, (it, ir)
    # |r_k - r_k^ref| <= 1e-10 r_k^ref + 1e-13 r_0 (the 1e-14 coarse solve
    # perturbs each cycle by ~1e-14 of the coarse right-hand side, against SuperLU's rounding)
    assert np.allclose(e, er, rtol=1e-10, atol=1e-13 * er[0]), (e, er)
    assert abs(c - cr) <= 1e-8
    assert np.abs(x - xr).max() <= 1e-8 * np.abs(xr).max()
    # the coarse solves themselves: every one converged to the GMRES tolerance
    Hc = H_.two_level(A, P, smoother=smoother)
    xd = torch_cuda.as_tensor(x0).cuda()
    Hc.cycle(torch_cuda.as_tensor(b).cuda(), xd, 5)
    st = Hc.coarse_stats()
    assert st["solver"] == "gmres" and st["solves"] == 5 and st["not_converged"] == 0
    assert st["max_rel_residual"] <= 1e-14 and st["last_iters"] >= 1


def test_pcg_breakdown_is_reported(ml, oracle, torch_cuda, monkeypatch):
    """An indefinite symmetric coarse operator (tridiag(1, 1, 1): spectrum (-1, 3), positive
    diagonal; P = I so A_H = A) passes the symmetry test, so PCG is chosen, and breaks down
    (p.Ap or r.z not positive). The breakdown is counted and the cycle raises CoarseSolveError.
    amg_2_v then inverts A_H densely (Gauss-Jordan with pivoting, as SuperLU would factor any
    nonsingular A_H) and reruns: n = 2001 is nonsingular (tridiag(1,1,1) of order n is singular
    iff 3 | n + 1), so the solve converges and matches the oracle's (scipy factorized) iterate;
    only a factorisation failure maps to (x, 1.0, zeros, 0), ns/lib/multigrid.py:167-170."""
    import scipy.sparse as sp
    torch = torch_cuda
    H_ = ml.hierarchy.Hierarchy
    n = 20000
    A = sp.diags([np.ones(n - 1), np.ones(n), np.ones(n - 1)], [-1, 0, 1], format="csr")
    P = sp.eye(n, format="csr")
    monkeypatch.setattr(H_, "TWO_LEVEL_DENSE_MAX", 64)
    H = H_.two_level(A, P, smoother="jacobi")
    assert H.pcg is not None
    b = torch.as_tensor(np.random.RandomState(1).randn(n)).cuda()
    xd = torch.zeros(n, dtype=torch.float64, device="cuda")
    with pytest.raises(ml.hierarchy.CoarseSolveError):
        H.cycle(b, xd, 3)
    assert H.coarse_stats()["breakdowns"] >= 1
    with pytest.raises(ml.hierarchy.CoarseSolveError):  # inside the preconditioner too
        H.gmres(b, rtol=1e-8, restart=5, maxiter=1)
    n = 2001
    A = sp.diags([np.ones(n - 1), np.ones(n), np.ones(n - 1)], [-1, 0, 1], format="csr")
    P = sp.eye(n, format="csr")
    assert H_.two_level(A, P).pcg is not None
    x0 = np.random.RandomState(0).randn(n)
    bb = np.random.RandomState(1).randn(n)
    x, c, e, it = ml.multigrid.amg_2_v(A, P, bb, x0, res_tol=1e-10, max_iter=7,
                                       engine="hierarchy")
    xr, cr, er, itr = oracle.amg_2_v(A, P, bb, x0, res_tol=1e-10, max_iter=7)
    assert it >= 1 and x is not x0
    assert np.linalg.norm(bb - A @ x) <= 1e-10 and e[-1] <= 1e-10
    assert np.linalg.norm(x - xr) <= 1e-10 * np.linalg.norm(xr)
    # A_H beyond the dense solver's size: the dense retry cannot run; the GMRES coarse solve
    # (inner hierarchy of the indefinite A_H as preconditioner) is tried next
    monkeypatch.setattr(H_, "DENSE_LIMIT", 1000)
    x, c, e, it = ml.multigrid.amg_2_v(A, P, bb, x0, res_tol=1e-10, max_iter=7,
                                       engine="hierarchy")
    print("indefinite A_H beyond DENSE_LIMIT:", it, c, e[:3])
    if it == 0:  # GMRES did not converge: the reference's failure tuple, never an exception
        assert x is x0 and c == 1.0 and np.array_equal(e, np.zeros(7))
    else:
        assert np.linalg.norm(x - xr) <= 1e-8 * np.linalg.norm(xr)
    # a singular A_H (tridiag(1, 1, 1) of order 2000: 3 | 2001) beyond DENSE_LIMIT: GMRES cannot
    # reach its tolerance for a b outside the range, the failure tuple as SuperLU's
    n = 2000
    A = sp.diags([np.ones(n - 1), np.ones(n), np.ones(n - 1)], [-1, 0, 1], format="csr")
    P = sp.eye(n, format="csr")
    x0 = np.random.RandomState(0).randn(n)
    bb = np.random.RandomState(1).randn(n)
    x, c, e, it = ml.multigrid.amg_2_v(A, P, bb, x0, res_tol=1e-10, max_iter=7,
                                       engine="hierarchy")
    assert x is x0 and c == 1.0 and it == 0 and np.array_equal(e, np.zeros(7))
