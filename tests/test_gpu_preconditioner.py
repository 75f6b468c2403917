"""GPU: the PETSc python-PC surface (ns/preconditioner/MLAMG.py:27-222, mirrored by
mlamg.preconditioner.MLAMG / MultilevelPC) and the package-level setup/precondition/solve,
driven through duck-typed petsc4py stand-ins (petsc4py/firedrake are not in the image).

MLAMG.apply (:199-212) draws x0 from the global np.random.normal and runs the two-level
weighted-Jacobi cycle until ||b - A x||_2 <= amg_rtol (:194) — checked against the oracle's
restatement of that driver (oracle.mlamg_amg_2_v) on the same x0 and P.
"""
import numpy as np
import pytest
import scipy.sparse as sp

pytestmark = pytest.mark.gpu


class _Mat:
    def __init__(self, A):
        self.A = A.tocsr()

    def getValuesCSR(self):
        return self.A.indptr, self.A.indices, self.A.data


class _PC:
    def __init__(self, A, prefix=""):
        self.m = _Mat(A)
        self.prefix = prefix

    def getOperators(self):
        return self.m, self.m

    def getOptionsPrefix(self):
        return self.prefix


class _Vec:
    def __init__(self, a=None, n=0):
        self.array_r = None if a is None else np.asarray(a, dtype=np.float64)
        self.out = np.zeros(n)

    def setArray(self, v):
        self.out = np.array(v, copy=True)


class _Viewer:
    def __init__(self):
        self.text = []

    def printfASCII(self, s):
        self.text.append(s)


@pytest.fixture(scope="module")
def ml():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mlamg.preconditioner
    import mlamg.problems
    return mlamg


@pytest.fixture(autouse=True)
def _clean_options(ml):
    ml.preconditioner._Options.store.clear()
    yield
    ml.preconditioner._Options.store.clear()


def test_mlamg_pc_apply_matches_reference_driver(ml, oracle):
    A = ml.problems.poisson_2d_5pt(48)
    Agg = ml.problems.box_aggregates_2d(48, 48, 3)
    P, _ = oracle.smoothed_aggregation_jacobi(A, Agg, omega=2.0 / 3.0)
    n = A.shape[0]
    b = np.random.RandomState(3).randn(n)
    pc = _PC(A)
    M = ml.preconditioner.MLAMG()
    M.set_prolongator(P)
    M.initialize(pc)
    assert M.amg_rtol == 1e-8 and abs(M.jacobi_weight - 2.0 / 3.0) < 1e-16
    X, Y = _Vec(b), _Vec(n=n)
    np.random.seed(11)
    M.apply(pc, X, Y)
    np.random.seed(11)
    x0 = np.random.normal(size=n)  # MLAMG.py:209, the same global-RNG draw
    Dinv_w = oracle.mlamg_dinv(A)
    xr, hr = oracle.mlamg_amg_2_v(A, P, Dinv_w, b, x0, amg_rtol=1e-8)
    assert hr[-1] <= 1e-8
    assert np.linalg.norm(b - A @ Y.out) <= 1e-8
    assert np.abs(Y.out - xr).max() <= 1e-8 * np.abs(xr).max()


def test_mlamg_pc_options_prefix_and_defaults(ml):
    A = ml.problems.poisson_2d_5pt(40)
    n = A.shape[0]
    ml.preconditioner._Options.store.update({"fs_mlamg_amg_rtol": 1e-4, "fs_mlamg_alpha": 0.2})
    pc = _PC(A, prefix="fs_")
    M = ml.preconditioner.MLAMG()
    M.initialize(pc)  # no user P: SA prolongator of seeded Bellman-Ford aggregates on the GPU
    assert M.amg_rtol == 1e-4 and M.alpha == 0.2
    assert M.H.n_levels == 2
    b = np.random.RandomState(0).randn(n)
    Y = _Vec(n=n)
    M.apply(pc, _Vec(b), Y)
    r = np.linalg.norm(b - A @ Y.out)
    assert r <= 1e-4
    M.update(pc)  # re-assembly hook rebuilds the solver (MLAMG.py:126)
    M.apply(pc, _Vec(b), Y)
    assert np.linalg.norm(b - A @ Y.out) <= 1e-4
    v = _Viewer()
    M.view(pc, v)
    assert any("MLAMG" in t for t in v.text)
    M.applyTranspose(pc, _Vec(b), Y)  # a no-op in the reference (:214-216)


@pytest.mark.parametrize("gmres", (True, False))
def test_multilevel_pc_apply_semantics(ml, gmres):
    """PyAMG PC apply (PyAMG.py:119): x0 = 0, ||b - A x|| <= amg_rtol * ||b|| (pyamg scales its
    tolerance by ||b||), GMRES acceleration unless amg_precondition_with_gmres is off; the
    global random generator is not touched (pyamg's solve draws nothing)."""
    A = ml.problems.poisson_3d_7pt(32)
    n = A.shape[0]
    ml.preconditioner._Options.store.update(
        {"pyamg_amg_rtol": 1e-6, "pyamg_amg_precondition_with_gmres": gmres})
    pc = _PC(A)
    M = ml.preconditioner.MultilevelPC()
    M.initialize(pc)
    assert M.H.n_levels >= 3 and M.amg_precon_gmres is gmres and M.amg_rtol == 1e-6
    b = 1e3 * np.random.RandomState(1).randn(n)
    Y = _Vec(n=n)
    calls = []
    real = M.H.gmres_householder
    M.H.gmres_householder = lambda *a, **kw: calls.append(kw) or real(*a, **kw)
    np.random.seed(5)
    st = np.random.get_state()
    M.apply(pc, _Vec(b), Y)
    assert np.array_equal(np.random.get_state()[1], st[1])
    r = np.linalg.norm(b - A @ Y.out)
    nb = np.linalg.norm(b)
    if gmres:
        # pyamg's budget and stop: krylov.gmres (Householder) without a restart value = one
        # outer cycle of <= 100 steps, stopped when the preconditioned residual
        # ||M r|| < tol ||M b|| (pyamg's left-preconditioned test); the true residual lands
        # near tol ||b||
        assert calls == [{"tol": 1e-6, "maxiter": 100}]
        x, st = M.H.gmres_householder(b, tol=1e-6, maxiter=100, return_info=True)
        assert np.array_equal(x, Y.out) and st["iters"] <= 100 and st["info"] == 0
        Mb = np.linalg.norm(M.H.precondition(b))
        assert st["residuals"][0] == pytest.approx(Mb, rel=1e-12)
        assert st["residuals"][-1] < 1e-6 * Mb
        assert r <= 3e-6 * nb
    else:
        assert calls == []
        assert r <= 1e-6 * nb
    assert r > 1e-9 * nb  # relative, not absolute: no over-solving to 1e-6 abs
    # zero right-hand side: zero solution
    M.apply(pc, _Vec(np.zeros(n)), Y)
    assert not np.any(Y.out)


@pytest.mark.parametrize("name", ("p2d_256", "c3_mesh"))
def test_gmres_matches_scipy_with_oracle_vcycle(ml, oracle, name):
    """Device GMRES (Hierarchy.gmres) vs scipy.sparse.linalg.gmres(A, b, rtol, restart=20,
    M = the oracle's V-cycle on the same hierarchy): the same number of Krylov steps and the same
    preconditioned residual estimates per step within 1e-10 relative + 1e-13 of the first
    (SURVEY.md §8(d) history bound); the iterate to rounding."""
    import os
    import scipy.sparse.linalg as spla
    import torch
    from mlamg import mesh
    from test_gpu_hierarchy import _oracle_levels_from_device
    if name == "p2d_256":
        A = ml.problems.poisson_2d_5pt(256)
    else:
        here = os.path.dirname(os.path.abspath(__file__))
        A = mesh.poisson_dirichlet(mesh.load_npz(os.path.join(here, "golden",
                                                               "cylflow_highres_mesh.npz")))[0]
    n = A.shape[0]
    H = ml.hierarchy.Hierarchy.build(A, alpha=0.1, max_coarse=500)
    lv = _oracle_levels_from_device(H)
    Ac = H.Ac.to_scipy()
    lu = spla.factorized(sp.csc_matrix(Ac))

    def vcycle(r):
        return oracle.vcycle_solve(lv, Ac, np.asarray(r).ravel(), np.zeros(n), 1, lu=lu)[0]

    Mop = spla.LinearOperator((n, n), matvec=vcycle, dtype=np.float64)
    b = np.random.RandomState(7).randn(n)
    for rtol in (1e-6, 1e-10):
        pres = []
        xr, info_r = spla.gmres(A, b, rtol=rtol, restart=20, maxiter=100, M=Mop,
                                callback=pres.append, callback_type="pr_norm")
        x, st = H.gmres(b, rtol=rtol, restart=20, maxiter=100, return_info=True)
        assert st["info"] == info_r == 0
        assert st["inner_iters"] == len(pres), (st["inner_iters"], len(pres))
        pres = np.array(pres)
        assert np.all(np.abs(st["presid"] - pres) <= 1e-10 * pres + 1e-13 * pres[0])
        assert np.linalg.norm(b - A @ x) <= rtol * np.linalg.norm(b)
        assert np.abs(x - xr).max() <= 1e-8 * np.abs(xr).max()
    # torch in -> torch out, and a non-zero initial guess
    xt = H.gmres(torch.as_tensor(b).cuda(), x0=torch.as_tensor(xr).cuda(), rtol=1e-10)
    assert isinstance(xt, torch.Tensor)
    assert np.linalg.norm(b - A @ xt.cpu().numpy()) <= 1e-10 * np.linalg.norm(b)


def test_setup_precondition_solve(ml):
    import torch
    from mlamg import preconditioner
    A = ml.problems.poisson_3d_7pt(24)
    n = A.shape[0]
    b = np.random.RandomState(2).randn(n)
    H = preconditioner.setup(A, alpha=0.1, max_coarse=100)
    # precondition = one V-cycle from a zero guess (numpy in, numpy out; tensor in, tensor out)
    z = preconditioner.precondition(H, b)
    xd = torch.zeros(n, dtype=torch.float64, device="cuda")
    H.cycle(torch.as_tensor(b).cuda(), xd, 1, use_graph=False)
    assert isinstance(z, np.ndarray) and np.array_equal(z, xd.cpu().numpy())
    zt = preconditioner.precondition(H, torch.as_tensor(b).cuda())
    assert isinstance(zt, torch.Tensor) and torch.equal(zt, xd)
    # solve: absolute tolerance on ||b - A x||_2, history returned on request
    x, hist = preconditioner.solve(H, b, tol=1e-9, return_history=True)
    assert hist[-1] <= 1e-9 and np.all(np.diff(hist) < 0)
    assert np.linalg.norm(b - A @ x) <= 1e-9 * 1.0001
    x2 = preconditioner.solve(A, b, tol=1e-9, alpha=0.1, max_coarse=100)
    # deterministic setup (same aggregates, operators); the kernels are re-autotuned, but every
    # candidate sums in scipy's order, so the iterate is bitwise the same
    assert np.array_equal(x2, x)
    # a non-zero initial guess is honoured
    x3, h3 = preconditioner.solve(H, b, x0=x, tol=1e-9, return_history=True)
    assert len(h3) == 1


def test_pc_errors_are_reraised(ml):
    M = ml.preconditioner.MLAMG()
    with pytest.raises(Exception):
        M.initialize(_PC(sp.csr_matrix((3, 4))))  # non-square operator
