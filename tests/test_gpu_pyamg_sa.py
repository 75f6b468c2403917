"""GPU: pyamg's smoothed_aggregation_solver recipe on the device (VERDICT r04 Missing #2).

The reference's PyAMG preconditioner builds `pyamg.aggregation.smoothed_aggregation_solver(P,
max_levels=...)` with pyamg's defaults (ns/preconditioner/PyAMG.py:94) and applies it through
`Amg.solve(b, tol, accel='gmres')` (:119). pyamg is absent here, so parity is unpinned: the device
kernels are checked bitwise against the oracle's restatement of pyamg's amg_core loops
(oracle/oracle.c pyamg_*), which tests/test_oracle_pyamg_sa.py pins to pyamg's own docstring
examples; the V-cycle (dense pinv product on the coarsest level) at rtol 1e-12."""
import numpy as np
import pytest
import scipy.sparse as sp

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch


@pytest.fixture(scope="module")
def ml(torch_cuda):
    import mlamg.graph
    import mlamg.hierarchy
    import mlamg.multigrid
    import mlamg.preconditioner
    import mlamg.problems
    import mlamg.sparse
    return mlamg


def _dev(ml, A):
    return ml.sparse.DeviceCSR.from_scipy(sp.csr_matrix(A))


def _nonsym_pattern(n, seed):
    """A random sparse matrix with a non-symmetric pattern, isolated rows and missing
    diagonals: exercises standard_aggregation's isolated marks and its pass-3 tail."""
    rng = np.random.default_rng(seed)
    M = sp.random(n, n, density=3.0 / n, random_state=rng, format="csr")
    M.data[:] = rng.uniform(-1, 1, M.nnz)
    M = M + sp.diags(rng.uniform(1, 2, n) * (rng.uniform(size=n) < 0.9))
    M = sp.csr_matrix(M)
    M.sort_indices()
    return M


def _long_rows(n, per_row, seed):
    """Symmetric, diagonally dominant, ~per_row entries per row (coarse-Galerkin-like rows; the
    wave-cooperative Gauss-Seidel kernel and its chunk loop past 64 entries)."""
    rng = np.random.default_rng(seed)
    M = sp.random(n, n, density=per_row / (2.0 * n), random_state=rng, format="csr")
    M.data[:] = -rng.uniform(0.1, 1.0, M.nnz)
    M = sp.csr_matrix(M + M.T)
    M = sp.csr_matrix(M + sp.diags(1.0 + np.asarray(abs(M).sum(axis=1)).ravel()))
    M.sort_indices()
    return M


def _matrices(ml):
    P = ml.problems
    return {
        "long_30": _long_rows(2500, 30, 4),
        "long_90": _long_rows(1500, 90, 6),
        "chain_2000": P.poisson_1d(2000),
        "poisson_64": P.poisson_2d_5pt(64),
        "poisson3d_18": P.poisson_3d_7pt(18),
        "randcoef_16": P.random_coeff_3d_7pt(16, seed=3, decades=2.0),
        "nonsym_3000": _nonsym_pattern(3000, 1),
        "doc_isolated": sp.csr_matrix(np.array([[1, 0, 0], [0, 1, 1], [0, 1, 1.0]])),
    }


def _csr_equal(D, S):
    D = D.to_scipy() if hasattr(D, "to_scipy") else D
    return (D.shape == S.shape and np.array_equal(D.indptr, S.indptr)
            and np.array_equal(D.indices, S.indices)
            and np.array_equal(D.data.view(np.int64), S.data.view(np.int64)))


@pytest.mark.parametrize("theta", [0.0, 0.25, 0.5])
def test_symmetric_strength_bitwise(ml, oracle, torch_cuda, theta):
    import ctypes
    from mlamg._lib import call, stream_ptr
    for name, A in _matrices(ml).items():
        h = ctypes.c_void_p()
        Ad = _dev(ml, A)  # kept alive across the call
        call("mlamg_symmetric_strength", Ad.handle, float(theta), ctypes.byref(h), stream_ptr())
        C = ml.sparse.DeviceCSR(h)
        assert _csr_equal(C, oracle.pyamg_symmetric_strength(A, theta)), (name, theta)


def _device_aggregation(ml, torch, C):
    import ctypes
    from mlamg._lib import call, ptr, stream_ptr
    n = C.shape[0]
    dev = torch.device("cuda", 0)
    agg = torch.empty(n, dtype=torch.int32, device=dev)
    cpts = torch.empty(n, dtype=torch.int32, device=dev)
    k, rounds = ctypes.c_int64(), ctypes.c_int32()
    Cd = _dev(ml, C)
    call("mlamg_standard_aggregation", Cd.handle, ptr(agg), ptr(cpts), ctypes.byref(k),
         ctypes.byref(rounds), stream_ptr())
    k = int(k.value)
    return agg.cpu().numpy(), cpts[:k].cpu().numpy(), k, int(rounds.value)


@pytest.mark.parametrize("theta", [0.0, 0.5])
def test_standard_aggregation_bitwise(ml, oracle, torch_cuda, theta):
    """Aggregates, Cpts and count equal amg_core's three sequential passes (the device decides
    pass 1 in parallel rounds) on chains, grids, random coefficients and a non-symmetric pattern
    with isolated rows (pass-3 tail)."""
    for name, A in _matrices(ml).items():
        C = oracle.pyamg_symmetric_strength(A, theta)
        agg_o, cpts_o, k_o = oracle.pyamg_standard_aggregation(C)
        agg_d, cpts_d, k_d, rounds = _device_aggregation(ml, torch_cuda, C)
        assert k_d == k_o, (name, k_d, k_o)
        assert np.array_equal(agg_d, agg_o), name
        assert np.array_equal(cpts_d, cpts_o), name
        assert rounds >= 1


def test_standard_aggregation_doc_examples(ml, torch_cuda):
    """pyamg's standard_aggregation docstring examples."""
    agg, cpts, k, _ = _device_aggregation(ml, torch_cuda, ml.problems.poisson_1d(4))
    assert k == 2 and agg.tolist() == [0, 0, 1, 1] and cpts.tolist() == [0, 3]
    C = sp.csr_matrix(np.array([[1, 0, 0], [0, 1, 1], [0, 1, 1.0]]))
    agg, cpts, k, _ = _device_aggregation(ml, torch_cuda, C)
    assert k == 1 and agg.tolist() == [-1, 0, 0]


@pytest.mark.parametrize("sweep", ["forward", "backward", "symmetric"])
@pytest.mark.parametrize("block", [False, True])
def test_gauss_seidel_directions_bitwise(ml, oracle, torch_cuda, sweep, block):
    """Forward, backward and symmetric sweeps, gauss_seidel and block_gauss_seidel arithmetic,
    on every GS kernel family (small systems take the LDS kernels, larger ones the windowed /
    pipelined / per-level ones)."""
    torch = torch_cuda
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(5)
    mats = dict(_matrices(ml))
    mats["poisson_600"] = ml.problems.poisson_2d_5pt(600)  # 600-row levels: the LDS-ring sweep
    # the ring sweep with zero-diagonal rows (gauss_seidel leaves them alone): stored zeros
    Z = sp.csr_matrix(mats["poisson_600"], copy=True)
    for i in (0, 7, 1234, 180_000, 359_999):
        Z.data[Z.indptr[i]:Z.indptr[i + 1]][Z.indices[Z.indptr[i]:Z.indptr[i + 1]] == i] = 0.0
    mats["poisson_600_zero_diag"] = Z
    # 13 entries a row (12 off-diagonals), couplings up to 19,997 rows apart (6,667 levels of 3
    # rows): the long-row ring sweep (k_gs_wring), with earlier-swept columns beyond its ring
    # horizon (8,192 positions) read back from the level-ordered values
    n = 20_000
    offs = (3, 150, 1001, 3001, 6007, 9001, 15013, 19997)
    O = sp.diags([np.full(n - o, -1.0 / (1 + k)) for k, o in enumerate(offs)], list(offs), (n, n))
    W = sp.csr_matrix(O + O.T + sp.identity(n) * 13.0)
    W.sort_indices()
    mats["offsets_20k"] = W
    W0 = W.copy()
    for i in (5, 10_000, 19_999):
        W0.data[W0.indptr[i]:W0.indptr[i + 1]][W0.indices[W0.indptr[i]:W0.indptr[i + 1]] == i] = 0.0
    mats["offsets_20k_zero_diag"] = W0
    # 37 entries a row: four slots per lane (k_gs_wring in 512-thread workgroups)
    offs2 = offs + (7, 11, 13, 17, 19, 23, 29, 31, 37, 41, 43, 47)
    O2 = sp.diags([np.full(n - o, -1.0 / (1 + k)) for k, o in enumerate(offs2)], list(offs2),
                  (n, n))
    W2 = sp.csr_matrix(O2 + O2.T + sp.identity(n) * 60.0)
    W2.sort_indices()
    mats["offsets_20k_long"] = W2
    for name, A in mats.items():
        if name == "doc_isolated":
            continue
        n = A.shape[0]
        b = rng.standard_normal(n)
        x0 = rng.standard_normal(n)
        G = ml.multigrid.GaussSeidel(_dev(ml, A), sweep, block=block)
        xd = torch.as_tensor(x0).to(dev)
        G.sweep(xd, torch.as_tensor(b).to(dev), 3)
        xo = x0.copy()
        if block:
            oracle.pyamg_block_gauss_seidel(A, xo, b, 3, sweep)
        elif sweep == "forward":
            oracle.gauss_seidel(A, xo, b, 3)
        else:  # gauss_seidel arithmetic backward / symmetric (zero diagonals: x_i kept)
            oracle.pyamg_gauss_seidel(A, xo, b, 3, sweep)
        assert np.array_equal(xd.cpu().numpy().view(np.int64), xo.view(np.int64)), (name, sweep)


def test_fit_candidates_and_csr_sub_bitwise(ml, oracle, torch_cuda):
    import ctypes
    from mlamg._lib import call, ptr, stream_ptr
    torch = torch_cuda
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(2)
    for name, A in _matrices(ml).items():
        C = oracle.pyamg_symmetric_strength(A, 0.0)
        agg, _, k = oracle.pyamg_standard_aggregation(C)
        B = rng.uniform(0.5, 2.0, A.shape[0])
        if name == "poisson_64":
            B[:7] = 0.0  # an all-zero aggregate: scale 0, R 0
        Agg = ml.graph.aggregate_op_device(torch.as_tensor(agg).to(dev), k)
        h = ctypes.c_void_p()
        Bc = torch.empty(k, dtype=torch.float64, device=dev)
        Bd = torch.as_tensor(B).to(dev)
        call("mlamg_fit_candidates", Agg.handle, ptr(Bd), 1e-10, ctypes.byref(h), ptr(Bc),
             stream_ptr())
        T = ml.sparse.DeviceCSR(h)
        To, Bco = oracle.pyamg_fit_candidates(agg, k, B)
        assert _csr_equal(T, To), name
        assert np.array_equal(Bc.cpu().numpy().view(np.int64), Bco.view(np.int64)), name
        # P = T - M with M = (scaled D^-1 A) @ T: scipy's binop, zeros dropped, columns sorted
        M = sp.csr_matrix(A) @ To
        h = ctypes.c_void_p()
        Md = _dev(ml, A) @ T
        call("mlamg_csr_sub", T.handle, Md.handle, ctypes.byref(h), stream_ptr())
        P = sp.csr_matrix(To - M)
        P.sort_indices()
        assert _csr_equal(ml.sparse.DeviceCSR(h), P), name


@pytest.mark.parametrize("case", ["poisson_64", "poisson3d_18", "randcoef_16"])
def test_pyamg_sa_hierarchy_and_cycle(ml, oracle, torch_cuda, case):
    """Every level's strength, aggregates, improved candidate, T, P and A_c are bitwise the
    oracle's restatement of smoothed_aggregation_solver (given the device's rho per level); one
    V-cycle (symmetric block GS, dense pinv product at the coarsest level) within 1e-12."""
    torch = torch_cuda
    A = sp.csr_matrix(_matrices(ml)[case])
    H = ml.hierarchy.Hierarchy.pyamg_sa(A)
    rhos = [L.lam for L in H.levels]
    levels, Ac = oracle.pyamg_sa_setup(A, rhos=rhos)
    assert len(levels) == len(H.levels) >= 2
    assert Ac.shape[0] <= 10 < levels[-1]["A"].shape[0]
    for i, (Ld, Lo) in enumerate(zip(H.levels, levels)):
        assert _csr_equal(Ld.A, Lo["A"]), (case, i)
        assert Ld.n_seeds == Lo["k"]
        assert np.array_equal(Ld.agg_col.cpu().numpy(), Lo["agg"]), (case, i)
        assert np.array_equal(Ld.B.cpu().numpy().view(np.int64), Lo["B"].view(np.int64)), i
        assert _csr_equal(Ld.P, Lo["P"]), (case, i)
        assert _csr_equal(Ld.R, Lo["R"]), (case, i)
    assert _csr_equal(H.Ac, Ac)
    rng = np.random.default_rng(7)
    b = rng.standard_normal(A.shape[0])
    dev = torch.device("cuda", 0)
    xd = torch.zeros(A.shape[0], dtype=torch.float64, device=dev)
    H.cycle(torch.as_tensor(b).to(dev), xd, 1, history=False)
    import scipy.linalg
    xo = oracle.pyamg_sa_vcycle(levels, scipy.linalg.pinv(Ac.toarray()), b, np.zeros_like(b))
    np.testing.assert_allclose(xd.cpu().numpy(), xo, rtol=1e-12, atol=1e-12 * np.abs(xo).max())
    # a convergent preconditioner: stationary cycles reduce the residual every cycle (the
    # 2-decade random-coefficient case slowly: theta = 0 strength, as pyamg's default)
    x = np.zeros_like(b)
    hist = H.cycle(torch.as_tensor(b).to(dev), torch.as_tensor(x).to(dev), 12)
    assert (np.diff(hist) < 0).all()
    assert hist[-1] < (1e-3 if case.startswith("poisson") else 0.1) * np.linalg.norm(b)


def test_factored_prolong_refused_on_pyamg_recipe(ml, torch_cuda):
    """pyamg's P = T - (omega/rho) D^-1 A T smooths the normalised candidate T, not the 0/1
    aggregate operator, so the factored form x += t - w D^-1 A t (t = Agg e) of
    Hierarchy.set_factored_prolong would be another prolongator: the call is refused
    (EUNSUPPORTED) and the cycle keeps pyamg's explicit P, bit for bit."""
    torch = torch_cuda
    from mlamg._lib import MLAMG_EUNSUPPORTED, MlamgError
    A = sp.csr_matrix(_matrices(ml)["poisson3d_18"])
    H = ml.hierarchy.Hierarchy.pyamg_sa(A)
    assert H.recipe == "pyamg_sa" and H.levels[0].agg_col is not None
    b = torch.as_tensor(np.random.default_rng(3).standard_normal(A.shape[0])).cuda()
    x1 = torch.zeros_like(b)
    h1 = H.cycle(b, x1, 3)
    with pytest.raises(MlamgError) as e:
        H.set_factored_prolong(0)
    assert e.value.code == MLAMG_EUNSUPPORTED
    x2 = torch.zeros_like(b)
    h2 = H.cycle(b, x2, 3)
    assert np.array_equal(h1, h2) and torch.equal(x1, x2)
    # the Bellman-Ford SA recipe (P = (I - w D^-1 A) Agg) still takes it
    Hb = ml.hierarchy.Hierarchy.build(ml.problems.poisson_3d_7pt(24), alpha=0.1, max_coarse=300)
    assert Hb.recipe == "mlamg_sa" and Hb.levels[0].sa_prolong
    Hb.set_factored_prolong(0)
    Hb.set_factored_prolong(0, on=False)


def test_multilevel_pc_uses_pyamg_recipe(ml, torch_cuda):
    """The PyAMG PC (PyAMG.py:13-130) builds pyamg's recipe by default and its GMRES apply meets
    the amg_rtol stop (1e-8 relative); 'mlamg_sa' selects the Bellman-Ford SA recipe."""
    A = ml.problems.poisson_2d_5pt(96)

    class PC:
        def getOperators(self):
            return None, A

        def getOptionsPrefix(self):
            return ""

    pc = ml.preconditioner.MultilevelPC()
    pc.initialize(PC())
    assert pc.H.recipe == "pyamg_sa"
    b = np.random.default_rng(0).standard_normal(A.shape[0])
    y = np.zeros_like(b)
    pc.apply(PC(), b, y)
    # Householder GMRES (pyamg's default) stops on ||M r|| < 1e-8 ||M b||: the true residual
    # lands near that
    assert np.linalg.norm(b - A @ y) <= 1e-7 * np.linalg.norm(b)
    ml.preconditioner._Options.store["pyamg_amg_gmres_orthog"] = "mgs"
    try:
        pc1 = ml.preconditioner.MultilevelPC()
        pc1.initialize(PC())
        y1 = np.zeros_like(b)
        pc1.apply(PC(), b, y1)
        assert np.linalg.norm(b - A @ y1) <= 1e-7 * np.linalg.norm(b)
    finally:
        ml.preconditioner._Options.store.pop("pyamg_amg_gmres_orthog", None)
    ml.preconditioner._Options.store["pyamg_amg_recipe"] = "mlamg_sa"
    try:
        pc2 = ml.preconditioner.MultilevelPC()
        pc2.initialize(PC())
        assert getattr(pc2.H, "recipe", None) != "pyamg_sa"
    finally:
        ml.preconditioner._Options.store.pop("pyamg_amg_recipe", None)


def test_pyamg_compat_solver_api(ml, oracle, torch_cuda):
    """`pyamg.aggregation.smoothed_aggregation_solver(P, max_levels=10)` under the compat alias
    (what ns/preconditioner/PyAMG.py:94 calls) and the MultilevelSolver calls of :119 and :129:
    solve with accel='gmres' and None, residuals, repr; the pieces under pyamg's names."""
    import scipy.sparse.linalg as spla
    from mlamg.pyamg_compat import aggregation, relaxation, strength
    A = ml.problems.poisson_2d_5pt(80)
    ml_solver = aggregation.smoothed_aggregation_solver(A, max_levels=10)
    text = repr(ml_solver)
    assert "MultilevelSolver" in text and "Number of Levels" in text
    assert len(ml_solver.levels) == ml_solver.H.n_levels and ml_solver.levels[-1].A.shape[0] <= 10
    assert 1.0 < ml_solver.operator_complexity() < 2.0
    b = np.random.default_rng(3).standard_normal(A.shape[0])
    res = []
    x = ml_solver.solve(b, tol=1e-8, accel="gmres", residuals=res)
    assert np.linalg.norm(b - A @ x) <= 1e-6 * np.linalg.norm(b) and len(res) >= 2
    res = []
    x, info = ml_solver.solve(b, tol=1e-8, residuals=res, return_info=True)
    assert info == 0 and res[-1] <= 1e-8 * np.linalg.norm(b) and res[0] == pytest.approx(
        np.linalg.norm(b))
    assert np.linalg.norm(b - A @ x) <= 1.01e-8 * np.linalg.norm(b)
    M = ml_solver.aspreconditioner()
    xs, code = spla.cg(A, b, rtol=1e-8, M=M)
    assert code == 0
    # the pieces
    C = strength.symmetric_strength_of_connection(A, 0.25)
    Co = oracle.pyamg_symmetric_strength(A, 0.25)
    assert np.array_equal(C.indices, Co.indices) and np.array_equal(C.data, Co.data)
    AggOp, Cpts = aggregation.standard_aggregation(C)
    agg_o, cpts_o, k_o = oracle.pyamg_standard_aggregation(Co)
    assert AggOp.shape == (A.shape[0], k_o) and np.array_equal(Cpts, cpts_o)
    assert np.array_equal(AggOp.indices, agg_o[agg_o >= 0])
    Q, R = aggregation.fit_candidates(AggOp, np.ones((A.shape[0], 1)))
    To, Bco = oracle.pyamg_fit_candidates(agg_o, k_o, np.ones(A.shape[0]))
    assert np.array_equal(Q.data, To.data) and np.array_equal(R.ravel(), Bco)
    xr = np.random.default_rng(4).standard_normal(A.shape[0])
    xo = xr.copy()
    relaxation.relaxation.block_gauss_seidel(A, xr, b, iterations=2, sweep="symmetric")
    oracle.pyamg_block_gauss_seidel(A, xo, b, 2, "symmetric")
    assert np.array_equal(xr, xo)
    with pytest.raises(NotImplementedError):
        aggregation.smoothed_aggregation_solver(A, aggregate="lloyd")


def test_pyamg_sa_edge_cases(ml, torch_cuda):
    """n <= max_coarse: no level, the solve is the pinv product (pyamg: len(levels) == 1), also
    for a singular (pure Neumann) operator (the minimum-norm solution); x0 given; max_levels=1
    and 2."""
    from mlamg.pyamg_compat import aggregation
    A = ml.problems.poisson_1d(8)
    s = aggregation.smoothed_aggregation_solver(A)
    assert s.H.n_levels == 1
    b = np.arange(1.0, 9.0)
    x = s.solve(b, tol=1e-12)
    np.testing.assert_allclose(A @ x, b, rtol=0, atol=1e-12 * np.abs(b).max() * 100)
    # singular (Neumann) coarse operator: the pinv coarse solve gives the minimum-norm solution
    n = 8
    N = sp.diags([-np.ones(n - 1), 2 * np.ones(n), -np.ones(n - 1)], [-1, 0, 1]).tolil()
    N[0, 0] = N[n - 1, n - 1] = 1.0
    N = sp.csr_matrix(N)
    rhs = np.sin(np.linspace(0, 2 * np.pi, n))
    rhs -= rhs.mean()
    xn = aggregation.smoothed_aggregation_solver(N).solve(rhs, tol=1e-12)
    np.testing.assert_allclose(N @ xn, rhs, atol=1e-12)
    assert abs(xn.sum()) < 1e-12
    for lv in (1, 2):
        s2 = aggregation.smoothed_aggregation_solver(ml.problems.poisson_2d_5pt(12), max_levels=lv)
        assert s2.H.n_levels == lv
    # no off-diagonal couplings (n > max_coarse): pyamg's n x 1 empty AggOp, a zero coarse
    # correction; the symmetric sweep alone solves the diagonal system
    d = np.linspace(1.0, 3.0, 50)
    sd = aggregation.smoothed_aggregation_solver(sp.diags(d).tocsr())
    assert sd.H.n_levels == 2 and sd.H.Ac.shape == (1, 1)
    assert sd.H.levels[0].P.shape == (50, 1) and sd.H.levels[0].P.nnz == 0
    bd = np.arange(1.0, 51.0)
    np.testing.assert_allclose(sd.solve(bd, tol=1e-12), bd / d, rtol=1e-15)
    P = ml.problems.poisson_2d_5pt(40)
    s3 = aggregation.smoothed_aggregation_solver(P)
    b3 = np.ones(P.shape[0])
    x1 = s3.solve(b3, tol=1e-6, maxiter=3)
    x2 = s3.solve(b3, x0=x1, tol=1e-10, maxiter=50)
    assert np.linalg.norm(b3 - P @ x2) <= 1e-10 * np.linalg.norm(b3)


@pytest.mark.parametrize("case", ["poisson_64", "randcoef_16"])
def test_gmres_householder_matches_oracle(ml, oracle, torch_cuda, case):
    """pyamg.krylov.gmres (orthog='householder', restrt=None) preconditioned by one V-cycle of
    the pyamg_sa hierarchy (Hierarchy.gmres_householder) against oracle/restated.py's numpy
    restatement driven by the oracle's own V-cycle: the same step count, info code and
    preconditioned-residual history (rtol 1e-6, atol 1e-10 ||M b||: fixed-order tree dots and
    a V-cycle equal to 1e-12 vs numpy's), x within
    1e-7 relative; the MGS GMRES (scipy's algorithm) takes the same number of steps +-1."""
    import scipy.linalg
    A = sp.csr_matrix(_matrices(ml)[case])
    H = ml.hierarchy.Hierarchy.pyamg_sa(A)
    levels, Ac = oracle.pyamg_sa_setup(A, rhos=[L.lam for L in H.levels])
    pinv = scipy.linalg.pinv(Ac.toarray())

    def M(r):
        return oracle.pyamg_sa_vcycle(levels, pinv, np.ascontiguousarray(r), np.zeros_like(r))

    b = np.random.default_rng(11).standard_normal(A.shape[0])
    for tol, maxiter in ((1e-8, 100), (1e-8, 3), (1e-5, None)):
        x, info = H.gmres_householder(b, tol=tol, maxiter=maxiter, return_info=True)
        xo, info_o, it_o, res_o = oracle.pyamg_gmres_householder(A, b, M, tol=tol,
                                                                 maxiter=maxiter)
        assert info["iters"] == it_o and info["info"] == info_o, (case, tol, maxiter)
        assert len(info["residuals"]) == len(res_o)
        np.testing.assert_allclose(info["residuals"], res_o, rtol=1e-6, atol=1e-10 * res_o[0])
        np.testing.assert_allclose(x, xo, rtol=0, atol=1e-7 * np.abs(xo).max())
    x, info = H.gmres_householder(b, tol=1e-8, maxiter=100, return_info=True)
    assert info["info"] == 0 and info["residuals"][-1] < 1e-8 * info["residuals"][0]
    _, mg = H.gmres(b, rtol=1e-8, restart=100, maxiter=1, return_info=True)
    assert abs(mg["inner_iters"] - info["iters"]) <= 1


def test_gmres_householder_edge_cases(ml, oracle, torch_cuda):
    """b = 0 (||b|| counts as 1: x stays 0, no step), x0 already the solution (no step), the
    exact preconditioner of an n <= max_coarse operator (the pinv coarse solve alone: one step,
    a lucky breakdown with a zero reflector tail), maxiter > n (clamped to n), a tensor in."""
    torch = torch_cuda
    A = ml.problems.poisson_2d_5pt(24)
    H = ml.hierarchy.Hierarchy.pyamg_sa(A)
    z = np.zeros(A.shape[0])
    x, info = H.gmres_householder(z, return_info=True)
    assert not x.any() and info["iters"] == 0 and info["info"] == 0
    assert len(info["residuals"]) == 1
    b = np.random.default_rng(2).standard_normal(A.shape[0])
    xs = H.gmres_householder(b, tol=1e-12, maxiter=200)
    x, info = H.gmres_householder(b, x0=xs, tol=1e-2, return_info=True)
    assert info["iters"] == 0 and np.array_equal(x, xs)
    # n = 8 <= max_coarse: M is the pinv of A itself
    A1 = ml.problems.poisson_1d(8)
    H1 = ml.hierarchy.Hierarchy.pyamg_sa(A1)
    assert H1.n_levels == 1
    b1 = np.arange(1.0, 9.0)
    x1, info1 = H1.gmres_householder(b1, tol=1e-10, maxiter=100, return_info=True)
    assert info1["iters"] == 1 and info1["info"] == 0
    # pyamg breaks before recording the converged step's estimate: initial and final norms only
    assert len(info1["residuals"]) == 2
    np.testing.assert_allclose(A1 @ x1, b1, atol=1e-12 * 8)
    Minv = np.linalg.pinv(A1.toarray())
    xo, info_o, it_o, _ = oracle.pyamg_gmres_householder(A1, b1, lambda r: Minv @ r, tol=1e-10,
                                                        maxiter=100)
    assert it_o == 1 and info_o == 0
    np.testing.assert_allclose(x1, xo, rtol=1e-12)
    bt = torch.as_tensor(b, device="cuda:0")
    xt = H.gmres_householder(bt, tol=1e-8)
    assert isinstance(xt, torch.Tensor) and xt.is_cuda
    assert np.linalg.norm(b - A @ xt.cpu().numpy()) <= 1e-6 * np.linalg.norm(b)
