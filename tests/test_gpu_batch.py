"""GPU: many independent reference-style amg_2_v solves at once (mlamg.multigrid.amg_2_v_batch —
the reference's per-grid task farm, ns/parallel/pool.py): one fused launch for the whole batch
(csrc/batch.hip, a workgroup per problem), or host threads with one HIP stream each over the
hierarchy engine. Every result must equal the sequential call of the same engine bit for bit,
and both engines match the oracle within the stated fp64 tolerances."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _problems(ml, oracle, count):
    out = []
    for i in range(count):
        m = 24 + 4 * (i % 7)
        A = ml.problems.poisson_2d_5pt(m)
        Agg = ml.problems.box_aggregates_2d(m, m, 3 if i % 2 else 2)
        P, _ = oracle.smoothed_aggregation_jacobi(A, Agg, omega=2.0 / 3.0)
        x0 = np.random.RandomState(i).randn(A.shape[0])
        b = np.random.RandomState(100 + i).randn(A.shape[0]) if i % 3 == 0 else np.zeros(A.shape[0])
        out.append((A, P, b, x0))
    return out


@pytest.mark.parametrize("ext", (False, True))
@pytest.mark.parametrize("smoother", ("gauss_seidel", "jacobi"))
def test_batch_equals_sequential(oracle, smoother, ext, monkeypatch):
    """Every problem of a batch equals its own single call bit for bit. ext=True (the default
    engine): problems with n_c > 300 take the device-wide coarse factor both alone and in the
    batch (the batch then runs phased; the others keep the one-workgroup factor, chosen by their
    own n_c); ext=False: everything on the one-workgroup path."""
    if not ext:
        monkeypatch.setenv("MLAMG_BATCH_NO_EXT", "1")
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mlamg.multigrid
    import mlamg.problems
    import mlamg as ml
    probs = _problems(ml, oracle, 14)
    # the batch runs every problem through the fused kernel (n_c <= FUSED_BATCH_MAX_NC); single
    # calls pick their engine by size, so they are asked for the fused one explicitly
    seq = [ml.multigrid.amg_2_v(A, P, b, x.copy(), res_tol=1e-10, smoother=smoother,
                                engine="fused") for A, P, b, x in probs]
    bat = ml.multigrid.amg_2_v_batch([(A, P, b, x.copy()) for A, P, b, x in probs], workers=6,
                                     res_tol=1e-10, smoother=smoother)
    assert len(bat) == len(seq)
    for i, ((xs, cs, es, its), (xb, cb, eb, itb)) in enumerate(zip(seq, bat)):
        assert its == itb and np.array_equal(es, eb), i
        assert np.array_equal(xs, xb), i
        assert cs == cb or (np.isnan(cs) and np.isnan(cb)), i


@pytest.mark.parametrize("smoother", ("gauss_seidel", "jacobi"))
def test_threaded_engine_equals_sequential(oracle, smoother):
    """The per-problem (hierarchy) engine of amg_2_v_batch: host threads, one stream each."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mlamg.multigrid
    import mlamg.problems
    import mlamg as ml
    probs = _problems(ml, oracle, 8)
    seq = [ml.multigrid.amg_2_v(A, P, b, x.copy(), res_tol=1e-10, smoother=smoother,
                                engine="hierarchy") for A, P, b, x in probs]
    bat = ml.multigrid.amg_2_v_batch([(A, P, b, x.copy()) for A, P, b, x in probs], workers=4,
                                     res_tol=1e-10, smoother=smoother, engine="hierarchy")
    for i, ((xs, cs, es, its), (xb, cb, eb, itb)) in enumerate(zip(seq, bat)):
        assert its == itb and np.array_equal(es, eb) and np.array_equal(xs, xb), i


@pytest.mark.parametrize("smoother", ("gauss_seidel", "jacobi"))
@pytest.mark.parametrize("mode", ("res", "err"))
def test_fused_matches_oracle_and_hierarchy(oracle, smoother, mode):
    """The fused one-launch solver (csrc/batch.hip) vs the oracle's amg_2_v (SuperLU coarse
    solve) and vs the per-operation hierarchy engine: same iteration counts, histories within
    rtol 1e-10 (Galerkin + dense inverse vs scipy + SuperLU: rounding only), conv factors within
    1e-8, iterates within 1e-9 of their max. Smoothing/restriction/prolongation are bitwise
    scipy's, so any larger deviation is a bug, not rounding."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mlamg.multigrid
    import mlamg.problems
    import mlamg as ml
    kw = {"res_tol": 1e-10} if mode == "res" else {"error_tol": 1e-8}
    for m, agg in ((17, 3), (40, 3), (64, 2), (90, 3)):
        A = ml.problems.poisson_2d_5pt(m)
        P, _ = oracle.smoothed_aggregation_jacobi(A, ml.problems.box_aggregates_2d(m, m, agg),
                                                  omega=2.0 / 3.0)
        x0 = np.random.RandomState(m).randn(A.shape[0])
        x0 /= np.linalg.norm(x0)
        # b = 0 (the reference's evaluation loops, utils/common.py:48): x -> 0, so the history
        # keeps its relative accuracy down to the tolerance; with b != 0 the residual's rounding
        # floor eps*|A||x| is reached near res_tol and the tail is not comparable to 1e-10
        b = np.zeros(A.shape[0])
        xr, cr, er, ir = oracle.amg_2_v(A, P, b, x0, smoother=smoother, jacobi_weight=0.666,
                                        max_iter=200, **kw)
        xf, cf, ef, itf = ml.multigrid.amg_2_v(A, P, b, x0, smoother=smoother, max_iter=200,
                                               engine="fused", **kw)
        xh, ch, eh, ith = ml.multigrid.amg_2_v(A, P, b, x0, smoother=smoother, max_iter=200,
                                               engine="hierarchy", **kw)
        assert itf == ir == ith, (m, itf, ir, ith)
        for e in (ef, eh):
            assert np.allclose(e, er, rtol=1e-10, atol=1e-14 * er[0]), (m, e, er)
        assert abs(cf - cr) <= 1e-8 and abs(ch - cr) <= 1e-8
        scale = max(np.abs(xr).max(), 1e-300)
        assert np.abs(xf - xr).max() <= 1e-9 * scale + 1e-14
        assert np.abs(xf - xh).max() <= 1e-9 * scale + 1e-14
    # a nonzero right-hand side: the solution itself (x -> A^-1 b = xs) agrees
    m = 48
    A = ml.problems.poisson_2d_5pt(m)
    P, _ = oracle.smoothed_aggregation_jacobi(A, ml.problems.box_aggregates_2d(m, m, 3),
                                              omega=2.0 / 3.0)
    xs = np.random.RandomState(1).randn(A.shape[0])
    x0 = np.zeros(A.shape[0])
    xr, cr, er, ir = oracle.amg_2_v(A, P, A @ xs, x0, smoother=smoother, max_iter=60, **kw)
    xf, cf, ef, itf = ml.multigrid.amg_2_v(A, P, A @ xs, x0, smoother=smoother, max_iter=60,
                                           engine="fused", **kw)
    assert np.abs(xf - xr).max() <= 1e-9 * np.abs(xs).max()
    assert np.allclose(ef[:10], er[:10], rtol=1e-10, atol=0)


def test_fused_batch_mixed_sizes_bitwise_single(oracle, monkeypatch):
    """One launch over problems of different sizes equals one launch per problem, bit for bit
    (each workgroup owns its problem; single calls held to the one-workgroup coarse factor)."""
    monkeypatch.setenv("MLAMG_BATCH_NO_EXT", "1")
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mlamg.multigrid
    import mlamg.problems
    import mlamg as ml
    probs = _problems(ml, oracle, 21)
    one = [ml.multigrid.amg_2_v(A, P, b, x, res_tol=1e-10, engine="fused") for A, P, b, x in probs]
    bat = ml.multigrid.amg_2_v_batch(probs, res_tol=1e-10)
    for i, (a, c) in enumerate(zip(one, bat)):
        assert a[3] == c[3] and np.array_equal(a[2], c[2]) and np.array_equal(a[0], c[0]), i


@pytest.mark.parametrize("smoother", ("gauss_seidel", "jacobi"))
def test_shared_shapes_values_differ(oracle, monkeypatch, smoother):
    """Problems with one sparsity pattern and different values (Voronoi jump coefficients, a
    value-nonsymmetric A on a symmetric pattern, a zero diagonal entry, separate or shared index
    arrays): the batch analyses each pattern once and gathers every problem's values on the
    device. Results equal one call per problem bit for bit, on a first call (patterns analysed),
    a second (patterns from the cache) and with the cache off."""
    monkeypatch.setenv("MLAMG_BATCH_NO_EXT", "1")
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import scipy.sparse as sp
    import mlamg.multigrid
    import mlamg as ml
    probs = []
    for i in range(12):
        m = (30, 37)[i % 2]
        A = ml.problems.jump_2d(m, ml.problems.voronoi_jumps(np.random.RandomState(i)))
        if i % 4 == 1:  # same pattern, values no longer symmetric: Gauss-Jordan coarse inverse
            A = A.copy()
            A.data[A.indptr[5] + 1] *= 1.5
        if i == 6 and smoother == "gauss_seidel":  # a zero diagonal: the sweep skips the row
            A = A.copy()
            A.data[(A.indices == 7) & (np.repeat(np.arange(A.shape[0]), np.diff(A.indptr)) == 7)] = 0.0
        if i % 3 == 2:  # shares its index arrays with the previous problem of its size
            B = probs[i - 2][0]
            A = sp.csr_matrix((A.data.copy(), B.indices, B.indptr), shape=A.shape)
        Agg = ml.problems.box_aggregates_2d(m, m, 3)
        P, _ = oracle.smoothed_aggregation_jacobi(ml.problems.poisson_2d_5pt(m), Agg,
                                                  omega=2.0 / 3.0)
        x0 = np.random.RandomState(50 + i).randn(A.shape[0])
        probs.append((A, P, np.zeros(A.shape[0]), x0))
    one = [ml.multigrid.amg_2_v(A, P, b, x, res_tol=1e-10, smoother=smoother, engine="fused",
                                max_iter=60) for A, P, b, x in probs]
    runs = [ml.multigrid.amg_2_v_batch(probs, res_tol=1e-10, smoother=smoother, max_iter=60),
            ml.multigrid.amg_2_v_batch(probs, res_tol=1e-10, smoother=smoother, max_iter=60)]
    monkeypatch.setenv("MLAMG_BATCH_NO_SHAPE_CACHE", "1")
    runs.append(ml.multigrid.amg_2_v_batch(probs, res_tol=1e-10, smoother=smoother, max_iter=60))
    for r, bat in enumerate(runs):
        for i, (a, c) in enumerate(zip(one, bat)):
            assert a[3] == c[3] and np.array_equal(a[2], c[2]), (r, i)
            assert np.array_equal(a[0], c[0]), (r, i)
    # and the values matter: two problems of one pattern converge differently
    assert not np.array_equal(one[0][2], one[2][2])


@pytest.mark.parametrize("smoother", ("gauss_seidel", "jacobi"))
def test_band_coarse_solve(oracle, monkeypatch, smoother):
    """Narrow-banded coarse operators (aggregates numbered along the grid: half-bandwidth
    kx + 1 <= 63) take the banded Cholesky factor and band substitutions: the same iteration
    counts as the dense coarse inverse (MLAMG_BATCH_NO_BAND) and as the oracle (SuperLU), and
    histories within fp64 rounding of both. Permuted aggregate numbers (wide band) keep the
    dense path; a symmetric indefinite A (the band factor meets a negative pivot) falls back
    to Gauss-Jordan, bitwise the dense path's fallback."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import scipy.sparse as sp
    import mlamg.multigrid
    import mlamg as ml
    cases = []
    for m, box, perm in ((20, 2, False), (45, 3, False), (64, 3, False), (96, 3, False),
                         (40, 3, True)):
        A = ml.problems.poisson_2d_5pt(m)
        Agg = ml.problems.box_aggregates_2d(m, m, box)
        if perm:
            Agg = sp.csr_matrix(Agg[:, np.random.RandomState(m).permutation(Agg.shape[1])])
        P, _ = oracle.smoothed_aggregation_jacobi(A, Agg, omega=2.0 / 3.0)
        x0 = np.random.RandomState(m).randn(A.shape[0])
        cases.append((A, P, np.zeros(A.shape[0]), x0 / np.linalg.norm(x0)))
    kw = dict(res_tol=1e-10, smoother=smoother, max_iter=100)
    band = [ml.multigrid.amg_2_v(*c, engine="fused", **kw) for c in cases]
    bat = ml.multigrid.amg_2_v_batch(cases, **kw)
    monkeypatch.setenv("MLAMG_BATCH_NO_BAND", "1")
    dense = [ml.multigrid.amg_2_v(*c, engine="fused", **kw) for c in cases]
    monkeypatch.delenv("MLAMG_BATCH_NO_BAND")
    for i, c in enumerate(cases):
        xr, cr, er, ir = oracle.amg_2_v(*c, jacobi_weight=0.666, **kw)
        assert band[i][3] == dense[i][3] == ir, (i, band[i][3], dense[i][3], ir)
        assert np.allclose(band[i][2], er, rtol=1e-10, atol=1e-14 * er[0]), i
        assert np.allclose(band[i][2], dense[i][2], rtol=1e-10, atol=1e-14 * er[0]), i
        scale = np.abs(xr).max()
        assert np.abs(band[i][0] - xr).max() <= 1e-9 * scale + 1e-14, i
        # the batch is bitwise its single calls
        assert bat[i][3] == band[i][3] and np.array_equal(bat[i][2], band[i][2]), i
        assert np.array_equal(bat[i][0], band[i][0]), i
    # symmetric indefinite: the band factor fails, Gauss-Jordan takes over (both paths alike)
    A = (ml.problems.poisson_2d_5pt(30) - 1.0 * sp.eye(900)).tocsr()
    A.sort_indices()
    P, _ = oracle.smoothed_aggregation_jacobi(ml.problems.poisson_2d_5pt(30),
                                              ml.problems.box_aggregates_2d(30, 30, 3),
                                              omega=2.0 / 3.0)
    c = (A, P, np.zeros(900), np.random.RandomState(1).randn(900))
    kw2 = dict(res_tol=1e-10, smoother=smoother, max_iter=20)
    a = ml.multigrid.amg_2_v(*c, engine="fused", **kw2)
    monkeypatch.setenv("MLAMG_BATCH_NO_BAND", "1")
    d = ml.multigrid.amg_2_v(*c, engine="fused", **kw2)
    assert a[3] == d[3] and np.array_equal(a[2], d[2], equal_nan=True)
    assert np.array_equal(a[0], d[0], equal_nan=True)


def test_fused_edge_cases(oracle):
    """Singular Galerkin operator -> (x, 1.0, zeros, 0) like the reference's failed
    factorisation (multigrid.py:167-170); max_iter 0 and 1 (conv-factor quirks); a row with more
    than 32 off-diagonals falls back to the hierarchy engine with the same results."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import scipy.sparse as sp
    import mlamg.multigrid
    import mlamg.problems
    import mlamg as ml
    m = 20
    A = ml.problems.poisson_2d_5pt(m)
    Agg = ml.problems.box_aggregates_2d(m, m, 4)
    P = sp.hstack([sp.csr_matrix(Agg, dtype=np.float64),
                   sp.csr_matrix((A.shape[0], 1))]).tocsr()     # an empty coarse column
    x0 = np.random.RandomState(0).randn(A.shape[0])
    x, c, e, it = ml.multigrid.amg_2_v(A, P, np.zeros(A.shape[0]), x0, res_tol=1e-10)
    xr, cr, er, ir = oracle.amg_2_v(A, P, np.zeros(A.shape[0]), x0, res_tol=1e-10)
    assert (it, c) == (ir, cr) == (0, 1.0) and np.array_equal(x, x0) and not np.any(e)
    P2, _ = oracle.smoothed_aggregation_jacobi(A, Agg, omega=2.0 / 3.0)
    for mi in (0, 1, 2):
        got = ml.multigrid.amg_2_v(A, P2, np.zeros(A.shape[0]), x0, res_tol=1e-300, max_iter=mi)
        ref = oracle.amg_2_v(A, P2, np.zeros(A.shape[0]), x0, res_tol=1e-300, max_iter=mi)
        assert got[3] == ref[3] == mi and len(got[2]) == mi
        assert np.allclose(got[1], ref[1], rtol=1e-10, atol=0)
    # a dense-ish operator: 40 off-diagonals per row -> hierarchy engine (same answers)
    rs = np.random.RandomState(5)
    n = 300
    B = sp.random(n, n, density=40 / n, random_state=rs, format="csr")
    Ad = (B + B.T + sp.diags(np.full(n, 100.0))).tocsr()
    Pd, _ = oracle.smoothed_aggregation_jacobi(
        Ad, sp.csr_matrix((np.ones(n), (np.arange(n), np.arange(n) // 5))), omega=2.0 / 3.0)
    xa = ml.multigrid.amg_2_v(Ad, Pd, np.zeros(n), x0[:n], res_tol=1e-10)
    xb = ml.multigrid.amg_2_v(Ad, Pd, np.zeros(n), x0[:n], res_tol=1e-10, engine="hierarchy")
    assert xa[3] == xb[3] and np.array_equal(xa[2], xb[2])


def test_fused_zero_diagonal_rows(oracle):
    """Rows whose stored diagonal is 0.0: pyamg's sweep leaves x_i alone (the one-wave sweep
    sends them to its sink slot), and the operator is no longer SPD, so the coarse solve takes
    the Gauss-Jordan fallback. Histories vs the oracle (SuperLU coarse solve)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mlamg.multigrid
    import mlamg.problems
    import mlamg as ml
    m = 24
    A0 = ml.problems.poisson_2d_5pt(m)
    P, _ = oracle.smoothed_aggregation_jacobi(A0, ml.problems.box_aggregates_2d(m, m, 3),
                                              omega=2.0 / 3.0)
    A = A0.copy()
    for i in (0, 37, 300, m * m - 1):
        lo, hi = A.indptr[i], A.indptr[i + 1]
        A.data[lo + np.flatnonzero(A.indices[lo:hi] == i)] = 0.0
    x0 = np.random.RandomState(11).randn(A.shape[0])
    b = np.random.RandomState(12).randn(A.shape[0])
    xr, cr, er, ir = oracle.amg_2_v(A, P, b, x0, res_tol=1e-300, max_iter=8)
    xf, cf, ef, itf = ml.multigrid.amg_2_v(A, P, b, x0, res_tol=1e-300, max_iter=8,
                                           engine="fused")
    assert itf == ir == 8
    assert np.allclose(ef, er, rtol=1e-10, atol=0), (ef, er)
    assert np.abs(xf - xr).max() <= 1e-9 * np.abs(xr).max()


def test_fused_wide_coarse(oracle, monkeypatch):
    """n_c = 2025 (> 1024 + panel: the column-per-thread update branch of the blocked
    Gauss-Jordan) and n = 8100 with 2x2 aggregates, vs the oracle. The one-workgroup coarse
    setup is forced (a single call this size otherwise factors device-wide)."""
    monkeypatch.setenv("MLAMG_BATCH_NO_EXT", "1")
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mlamg.multigrid
    import mlamg.problems
    import mlamg as ml
    m = 90
    A = ml.problems.poisson_2d_5pt(m)
    P, _ = oracle.smoothed_aggregation_jacobi(A, ml.problems.box_aggregates_2d(m, m, 2),
                                              omega=2.0 / 3.0)
    assert P.shape[1] == 2025
    x0 = np.random.RandomState(3).randn(A.shape[0])
    xr, cr, er, ir = oracle.amg_2_v(A, P, np.zeros(A.shape[0]), x0, res_tol=1e-10)
    xf, cf, ef, itf = ml.multigrid.amg_2_v(A, P, np.zeros(A.shape[0]), x0, res_tol=1e-10,
                                           engine="fused")
    assert itf == ir and np.allclose(ef, er, rtol=1e-10, atol=0) and abs(cf - cr) <= 1e-8


@pytest.mark.parametrize("m,agg", ((48, 2), (96, 3)))
def test_fused_single_device_wide_coarse(oracle, monkeypatch, m, agg):
    """A single fused call with n_c > 300 (576, 1024) builds its coarse inverse with the
    device-wide inverse Cholesky factor (csrc/dense.hip) instead of one workgroup's: same
    iteration count and histories as the one-workgroup factor and the oracle (SuperLU) to
    rounding (rtol 1e-10), iterates within 1e-9 of their max."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mlamg.multigrid
    import mlamg.problems
    import mlamg as ml
    A = ml.problems.poisson_2d_5pt(m)
    P, _ = oracle.smoothed_aggregation_jacobi(A, ml.problems.box_aggregates_2d(m, m, agg),
                                              omega=2.0 / 3.0)
    assert P.shape[1] > 512
    x0 = np.random.RandomState(m).randn(A.shape[0])
    b = np.zeros(A.shape[0])
    xe, ce, ee, ie = ml.multigrid.amg_2_v(A, P, b, x0, res_tol=1e-10, engine="fused")
    monkeypatch.setenv("MLAMG_BATCH_NO_EXT", "1")
    xw, cw, ew, iw = ml.multigrid.amg_2_v(A, P, b, x0, res_tol=1e-10, engine="fused")
    xr, cr, er, ir = oracle.amg_2_v(A, P, b, x0, res_tol=1e-10)
    assert ie == iw == ir
    for e in (ee, ew):
        assert np.allclose(e, er, rtol=1e-10, atol=0)
    scale = np.abs(xr).max()
    assert np.abs(xe - xr).max() <= 1e-9 * scale and np.abs(xe - xw).max() <= 1e-9 * scale


def test_fused_phased_edge_cases(oracle):
    """The phased single-call path (n_c > 300: device-wide Galerkin and factor, cycles split
    into workgroup half-cycles and an all-CU coarse solve) on the edge cases of the one-launch
    path: a singular Galerkin operator (the reference's early return), max_iter 0 / 1 / 2, rows
    with a zero diagonal (not SPD: the Gauss-Jordan setup is relaunched), and a non-symmetric
    operator (no device-wide factor; Gauss-Jordan in the setup kernel)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import scipy.sparse as sp
    import mlamg.multigrid
    import mlamg.problems
    import mlamg as ml
    m = 40
    A = ml.problems.poisson_2d_5pt(m)
    Agg = ml.problems.box_aggregates_2d(m, m, 2)
    assert Agg.shape[1] > 300
    x0 = np.random.RandomState(4).randn(A.shape[0])
    z = np.zeros(A.shape[0])
    # singular: an empty coarse column
    Ps = sp.hstack([sp.csr_matrix(Agg, dtype=np.float64), sp.csr_matrix((A.shape[0], 1))]).tocsr()
    x, c, e, it = ml.multigrid.amg_2_v(A, Ps, z, x0, res_tol=1e-10, engine="fused")
    assert (it, c) == (0, 1.0) and np.array_equal(x, x0) and not np.any(e)
    P, _ = oracle.smoothed_aggregation_jacobi(A, Agg, omega=2.0 / 3.0)
    for mi in (0, 1, 2):
        got = ml.multigrid.amg_2_v(A, P, z, x0, res_tol=1e-300, max_iter=mi, engine="fused")
        ref = oracle.amg_2_v(A, P, z, x0, res_tol=1e-300, max_iter=mi)
        assert got[3] == ref[3] == mi and len(got[2]) == mi
        assert np.allclose(got[2], ref[2], rtol=1e-10, atol=0)
        assert np.abs(got[0] - ref[0]).max() <= 1e-9 * np.abs(ref[0]).max()
    # zero diagonal rows (A_H no longer SPD in floating point: relaunched Gauss-Jordan)
    Az = A.copy()
    for i in (0, 55, 777, A.shape[0] - 1):
        lo, hi = Az.indptr[i], Az.indptr[i + 1]
        Az.data[lo + np.flatnonzero(Az.indices[lo:hi] == i)] = 0.0
    b = np.random.RandomState(5).randn(A.shape[0])
    # a non-symmetric operator (host check: no device-wide factor at all)
    An = A.copy().tolil()
    An[3, 4] = -1.5
    An = An.tocsr()
    for M in (Az, An):
        xr, cr, er, ir = oracle.amg_2_v(M, P, b, x0, res_tol=1e-300, max_iter=6)
        xf, cf, ef, itf = ml.multigrid.amg_2_v(M, P, b, x0, res_tol=1e-300, max_iter=6,
                                               engine="fused")
        assert itf == ir == 6
        assert np.allclose(ef, er, rtol=1e-10, atol=0), (ef, er)
        assert np.abs(xf - xr).max() <= 1e-9 * np.abs(xr).max()


@pytest.mark.parametrize("smoother", ("gauss_seidel", "jacobi"))
def test_phased_batch_equals_one_launch(oracle, monkeypatch, smoother):
    """A batch whose largest coarse operator has n_c > 300 runs phased (each problem's cycles on
    its workgroup, every problem's coarse solve — L^-1 then L^-T passes, or the Gauss-Jordan
    inverse — spread over the CUs, a done counter ending the launches). With the one-workgroup
    factors (MLAMG_BATCH_NO_BATCH_EXT) it is the same arithmetic as the one-launch batch, so the
    same bits, problems finishing at different cycles included; by default its SPD operators are
    factored device-wide in one batched launch sequence (dense.hip): same iteration counts,
    histories within rtol 1e-10 (+ 1e-12 of the first norm), iterates within 1e-9 of their max."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mlamg.multigrid
    import mlamg.problems
    import mlamg as ml
    probs = _problems(ml, oracle, 14)
    assert max(P.shape[1] for _, P, _, _ in probs) > 300
    # a non-symmetric operator (Gauss-Jordan inverse, mode 0) in the mix
    A, P, b, x = probs[3]
    A = A.tolil()
    A[3, 4] = -1.5
    probs[3] = (A.tocsr(), P, b, x)
    ext = ml.multigrid.amg_2_v_batch(probs, res_tol=1e-10, smoother=smoother)
    monkeypatch.setenv("MLAMG_BATCH_NO_BATCH_EXT", "1")
    ph = ml.multigrid.amg_2_v_batch(probs, res_tol=1e-10, smoother=smoother)
    monkeypatch.setenv("MLAMG_BATCH_NO_PHASED_BATCH", "1")
    one = ml.multigrid.amg_2_v_batch(probs, res_tol=1e-10, smoother=smoother)
    assert len({r[3] for r in ph}) > 1  # not all problems stop at the same cycle
    for i, (a, c) in enumerate(zip(ph, one)):
        assert a[3] == c[3] and np.array_equal(a[2], c[2]) and np.array_equal(a[0], c[0]), i
    for i, (a, c) in enumerate(zip(ext, one)):
        # (b != 0 problems reach the residual's rounding floor near res_tol: atol 1e-12 err_0)
        assert a[3] == c[3] and np.allclose(a[2], c[2], rtol=1e-10, atol=1e-12 * c[2][0]), i
        assert np.abs(a[0] - c[0]).max() <= 1e-9 * np.abs(c[0]).max(), i
