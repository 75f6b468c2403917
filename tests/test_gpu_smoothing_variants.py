"""GPU parity of the V-cycle executor for every (pre, post) smoothing count, not only V(1,1), and
of the tolerance test at tol = 0.

The executor fuses the end-of-cycle residual with the next cycle's first pre-smoothing sweep
only when the cycle's result lands in the ping-pong buffer ((nu_pre - 1 + nu_post) odd,
csrc/hier.hip fused_presmooth); V(2,1) / V(1,2) / V(2,2) / V(0,k) exercise both branches against
the oracle's restatement of ns/lib/multigrid.py:111-210 (jacobi smoother) and
ns/preconditioner/MLAMG.py:148-197, and the multilevel executor against oracle.vcycle_solve.

tol = 0: the reference stops on `e <= tol` (multigrid.py:197, MLAMG.py:194), so a zero rhs with a
zero guess stops after one cycle with err = [0.] and conv_factor 0 (len(err) == 1, :201)."""
import numpy as np
import pytest

from conftest import golden_csr

pytestmark = pytest.mark.gpu

NU = ((1, 1), (2, 1), (1, 2), (2, 2), (3, 1), (0, 1), (1, 0), (0, 2))


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


def _P1(golden):
    return golden_csr(golden, "c1_P")


@pytest.mark.parametrize("nu", NU)
def test_amg_2_v_jacobi_smoothing_counts(golden, ml, oracle, nu):
    """amg_2_v(smoother='jacobi') for V(nu_pre, nu_post), both tolerance modes, vs the oracle.
    Tolerance as every two-level test: the coarse solve is a dense inverse where the reference
    factorises with SuperLU (differences ~1e-16 relative per cycle)."""
    A, P = golden_csr(golden, "c1"), _P1(golden)
    x0 = np.random.RandomState(0).normal(0, 1, 1024)
    # b = A xs with xs = O(1): the iterate stays O(1), so the dense-inverse vs SuperLU rounding
    # difference stays ~1e-15 of the history (with a random b, x grows to ~5e3 on this 1D
    # operator and both CPU variants already differ by ~1e-12 absolute)
    b = A @ np.random.RandomState(1).normal(0, 1, 1024)
    pre, post = nu
    for kw in ({"res_tol": 1e-300}, {"error_tol": 1e-300}):
        xr, cr, er, ir = oracle.amg_2_v(A, P, b, x0, pre, post, 0.666, max_iter=9,
                                        smoother="jacobi", **kw)
        for use_graph in (False, True):
            x, c, e, it = ml.multigrid.amg_2_v(A, P, b, x0, pre, post, 0.666, max_iter=9,
                                               smoother="jacobi", use_graph=use_graph, **kw)
            assert it == ir == 9
            assert np.allclose(e, er, rtol=1e-10, atol=1e-13 * er[0]), (nu, kw, e, er)
            assert abs(c - cr) <= 1e-8
            assert np.allclose(x, xr, rtol=1e-9, atol=1e-12 * np.abs(xr).max())


@pytest.mark.parametrize("nu", ((2, 1), (1, 2), (2, 2), (3, 1)))
def test_mlamg_amg_2_v_smoothing_counts(golden, ml, oracle, nu):
    """MLAMG.amg_2_v (MLAMG.py:148-197) with pre/post counts other than 1. The coarse solve is a
    dense inverse (inverse Cholesky factor) against the oracle's SuperLU: rounding-level
    differences, amplified by cond(A_H) ~ 1e5 of this 1D problem, so the iterate is compared
    within 1e-9 of its max (its smallest entries are 1e-4 of the max)."""
    A, P = golden_csr(golden, "c1"), _P1(golden)
    x0 = np.random.RandomState(0).normal(0, 1, 1024)
    b = np.zeros(1024)
    xr, hr = oracle.mlamg_amg_2_v(A, P, oracle.mlamg_dinv(A), b, x0, nu[0], nu[1], max_iter=7,
                                  amg_rtol=1e-300)
    x, h = ml.multigrid.amg_2_v_jacobi(A, P, b, x0, pre_smoothing_steps=nu[0],
                                       post_smoothing_steps=nu[1], max_iter=7, tol=1e-300,
                                       history=True)
    assert len(h) == len(hr) == 7
    assert np.allclose(h, hr, rtol=1e-10, atol=1e-13 * hr[0])
    assert np.abs(x - xr).max() <= 1e-9 * np.abs(xr).max(), np.abs(x - xr).max() / np.abs(xr).max()


@pytest.mark.parametrize("nu", ((2, 1), (1, 2), (2, 2), (0, 1)))
def test_multilevel_smoothing_counts(ml, oracle, torch_cuda, nu):
    """Multilevel executor V(nu_pre, nu_post) vs oracle.vcycle_solve on the device's operators
    (bitwise but for the coarsest dense solve: rtol 1e-11 on the history)."""
    from test_gpu_hierarchy import _oracle_levels_from_device
    torch = torch_cuda
    A = ml.problems.poisson_2d_5pt(48)
    H = ml.hierarchy.Hierarchy.build(A, alpha=0.1, max_coarse=100, nu_pre=nu[0], nu_post=nu[1])
    assert H.n_levels >= 2
    lv = _oracle_levels_from_device(H)
    n = A.shape[0]
    x0 = np.random.RandomState(0).randn(n)
    b = np.random.RandomState(1).randn(n)
    xo, ho = oracle.vcycle_solve(lv, H.Ac.to_scipy(), b, x0, 5, nu_pre=nu[0], nu_post=nu[1])
    for use_graph in (False, True):
        xd = torch.as_tensor(x0).cuda()
        hd = H.cycle(torch.as_tensor(b).cuda(), xd, 5, use_graph=use_graph)
        assert np.allclose(hd, ho, rtol=1e-11, atol=0), (nu, hd, ho)
        assert np.allclose(xd.cpu().numpy(), xo, rtol=1e-10, atol=1e-12 * np.abs(xo).max())


@pytest.mark.parametrize("smoother", ("gauss_seidel", "jacobi"))
def test_amg_2_v_zero_tolerance_zero_norm(golden, ml, oracle, smoother):
    """res_tol = 0 / error_tol = 0 with b = 0, x0 = 0: the norm is exactly 0 after the first
    cycle, so the reference returns err = [0.], 1 iteration, conv_factor 0."""
    A, P = golden_csr(golden, "c1"), _P1(golden)
    z = np.zeros(1024)
    for kw in ({"res_tol": 0.0}, {"error_tol": 0.0}):
        xr, cr, er, ir = oracle.amg_2_v(A, P, z, z, max_iter=50, smoother=smoother, **kw)
        assert ir == 1 and er.tolist() == [0.0] and cr == 0
        x, c, e, it = ml.multigrid.amg_2_v(A, P, z, z, max_iter=50, smoother=smoother, **kw)
        assert it == 1 and list(e) == [0.0] and c == 0 and not np.any(x)


def test_hierarchy_cycle_tol_none_vs_zero(ml, torch_cuda):
    """Hierarchy.cycle: tol=None runs every cycle; tol=0 stops on the first exactly-zero norm."""
    torch = torch_cuda
    A = ml.problems.poisson_2d_5pt(32)
    H = ml.hierarchy.Hierarchy.build(A, alpha=0.1, max_coarse=50)
    n = A.shape[0]
    z = torch.zeros(n, dtype=torch.float64, device="cuda")
    assert len(H.cycle(z, z.clone(), 7)) == 7
    h = H.cycle(z, z.clone(), 7, tol=0.0)
    assert len(h) == 1 and h[0] == 0.0
