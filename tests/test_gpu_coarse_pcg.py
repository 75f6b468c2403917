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
