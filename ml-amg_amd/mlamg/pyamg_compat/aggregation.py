"""pyamg.aggregation (4.x) subset, on the device: lloyd_aggregation (mlamg.graph),
standard_aggregation, fit_candidates and smoothed_aggregation_solver (mlamg.hierarchy.pyamg_sa:
the solver ns/preconditioner/PyAMG.py:94 builds; pyamg absent, parity unpinned)."""
import numpy as np
import scipy.sparse as sp

from ..graph import pyamg_lloyd_aggregation as lloyd_aggregation  # noqa: F401


def _dev(M):
    from ..sparse import DeviceCSR
    return M if isinstance(M, DeviceCSR) else DeviceCSR.from_scipy(sp.csr_matrix(M))


def standard_aggregation(C):
    """(AggOp int8 CSR n x k, Cpts): amg_core's three greedy passes (device rounds, bitwise)."""
    import ctypes
    import torch
    from .._lib import call, ptr, stream_ptr
    if not sp.isspmatrix_csr(C):
        raise TypeError("expected csr_matrix")
    if C.shape[0] != C.shape[1]:
        raise ValueError("expected square matrix")
    n = C.shape[0]
    Cd = _dev(C)
    dev = torch.device("cuda", torch.cuda.current_device())
    agg = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    cpts = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    k, rounds = ctypes.c_int64(), ctypes.c_int32()
    call("mlamg_standard_aggregation", Cd.handle, ptr(agg), ptr(cpts), ctypes.byref(k),
         ctypes.byref(rounds), stream_ptr())
    k = int(k.value)
    a = agg[:n].cpu().numpy()
    Cp = cpts[:k].cpu().numpy().astype(C.indptr.dtype)
    if k == 0:
        return sp.csr_matrix((n, 1), dtype="int8"), np.array([], dtype=C.indptr.dtype)
    rows = np.nonzero(a >= 0)[0]
    AggOp = sp.csr_matrix((np.ones(len(rows), dtype="int8"), (rows, a[rows])), shape=(n, k))
    return AggOp, Cp


def fit_candidates(AggOp, B, tol=1e-10):
    """(Q, R) for one candidate (B of shape (n, 1)): Q = per-aggregate normalised B, R = the
    norms (amg_core fit_candidates_common, device)."""
    import ctypes
    import torch
    from .._lib import call, ptr, stream_ptr
    from ..sparse import DeviceCSR
    B = np.asarray(B, dtype=np.float64)
    if B.ndim == 2 and B.shape[1] != 1 or B.size != AggOp.shape[0]:
        raise NotImplementedError("one candidate: B of shape (n, 1)")
    A = sp.csr_matrix(AggOp, dtype=np.float64)
    Ad = DeviceCSR.from_scipy(A)
    dev = torch.device("cuda", torch.cuda.current_device())
    Bd = torch.as_tensor(np.ascontiguousarray(B.reshape(-1))).to(dev)
    Bc = torch.empty(max(A.shape[1], 1), dtype=torch.float64, device=dev)
    h = ctypes.c_void_p()
    call("mlamg_fit_candidates", Ad.handle, ptr(Bd), float(tol), ctypes.byref(h), ptr(Bc),
         stream_ptr())
    return DeviceCSR(h).to_scipy(), Bc[:A.shape[1]].cpu().numpy().reshape(-1, 1)


def smoothed_aggregation_solver(A, B=None, BH=None, symmetry="hermitian", strength="symmetric",
                                aggregate="standard", smooth=("jacobi", {"omega": 4.0 / 3.0}),
                                presmoother=("block_gauss_seidel", {"sweep": "symmetric"}),
                                postsmoother=("block_gauss_seidel", {"sweep": "symmetric"}),
                                improve_candidates=(("block_gauss_seidel",
                                                     {"sweep": "symmetric", "iterations": 4}),
                                                    None),
                                max_levels=10, max_coarse=10, diagonal_dominance=False,
                                keep=False, **kwargs):
    """pyamg's smoothed_aggregation_solver with its default recipe on the device (Hierarchy.
    pyamg_sa); returns a MultilevelSolver. Arguments other than the defaults, max_levels,
    max_coarse, B (one candidate) and strength=('symmetric', {'theta': t}) raise
    NotImplementedError."""
    from ..hierarchy import Hierarchy
    from .multilevel import MultilevelSolver
    theta = 0.0
    if isinstance(strength, tuple) and strength[0] == "symmetric":
        theta = float(dict(strength[1]).get("theta", 0.0))
    elif strength != "symmetric":
        raise NotImplementedError("strength must be 'symmetric' (pyamg's default)")
    omega = 4.0 / 3.0
    if isinstance(smooth, tuple) and len(smooth) == 2 and smooth[0] == "jacobi":
        omega = float(dict(smooth[1]).get("omega", omega))
    elif smooth != "jacobi":
        raise NotImplementedError("smooth must be 'jacobi' (pyamg's default)")
    defaults_ok = (symmetry == "hermitian" and aggregate == "standard" and BH is None
                   and not diagonal_dominance and not keep
                   and presmoother == postsmoother == ("block_gauss_seidel",
                                                       {"sweep": "symmetric"}))
    imp = improve_candidates[0] if isinstance(improve_candidates, (list, tuple)) else None
    iters = 0
    if imp is not None:
        if imp[0] != "block_gauss_seidel" or imp[1].get("sweep") != "symmetric":
            defaults_ok = False
        iters = int(imp[1].get("iterations", 1))
    if not defaults_ok or kwargs.get("coarse_solver", "pinv") != "pinv":
        raise NotImplementedError("only pyamg's default smoothed-aggregation recipe")
    if not (sp.isspmatrix_csr(A) or hasattr(A, "handle")):
        A = sp.csr_matrix(A)
    H = Hierarchy.pyamg_sa(A, max_levels=int(max_levels), max_coarse=int(max_coarse),
                           theta=theta, omega=omega, improve_iterations=iters, B=B)
    return MultilevelSolver(H)
