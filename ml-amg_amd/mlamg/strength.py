"""Strength-of-connection measures of the reference's loops, on the device.

Mirrors utils/common.py:25-31 (`strength_measure_funcs`: 'abs', 'evolution', 'invabs', 'unit',
'olson'; 'olson' is the default measure of utils/common.py:53, utils/evaluate_dataset.py:76,84,
utils/evaluate_model.py:40, utils/train_one_sample.py:61) and the pyamg function those measures
call, `pyamg.strength.evolution_strength_of_connection` (pyamg is absent here: restated in
csrc/strength.hip; parity unpinned).

The measures take and return scipy CSR like the reference; `device=True` returns a DeviceCSR
instead (what mlamg.hierarchy consumes).
"""
from __future__ import annotations

import ctypes

import numpy as np
import scipy.sparse as sp

from ._lib import call, ptr, stream_ptr
from .sparse import DeviceCSR


def _prepared(A):
    """A as pyamg works on it: CSR, explicit zeros eliminated, ascending column indices."""
    if sp.isspmatrix_bsr(A):
        raise NotImplementedError("BSR input (numPDEs > 1) is not supported")
    if not sp.isspmatrix_csr(A):
        raise TypeError("expected csr_matrix or bsr_matrix")
    A = A.astype(np.float64, copy=True)
    A.eliminate_zeros()
    A.sort_indices()
    return A


def spectral_radius_dinv_a(A_dev):
    """rho(D^-1 A) by the device Lanczos lambda_max of the symmetric D^-1/2 A D^-1/2 (exact to
    ~1e-12; the opt-in rho='lanczos' of the measures below and what Hierarchy.build uses)."""
    from .multigrid import lambda_max_dinv_a
    lam, _ = lambda_max_dinv_a(A_dev)
    return abs(lam)


def _pyamg_norm(x):
    """pyamg.util.linalg.norm(x): sqrt(inner(conj(x), x).real) of the raveled vector."""
    x = np.ravel(x)
    return np.sqrt(np.inner(x.conj(), x).real)


class _DeviceMatvec:
    """v -> M @ v for host (n, 1) vectors with the product on the device: the device SpMV sums
    every row in stored order like scipy's csr_matvec, so the host Arnoldi around it sees
    scipy's bits. A complex v (a complex Ritz vector after a restart) is two real products:
    scipy multiplies (a + 0i)(x_r + i x_i), whose parts a*x_r - 0*x_i and a*x_i + 0*x_r equal
    a*x_r and a*x_i except possibly in the sign of an exactly zero row sum."""

    def __init__(self, M_dev):
        import torch
        self.M = M_dev
        self.torch = torch
        self.dev = torch.device("cuda", torch.cuda.current_device())

    def _real(self, v):
        t = self.torch.as_tensor(np.ascontiguousarray(v, dtype=np.float64)).to(self.dev)
        return self.M.matvec(t).cpu().numpy()

    def __call__(self, v):
        flat = np.ravel(v)
        if np.iscomplexobj(flat):
            y = self._real(flat.real) + 1j * self._real(flat.imag)
        else:
            y = self._real(flat)
        return y.reshape(-1, 1)


def approximate_spectral_radius(M_dev, tol=0.01, maxiter=15, restart=5):
    """pyamg.util.linalg.approximate_spectral_radius(M) (pyamg 4.x/5.x, absent here; called by
    evolution_strength_of_connection on D^-1 A): Arnoldi with modified Gram-Schmidt from
    np.random.rand(n, 1) — n draws from numpy's GLOBAL generator, exactly as pyamg consumes
    them, so a caller that seeds (utils/evaluate_model.py:53-55, utils/common.py:51-58) sees
    the same generator state afterwards —, restarted up to `restart` times from the dominant
    Ritz vector until |H[m, m-1] y_m| / |ev| < tol. The products M @ v run on the device
    (bitwise csr_matvec); the Krylov vectors, inner products and the small eigenproblem
    (scipy.linalg.eig) are host numpy, the same calls pyamg makes. Returns |ev_max| (float)."""
    import scipy.linalg
    n = M_dev.shape[0]
    if M_dev.shape[0] != M_dev.shape[1]:
        raise ValueError("expected square A")
    if maxiter < 1:
        raise ValueError("expected maxiter > 0")
    if restart < 0:
        raise ValueError("expected restart >= 0")
    matvec = _DeviceMatvec(M_dev)
    v0 = np.random.rand(n, 1)
    maxiter = min(n, maxiter)
    breakdown = np.finfo(np.float64).eps * 1e6
    ev = evect = None
    max_index = 0
    for _ in range(restart + 1):
        # pyamg _approximate_eigenvalues(A, maxiter, initial_guess=v0)
        v0 = v0 / _pyamg_norm(v0)
        H = np.zeros((maxiter + 1, maxiter), dtype=np.result_type(v0.dtype, np.float64))
        V = [v0]
        flag = False
        j = 0
        for j in range(maxiter):
            w = matvec(V[-1])
            for i, v in enumerate(V):
                H[i, j] = np.dot(np.conjugate(v.ravel()), w.ravel())
                w = w - H[i, j] * v
            H[j + 1, j] = _pyamg_norm(w)
            if H[j + 1, j] < breakdown:
                flag = True
                if H[j + 1, j] != 0:
                    w = w / H[j + 1, j]
                V.append(w)
                break
            w = w / H[j + 1, j]
            V.append(w)
        ev, evect = scipy.linalg.eig(H[:j + 1, :j + 1], left=False, right=True)
        nvecs = ev.shape[0]
        max_index = np.abs(ev).argmax()
        error = H[nvecs, nvecs - 1] * evect[-1, max_index]
        v0 = np.dot(np.hstack(V[:-1]), evect[:, max_index].reshape(-1, 1))
        if np.abs(error) / np.abs(ev[max_index]) < tol or flag:
            break
    return float(np.abs(ev[max_index]))


def pyamg_dinv(A):
    """get_diagonal(A, inv=True) with Dinv[D == 0] = 1 (pyamg evolution_strength_of_connection's
    scaling of A before its spectral radius estimate)."""
    D = A.diagonal()
    Dinv = np.zeros_like(D, dtype=np.float64)
    mask = D != 0.0
    Dinv[mask] = 1.0 / D[mask]
    Dinv[D == 0] = 1.0
    return Dinv


def spectral_radius_pyamg(A):
    """rho(D^-1 A) as pyamg's evolution measure estimates it: D^-1 A formed from A as given
    (stored order kept, before pyamg's eliminate_zeros / sort_indices) by row scaling on the
    device, then approximate_spectral_radius (consumes n global-RNG draws)."""
    A = A.tocsr() if not sp.isspmatrix_csr(A) else A
    A = A.astype(np.float64, copy=False)
    d = pyamg_dinv(A)
    import torch
    d_dev = torch.as_tensor(d).to(torch.device("cuda", torch.cuda.current_device()))
    A_dev = DeviceCSR.from_scipy(A)
    h = ctypes.c_void_p()
    # zero products dropped by the row scaling never change a csr_matvec sum (the running sum
    # starts at +0.0 and is never -0.0, so adding a signed zero leaves it unchanged)
    call("mlamg_csr_scale_rows", A_dev.handle, ptr(d_dev), 0, ctypes.byref(h), stream_ptr())
    return approximate_spectral_radius(DeviceCSR(h))


MODES = {"evolution_soc": 0, "evolution": 1, "olson": 2}


def evolution_device(A_dev, mode="olson", rho=None, epsilon=4.0):
    """The measure of a device CSR (ascending columns — every Galerkin level is), as a new
    DeviceCSR; mode 'evolution_soc' (pyamg's function), 'evolution' or 'olson'
    (utils/common.py:27,30). rho: rho(D^-1 A), default (None or 'lanczos') the device Lanczos
    value — this is the hierarchy's path, which draws nothing from the global generator."""
    if rho is None or rho == "lanczos":
        rho = spectral_radius_dinv_a(A_dev)
    h = ctypes.c_void_p()
    call("mlamg_evolution_strength", A_dev.handle, float(rho), float(epsilon), int(MODES[mode]),
         ctypes.byref(h), stream_ptr())
    return DeviceCSR(h)


def _evolution(A, mode, epsilon=4.0, rho=None, device=False):
    """rho=None: pyamg's own estimate (seeded Arnoldi on the global generator, the reference
    call's behaviour); rho='lanczos': the device Lanczos value; a number: that value."""
    if rho is None:
        rho = spectral_radius_pyamg(A)
    C = evolution_device(DeviceCSR.from_scipy(_prepared(A)), mode, rho=rho, epsilon=epsilon)
    return C if device else C.to_scipy()


def evolution_strength_of_connection(A, B=None, epsilon=4.0, k=2, proj_type="l2",
                                     block_flag=False, symmetrize_measure=True, *, rho=None,
                                     device=False):
    """pyamg.strength.evolution_strength_of_connection at the arguments the reference uses
    (utils/common.py:27,30: all defaults). Other time-step counts, near-nullspace vectors,
    projections or an unsymmetrized measure raise NotImplementedError. `rho` overrides the
    spectral radius estimate of D^-1 A."""
    if epsilon < 1.0:
        raise ValueError("expected epsilon > 1.0")
    if k <= 0:
        raise ValueError("number of time steps must be > 0")
    if proj_type not in ("l2", "D_A"):
        raise ValueError('proj_type must be "l2" or "D_A"')
    if B is not None and not np.all(np.asarray(B) == 1.0):
        raise NotImplementedError("only B = ones (the reference's default)")
    if k != 2 or proj_type != "l2" or block_flag or not symmetrize_measure:
        raise NotImplementedError("only k=2, proj_type='l2', symmetrize_measure=True")
    return _evolution(A, "evolution_soc", epsilon=epsilon, rho=rho, device=device)


def evolution(A, *, rho=None, device=False):
    """utils/common.py:27: evolution(A) + 0.1 * unit(A)."""
    return _evolution(A, "evolution", rho=rho, device=device)


def olson(A, *, rho=None, device=False):
    """utils/common.py:30: evolution(A) + 1/|A| (the reference's default measure)."""
    return _evolution(A, "olson", rho=rho, device=device)


def _elementwise(A, mode, device=False):
    from .hierarchy import STRENGTH_MODES, strength
    A = A.tocsr() if not sp.isspmatrix_csr(A) else A
    C = strength(DeviceCSR.from_scipy(A), mode)
    return C if device else C.to_scipy()


strength_measure_funcs = {
    "abs": lambda A: _elementwise(A, "abs"),
    "evolution": evolution,
    "invabs": lambda A: _elementwise(A, "invabs"),
    "unit": lambda A: _elementwise(A, "unit"),
    "olson": olson,
}
