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

from ._lib import call, stream_ptr
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
    """rho(D^-1 A) for the evolution time step: the device Lanczos lambda_max of the symmetric
    D^-1/2 A D^-1/2 (pyamg estimates the same quantity by a 15-step restarted Arnoldi from a
    seeded random vector, to a 1e-2 relative tolerance)."""
    from .multigrid import lambda_max_dinv_a
    lam, _ = lambda_max_dinv_a(A_dev)
    return abs(lam)


MODES = {"evolution_soc": 0, "evolution": 1, "olson": 2}


def evolution_device(A_dev, mode="olson", rho=None, epsilon=4.0):
    """The measure of a device CSR (ascending columns — every Galerkin level is), as a new
    DeviceCSR; mode 'evolution_soc' (pyamg's function), 'evolution' or 'olson'
    (utils/common.py:27,30). rho: rho(D^-1 A), default the device Lanczos value."""
    if rho is None:
        rho = spectral_radius_dinv_a(A_dev)
    h = ctypes.c_void_p()
    call("mlamg_evolution_strength", A_dev.handle, float(rho), float(epsilon), int(MODES[mode]),
         ctypes.byref(h), stream_ptr())
    return DeviceCSR(h)


def _evolution(A, mode, epsilon=4.0, rho=None, device=False):
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
