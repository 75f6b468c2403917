"""pyamg.multilevel.MultilevelSolver (4.x) subset, over a device hierarchy: what the reference's
PyAMG preconditioner uses of the object `pyamg.aggregation.smoothed_aggregation_solver` returns
(ns/preconditioner/PyAMG.py:94 builds it, :119 calls `solve(b, tol=amg_rtol, accel='gmres' or
None)`, :129 prints it). pyamg is absent: the semantics follow pyamg 4.x's solve (tolerance
relative to ||b||, at most maxiter cycles or Krylov steps, one V-cycle from a zero guess as the
preconditioner); parity unpinned."""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla


class _Level:
    """One level: A (and P, R above the coarsest) as scipy CSR, downloaded on first access."""

    def __init__(self, A_dev, P_dev=None, R_dev=None):
        self._dev = {"A": A_dev, "P": P_dev, "R": R_dev}
        self._host = {}

    def _get(self, k):
        if k not in self._host:
            d = self._dev[k]
            self._host[k] = None if d is None else d.to_scipy()
        return self._host[k]

    A = property(lambda self: self._get("A"))
    P = property(lambda self: self._get("P"))
    R = property(lambda self: self._get("R"))


class MultilevelSolver:
    """solve / aspreconditioner / complexities / repr of pyamg's MultilevelSolver."""

    def __init__(self, H, coarse_solver="pinv"):
        self.H = H
        self.coarse_solver_name = coarse_solver
        self.levels = [_Level(L.A, L.P, L.R) for L in H.levels] + [_Level(H.Ac)]

    def _nnz(self):
        return [L.A.nnz for L in self.H.levels] + [self.H.Ac.nnz]

    def _rows(self):
        return [L.A.shape[0] for L in self.H.levels] + [self.H.Ac.shape[0]]

    def operator_complexity(self):
        nnz = self._nnz()
        return float(sum(nnz)) / nnz[0]

    def grid_complexity(self):
        rows = self._rows()
        return float(sum(rows)) / rows[0]

    def __repr__(self):
        rows, nnz = self._rows(), self._nnz()
        out = ["MultilevelSolver",
               f"Number of Levels:     {len(rows)}",
               f"Operator Complexity:  {self.operator_complexity():6.3f}",
               f"Grid Complexity:      {self.grid_complexity():6.3f}",
               f"Coarse Solver:        {self.coarse_solver_name!r}",
               "  level   unknowns     nonzeros"]
        total = float(sum(nnz))
        for i, (n, z) in enumerate(zip(rows, nnz)):
            out.append(f"{i:>6} {n:>11} {z:>12} [{100.0 * z / total:2.2f}%]")
        return "\n".join(out) + "\n"

    def aspreconditioner(self, cycle="V"):
        """One V-cycle from a zero guess as a scipy LinearOperator (pyamg: solve(b, maxiter=1))."""
        if str(cycle).upper() != "V":
            raise NotImplementedError("only V-cycles")
        n = self._rows()[0]
        return spla.LinearOperator((n, n), matvec=lambda b: self.H.precondition(
            np.ascontiguousarray(np.ravel(b), dtype=np.float64)), dtype=np.float64)

    def solve(self, b, x0=None, tol=1e-5, maxiter=100, cycle="V", accel=None, callback=None,
              residuals=None, return_info=False):
        """pyamg MultilevelSolver.solve: accel=None runs V-cycles from x0 (zeros) while the
        residual exceeds tol * ||b|| (||b|| = 0: absolute) and fewer than maxiter cycles ran
        (info: 0 converged, maxiter otherwise); accel='gmres' runs pyamg.krylov.gmres (its
        default Householder orthogonalisation, Hierarchy.gmres_householder) preconditioned by
        one V-cycle: one cycle of at most maxiter steps to a preconditioned residual below tol
        times its initial value (info: 0 converged, else the steps taken; residuals: the
        preconditioned residual norms, as pyamg records them). Returns x (and info with
        return_info)."""
        import torch
        from ..sparse import to_device_vec
        if str(cycle).upper() != "V":
            raise NotImplementedError("only V-cycles")
        if callback is not None:
            raise NotImplementedError("callback is not supported")
        b = np.ascontiguousarray(np.ravel(b), dtype=np.float64)
        H = self.H
        if accel is not None:
            if accel != "gmres":
                raise NotImplementedError("accel must be None or 'gmres'")
            x, info = H.gmres_householder(b, x0=x0, tol=tol, maxiter=int(maxiter),
                                          return_info=True)
            if residuals is not None:
                residuals[:] = list(info["residuals"])
            return (x, info["info"]) if return_info else x
        normb = float(np.linalg.norm(b))
        if normb == 0.0:
            normb = 1.0  # pyamg: an absolute tolerance
        bd = to_device_vec(b)
        xd = (torch.zeros_like(bd) if x0 is None
              else to_device_vec(np.ascontiguousarray(np.ravel(x0), dtype=np.float64)).clone())
        A0 = H.levels[0].A if H.levels else H.Ac
        r0 = float(torch.linalg.vector_norm(bd - A0.matvec(xd)))
        hist = [r0]
        if r0 > tol * normb and maxiter > 0:
            hist += list(H.cycle(bd, xd, int(maxiter), tol=tol * normb))
        if residuals is not None:
            residuals[:] = hist
        x = xd.cpu().numpy()
        code = 0 if hist[-1] <= tol * normb else int(maxiter)
        return (x, code) if return_info else x
