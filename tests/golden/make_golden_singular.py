"""Golden vectors of the reference's SINGULAR two-level driver (ns/lib/multigrid.py:111-210 with
singular=True: lsqr coarse solve, mean removal — the Neumann path its callers select with
neumann_solve, e.g. utils/evaluate_model.py:94,172) -> tests/golden/reference_singular.npz.

Container-only, like make_golden.py (same stubs: pyamg.relaxation.gauss_seidel delegates to the
oracle's restatement; scipy's lsqr is the real one). Inputs: Neumann Laplacians (constant
nullspace), box aggregates, P = (I - (2/3) D^-1 A) Agg formed with scipy (the
demos/1d_poisson.py:59-60 form, no ARPACK), consistent right-hand sides (zero mean).

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_singular.py
"""
from __future__ import annotations

import os
import sys

import numpy as np
import scipy.sparse as sp

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import make_golden  # noqa: E402


def neumann_1d(n):
    A = (sp.eye(n) * 2 - sp.eye(n, k=-1) - sp.eye(n, k=1)).tolil()
    A[0, 0] = 1.0
    A[n - 1, n - 1] = 1.0
    return A.tocsr()


def neumann_2d(m):
    T = neumann_1d(m)
    A = (sp.kron(sp.eye(m), T) + sp.kron(T, sp.eye(m))).tocsr()
    A.sort_indices()
    return A


def box_agg(n, size):
    k = (n + size - 1) // size
    return sp.csr_matrix((np.ones(n), (np.arange(n), np.arange(n) // size)), shape=(n, k))


def sa_p(A, Agg, w=2.0 / 3.0):
    Dinv = sp.diags(1.0 / A.diagonal())
    return ((sp.eye(A.shape[0]) - w * Dinv @ A) @ Agg).tocsr()


def main():
    mg, _, _ = make_golden.load_reference()
    out = {}
    cases = {
        "n1d": (neumann_1d(300), 3, "res"),
        "n2d": (neumann_2d(24), 4, "err"),
    }
    for key, (A, size, mode) in cases.items():
        n = A.shape[0]
        P = sa_p(A, box_agg(n, size))
        rs = np.random.RandomState(5)
        x0 = rs.normal(0, 1, n)
        if mode == "res":
            b = rs.randn(n)
            b -= b.mean()
            xr, conv, err, it = mg.amg_2_v(A, P, b, x0, res_tol=1e-8, singular=True, max_iter=60)
        else:
            b = np.zeros(n)
            xr, conv, err, it = mg.amg_2_v(A, P, b, x0, error_tol=1e-9, singular=True,
                                           max_iter=60)
        for name, M in (("A", A), ("P", P)):
            out[f"{key}_{name}_indptr"] = M.indptr.astype(np.int32)
            out[f"{key}_{name}_indices"] = M.indices.astype(np.int32)
            out[f"{key}_{name}_data"] = M.data
            out[f"{key}_{name}_shape"] = np.array(M.shape)
        out[f"{key}_x0"], out[f"{key}_b"] = x0, b
        out[f"{key}_x"], out[f"{key}_conv"], out[f"{key}_err"] = xr, np.float64(conv), err
        print(key, n, "iters", it, "conv", conv, "err", err[0], "->", err[-1])
    np.savez(os.path.join(HERE, "reference_singular.npz"), **out)


if __name__ == "__main__":
    main()
