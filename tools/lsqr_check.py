"""Device LSQR vs scipy.sparse.linalg.lsqr on the golden singular Galerkin operator (GPU box)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "ml-amg_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import scipy.sparse as sp  # noqa: E402
import scipy.sparse.linalg as spla  # noqa: E402


def main():
    import torch  # noqa: F401
    from conftest import golden_csr
    from mlamg import multigrid
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "reference_singular.npz")))
    A, P = golden_csr(g, "n2d_A"), golden_csr(g, "n2d_P")
    AH = (P.T @ A @ P).tocsr()
    rs = np.random.RandomState(3)
    rhs = P.T @ rs.randn(A.shape[0])
    for lim in (1, 2, 3, 5, 10, 20, 40, 83, None):
        xr, istop, itn = spla.lsqr(AH, rhs, iter_lim=lim)[:3]
        x, istop_d, itn_d = multigrid.lsqr(AH, rhs, iter_lim=lim)
        d = np.abs(x - xr).max() / np.abs(xr).max()
        print(f"iter_lim={lim}: scipy ({istop},{itn}) device ({istop_d},{itn_d}) rel diff {d:.3e}")
    M = sp.random(300, 120, density=0.05, random_state=rs, format="csr") + sp.eye(300, 120, format="csr")
    b = rs.randn(300)
    xr, istop, itn = spla.lsqr(M, b)[:3]
    x, istop_d, itn_d = multigrid.lsqr(M.tocsr(), b)
    print("rect", istop, itn, istop_d, itn_d, np.abs(x - xr).max() / np.abs(xr).max())


if __name__ == "__main__":
    main()
