"""One forward sweep of each Gauss-Seidel arithmetic on the long-offset test operator of
tests/test_gpu_pyamg_sa.py (13 entries a row, couplings up to 19,997 rows apart): run under
rocprofv3 --kernel-trace --stats to see which sweep kernel takes it.

  python tools/gs_probe.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ml-amg_amd")]

import numpy as np  # noqa: E402
import scipy.sparse as sp  # noqa: E402
import torch  # noqa: E402

from mlamg import multigrid, sparse  # noqa: E402

n = 20_000
offs = (3, 150, 1001, 3001, 6007, 9001, 15013, 19997)
O = sp.diags([np.full(n - o, -1.0 / (1 + k)) for k, o in enumerate(offs)], list(offs), (n, n))
W = sp.csr_matrix(O + O.T + sp.identity(n) * 13.0)
W.sort_indices()
offs2 = offs + (7, 11, 13, 17, 19, 23, 29, 31, 37, 41, 43, 47)  # 37 entries a row
O2 = sp.diags([np.full(n - o, -1.0 / (1 + k)) for k, o in enumerate(offs2)], list(offs2), (n, n))
W2 = sp.csr_matrix(O2 + O2.T + sp.identity(n) * 60.0)
W2.sort_indices()
b = torch.ones(n, dtype=torch.float64, device="cuda:0")
for M in (W, W2):
    Wd = sparse.DeviceCSR.from_scipy(M)
    for block in (False, True):
        G = multigrid.GaussSeidel(Wd, "forward", block=block)
        x = torch.zeros_like(b)
        G.sweep(x, b, 1)
        torch.cuda.synchronize()
        print("max row", int(np.diff(M.indptr).max()), "block", block, float(x.sum()))
