"""Exact lexicographic Gauss-Seidel (pyamg semantics) on the device vs the oracle's C sweep
(the restated pyamg amg_core loop, 1 thread) on 2D 5-point grids; and the reference driver
amg_2_v (GS smoother) end to end. Run on the GPU box."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ml-amg_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mlamg import multigrid, problems, sparse  # noqa: E402
from oracle import restated as orc  # noqa: E402

for m in (48, 128, 256, 512, 1024):
    A = problems.poisson_2d_5pt(m)
    n = A.shape[0]
    b = np.random.RandomState(0).randn(n)
    x = np.zeros(n)
    G = multigrid.GaussSeidel(sparse.as_device(A))
    xd = torch.zeros(n, dtype=torch.float64, device="cuda")
    bd = torch.as_tensor(b).cuda()
    G.sweep(xd, bd, 1)
    torch.cuda.synchronize()
    reps = 20 if m <= 256 else 5
    t0 = time.perf_counter()
    G.sweep(xd, bd, reps)
    torch.cuda.synchronize()
    tg = (time.perf_counter() - t0) / reps
    t0 = time.perf_counter()
    for _ in range(3):
        orc.gauss_seidel(A, x, b, iterations=1)
    tc = (time.perf_counter() - t0) / 3
    print(f"{m}^2 n={n}: device GS sweep {tg*1e3:.3f} ms, oracle C sweep (1 thread) {tc*1e3:.3f} ms", flush=True)
