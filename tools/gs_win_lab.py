"""Windowed Gauss-Seidel sweep timing on 2D 5-point grids: per-sweep and per-level time of one
launch of `reps` sweeps (A/B of lab variants with MLAMG_LIB=...). Run on the GPU box."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ml-amg_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mlamg import multigrid, problems, sparse  # noqa: E402

tag = os.path.basename(os.environ.get("MLAMG_LIB", "default"))
for m in [int(a) for a in sys.argv[1:]] or (128, 192, 256):
    A = problems.poisson_2d_5pt(m)
    n = A.shape[0]
    G = multigrid.GaussSeidel(sparse.as_device(A))
    xd = torch.zeros(n, dtype=torch.float64, device="cuda")
    bd = torch.as_tensor(np.random.RandomState(0).randn(n)).cuda()
    G.sweep(xd, bd, 2)
    torch.cuda.synchronize()
    reps = 50
    t0 = time.perf_counter()
    G.sweep(xd, bd, reps)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / reps
    print(f"{tag} {m}^2: {t * 1e6:.1f} us/sweep, {t * 1e9 / (2 * m - 1):.0f} ns/level", flush=True)
