"""End-to-end time of one reference-style amg_2_v call (two-level, GS smoother, res_tol) on small
grids — the per-problem unit of the reference's training/evaluation loops (utils/common.py:77) —
device path vs the oracle's CPU restatement (scipy factorized + the C GS sweep). Run on the GPU
box."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ml-amg_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mlamg import multigrid, problems  # noqa: E402
from oracle import restated as orc  # noqa: E402

torch.cuda.set_device(0)
for m in (32, 48, 96, 192):
    A = problems.poisson_2d_5pt(m)
    Agg = problems.box_aggregates_2d(m, m, 3)
    P, _ = orc.smoothed_aggregation_jacobi(A, Agg, omega=2.0 / 3.0)
    n = A.shape[0]
    x0 = np.random.RandomState(0).randn(n)
    b = np.zeros(n)
    multigrid.amg_2_v(A, P, b, x0, res_tol=1e-10)  # warm
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        x, conv, err, it = multigrid.amg_2_v(A, P, b, x0, res_tol=1e-10)
    tg = (time.perf_counter() - t0) / reps
    t0 = time.perf_counter()
    for _ in range(reps):
        xr, convr, errr, itr = orc.amg_2_v(A, P, b, x0, res_tol=1e-10)
    tc = (time.perf_counter() - t0) / reps
    print(f"{m}^2 n={n} n_c={P.shape[1]}: device amg_2_v {tg*1e3:.1f} ms ({it} it, conv {conv:.5f}); "
          f"CPU restatement {tc*1e3:.1f} ms ({itr} it, conv {convr:.5f})", flush=True)

# throughput of many independent solves (the reference's task farm over a dataset of grids)
probs = []
for i in range(48):
    m = 32 + 16 * (i % 3)
    A = problems.poisson_2d_5pt(m)
    Agg = problems.box_aggregates_2d(m, m, 3)
    P, _ = orc.smoothed_aggregation_jacobi(A, Agg, omega=2.0 / 3.0)
    probs.append((A, P, np.zeros(A.shape[0]), np.random.RandomState(i).randn(A.shape[0])))
t0 = time.perf_counter()
for A, P, b, x0 in probs:
    orc.amg_2_v(A, P, b, x0, res_tol=1e-10)
tc = time.perf_counter() - t0
print(f"48 grids (32^2..64^2): CPU restatement sequential {tc*1e3:.0f} ms ({tc/48*1e3:.2f} ms/grid, 1 core)", flush=True)
for w in (1, 4, 8, 16):
    multigrid.amg_2_v_batch(probs[:8], workers=w, res_tol=1e-10)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    multigrid.amg_2_v_batch(probs, workers=w, res_tol=1e-10)
    torch.cuda.synchronize()
    tg = time.perf_counter() - t0
    print(f"48 grids: device amg_2_v_batch workers={w}: {tg*1e3:.0f} ms ({tg/48*1e3:.2f} ms/grid)", flush=True)
