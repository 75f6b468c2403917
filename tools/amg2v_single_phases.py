"""Phase breakdown of single fused amg_2_v calls (MLAMG_BATCH_TIMING=1: host phases and the
device's per-phase wall clocks go to stderr) next to the Python call's own time."""
import os
import sys
import time

os.environ["MLAMG_BATCH_TIMING"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ml-amg_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from mlamg import multigrid, problems  # noqa: E402
import oracle.restated as orc  # noqa: E402

torch.cuda.set_device(0)
for m in [int(a) for a in sys.argv[1:]] or (32, 64, 96):
    A = problems.poisson_2d_5pt(m)
    P, _ = orc.smoothed_aggregation_jacobi(A, problems.box_aggregates_2d(m, m, 3), omega=2.0 / 3.0)
    x0 = np.random.RandomState(0).randn(A.shape[0])
    b = np.zeros(A.shape[0])
    for rep in range(3):
        t0 = time.perf_counter()
        out = multigrid.amg_2_v(A, P, b, x0, res_tol=1e-10, engine="fused")
        sys.stderr.flush()
        print(f"{m}^2 rep {rep}: python call {1e3 * (time.perf_counter() - t0):.3f} ms, "
              f"iters {out[3]}", flush=True)
        sys.stdout.flush()
