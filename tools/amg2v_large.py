"""Two-level amg_2_v beyond the fused engine's limits (n > 16384: the per-operation hierarchy
engine) against the CPU restatement on one core: 160^2 .. 256^2, box aggregates of 3."""
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ml-amg_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from mlamg import multigrid, problems  # noqa: E402
from mlamg.hierarchy import Hierarchy  # noqa: E402
import oracle.restated as orc  # noqa: E402

torch.cuda.set_device(0)
if os.environ.get("DENSE_MAX"):  # A/B: the two-level coarse solve's dense-inverse limit
    Hierarchy.TWO_LEVEL_DENSE_MAX = int(os.environ["DENSE_MAX"])
for m in [int(a) for a in sys.argv[1:]] or (160, 192, 256):
    A = problems.poisson_2d_5pt(m)
    P, _ = orc.smoothed_aggregation_jacobi(A, problems.box_aggregates_2d(m, m, 3), omega=2.0 / 3.0)
    x0 = np.random.RandomState(0).randn(A.shape[0])
    b = np.zeros(A.shape[0])
    row = {"grid": f"{m}^2", "n": A.shape[0], "n_c": P.shape[1],
           "dense_max": Hierarchy.TWO_LEVEL_DENSE_MAX}
    multigrid.amg_2_v(A, P, b, x0, res_tol=1e-10)
    gc.collect()  # a full collection costs ~30 ms with torch loaded: not inside the first call
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        out = multigrid.amg_2_v(A, P, b, x0, res_tol=1e-10)
        ts.append(time.perf_counter() - t0)
    row["device_ms"] = round(float(np.median(ts)) * 1e3, 2)  # median of 5 calls
    row["device_ms_all"] = [round(t * 1e3, 1) for t in ts]
    row["iters"] = out[3]
    t0 = time.perf_counter()
    ref = orc.amg_2_v(A, P, b, x0, res_tol=1e-10)
    row["cpu_1core_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
    row["iters_cpu"] = ref[3]
    print(json.dumps(row), flush=True)
