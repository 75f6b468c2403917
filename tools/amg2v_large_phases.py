"""Setup / cycle split of the large two-level amg_2_v (hierarchy engine, PCG coarse solve when
n_c > TWO_LEVEL_DENSE_MAX): where the 320^2 call's time goes (last table)."""
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
from mlamg.sparse import to_device_vec  # noqa: E402
import oracle.restated as orc  # noqa: E402

torch.cuda.set_device(0)
if os.environ.get("INNER_MAX_COARSE"):  # A/B: where the PCG preconditioner stops coarsening
    Hierarchy.PCG_INNER_MAX_COARSE = int(os.environ["INNER_MAX_COARSE"])
if os.environ.get("INNER_NU"):
    Hierarchy.PCG_INNER_NU = int(os.environ["INNER_NU"])


def T():
    torch.cuda.synchronize()
    return time.perf_counter()


for m in [int(a) for a in sys.argv[1:]] or (320,):
    A = problems.poisson_2d_5pt(m)
    P, _ = orc.smoothed_aggregation_jacobi(A, problems.box_aggregates_2d(m, m, 3), omega=2.0 / 3.0)
    x0 = np.random.RandomState(0).randn(A.shape[0])
    b = np.zeros(A.shape[0])
    multigrid.amg_2_v(A, P, b, x0, res_tol=1e-10)
    H = out = None
    for rep in range(2):
        tf = T()
        H = out = None  # free the previous rep's device objects outside the timed phases
        td = T()
        gc.collect()
        tg = T()
        gc.collect()
        t0 = T()
        free_ms = {"del": round((td - tf) * 1e3, 2), "gc": round((tg - td) * 1e3, 2),
                   "gc_again": round((t0 - tg) * 1e3, 2)}
        H = Hierarchy.two_level(A, P, omega=2.0 / 3.0, smoother="gauss_seidel")
        t1 = T()
        xd = to_device_vec(x0).clone()
        bd = to_device_vec(b)
        t2 = T()
        err = H.cycle(bd, xd, 500, tol=1e-10)
        t3 = T()
        t4 = T()
        out = multigrid.amg_2_v(A, P, b, x0, res_tol=1e-10)
        t5 = T()
        row = {"grid": f"{m}^2", "n_c": P.shape[1], "pcg": H.pcg is not None,
               "inner_max_coarse": Hierarchy.PCG_INNER_MAX_COARSE,
               "inner_nu": Hierarchy.PCG_INNER_NU,
               "inner_levels": len(H.inner.levels) if H.inner is not None else None,
               "coarse_stats": H.coarse_stats(),
               "setup_phases_ms": {k: round(v * 1e3, 2) for k, v in H.timings.items()},
               "inner_build_ms": ({k: round(v * 1e3, 2) for k, v in H.inner.timings.items()
                                   if isinstance(v, float)} if H.inner is not None else None),
               "setup_ms": round((t1 - t0) * 1e3, 2), "free_prev_ms": free_ms, "cycle_ms": round((t3 - t2) * 1e3, 2),
               "cycles": len(err) if hasattr(err, "__len__") else None,
               "amg_2_v_ms": round((t5 - t4) * 1e3, 2), "iters": out[3]}
        print(json.dumps(row), flush=True)
