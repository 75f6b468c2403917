"""A/B timing of the fused amg_2_v engine (run once per library with MLAMG_LIB=...): the
48-grid 32^2-64^2 batch (best of 5) and single calls at 64^2 / 96^2 / 128^2 (best of 5)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ml-amg_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from mlamg import multigrid, problems  # noqa: E402
import oracle.restated as orc  # noqa: E402
from tools.amg2v_timing import make_farm  # noqa: E402


def best(f, reps=5):
    f()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        t.append(time.perf_counter() - t0)
    return round(min(t) * 1e3, 3)


def main():
    torch.cuda.set_device(0)
    out = {"lib": os.environ.get("MLAMG_LIB", "in-tree")}
    probs = make_farm()
    out["batch48_ms"] = best(lambda: multigrid.amg_2_v_batch(probs, res_tol=1e-10))
    for m in (32, 48, 64, 96, 128):
        A = problems.poisson_2d_5pt(m)
        P, _ = orc.smoothed_aggregation_jacobi(A, problems.box_aggregates_2d(m, m, 3),
                                               omega=2.0 / 3.0)
        x0 = np.random.RandomState(0).randn(A.shape[0])
        b = np.zeros(A.shape[0])
        out[f"single{m}_ms"] = best(lambda: multigrid.amg_2_v(A, P, b, x0, res_tol=1e-10,
                                                              engine="fused"))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
