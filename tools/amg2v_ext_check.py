"""Single fused amg_2_v calls with the device-wide coarse factor (n_c > 512) against the
one-workgroup coarse setup (MLAMG_BATCH_NO_EXT=1) and the hierarchy engine: times and agreement."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ml-amg_amd"), ROOT]
import torch  # noqa: E402
from mlamg import multigrid, problems  # noqa: E402
import oracle.restated as orc  # noqa: E402


def timed(f, reps=5):
    f()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = f()
    return out, (time.perf_counter() - t0) / reps * 1e3


def main():
    torch.cuda.set_device(0)
    for m in [int(a) for a in sys.argv[1:]] or (64, 96, 128):
        A = problems.poisson_2d_5pt(m)
        P, _ = orc.smoothed_aggregation_jacobi(A, problems.box_aggregates_2d(m, m, 3),
                                               omega=2.0 / 3.0)
        n = A.shape[0]
        x0 = np.random.RandomState(0).randn(n)
        b = np.zeros(n)
        row = {"grid": f"{m}^2", "n_c": P.shape[1]}
        res = {}
        for tag, eng, env in (("ext", "fused", None), ("wg", "fused", "1"), ("hier", "hierarchy", None)):
            if env:
                os.environ["MLAMG_BATCH_NO_EXT"] = env
            else:
                os.environ.pop("MLAMG_BATCH_NO_EXT", None)
            out, ms = timed(lambda: multigrid.amg_2_v(A, P, b, x0, res_tol=1e-10, engine=eng))
            res[tag] = out
            row[f"{tag}_ms"] = round(ms, 3)
            row[f"{tag}_iters"] = int(out[3])
        os.environ.pop("MLAMG_BATCH_NO_EXT", None)
        row["ext_vs_wg_maxdiff"] = float(np.max(np.abs(res["ext"][0] - res["wg"][0])))
        row["ext_vs_hier_maxdiff"] = float(np.max(np.abs(res["ext"][0] - res["hier"][0])))
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
