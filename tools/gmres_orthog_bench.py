"""Wall time of the PyAMG PC's Krylov apply on the pyamg_sa hierarchy: Householder GMRES
(pyamg.krylov.gmres's default, Hierarchy.gmres_householder) against the restarted-MGS GMRES
(Hierarchy.gmres), both one cycle of at most 100 steps to tol 1e-8, from a zero guess.

  python tools/gmres_orthog_bench.py [--case poisson2d:1024 ...] [--reps 3] [--out FILE]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ml-amg_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mlamg import problems  # noqa: E402
from mlamg.hierarchy import Hierarchy  # noqa: E402


def make(case):
    kind, n = case.split(":")
    n = int(n)
    return problems.poisson_2d_5pt(n) if kind == "poisson2d" else problems.poisson_3d_7pt(n)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", action="append", default=None)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = []
    for case in a.case or ["poisson2d:1024", "poisson3d:128"]:
        A = make(case)
        H = Hierarchy.pyamg_sa(A)
        b = torch.as_tensor(np.random.default_rng(0).standard_normal(A.shape[0]), device="cuda:0")
        row = {"case": case, "rows": A.shape[0], "levels": H.n_levels}
        for name, fn in (
                ("householder", lambda: H.gmres_householder(b, tol=1e-8, maxiter=100,
                                                            return_info=True)),
                ("mgs", lambda: H.gmres(b, rtol=1e-8, restart=100, maxiter=1,
                                        return_info=True))):
            fn()
            ts = []
            for _ in range(a.reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                x, info = fn()
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            xr = x.cpu().numpy()
            bn = b.cpu().numpy()
            row[name] = {"ms": round(1e3 * min(ts), 2),
                         "steps": info.get("iters", info.get("inner_iters")),
                         "info": info["info"],
                         "true_relres": float(np.linalg.norm(bn - A @ xr) / np.linalg.norm(bn))}
        t0 = time.perf_counter()
        for _ in range(a.reps):
            H.precondition(b)
        torch.cuda.synchronize()
        row["vcycle_ms"] = round(1e3 * (time.perf_counter() - t0) / a.reps, 2)
        print(json.dumps(row), flush=True)
        rows.append(row)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
