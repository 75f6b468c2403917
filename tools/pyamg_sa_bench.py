"""The PyAMG preconditioner's hierarchy (pyamg smoothed_aggregation_solver recipe,
ns/preconditioner/PyAMG.py:94) on the device: setup phases, V-cycle time and the PC's GMRES
apply (PyAMG.py:119, rtol 1e-8), against the oracle's restatement on the host (scipy + the C
amg_core loops, one thread) for the same problem.

  python tools/pyamg_sa_bench.py --case poisson2d:1024 --case poisson3d:128 --out FILE
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ml-amg_amd")]

import numpy as np  # noqa: E402


def problem(spec):
    import mlamg.problems as P
    kind, size = spec.split(":")
    m = int(size)
    if kind == "poisson2d":
        return P.poisson_2d_5pt(m)
    if kind == "poisson3d":
        return P.poisson_3d_7pt(m)
    if kind == "randcoef3d":
        return P.random_coeff_3d_7pt(m, seed=0, decades=1.0)
    raise ValueError(spec)


def run(spec, cpu=True, cycles=20):
    import torch
    from mlamg.hierarchy import Hierarchy
    A = problem(spec)
    n = A.shape[0]
    dev = torch.device("cuda", 0)
    out = {"case": spec, "n": n, "nnz": int(A.nnz)}
    Hierarchy.pyamg_sa(problem(spec.split(":")[0] + ":16"))  # warm the kernels
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    H = Hierarchy.pyamg_sa(A)
    torch.cuda.synchronize()
    out["setup_s"] = round(time.perf_counter() - t0, 4)
    out["setup_phases_s"] = {k: round(v, 4) for k, v in H.timings.items()}
    out["levels"] = [{"n": L.A.shape[0], "nnz": L.A.nnz, "aggregates": L.n_seeds,
                      "pass1_rounds": L.bf_sweeps, "rho": L.lam,
                      "gs_levels": L.gs.n_levels} for L in H.levels]
    out["coarse_n"] = H.Ac.shape[0]
    rng = np.random.default_rng(0)
    b = rng.standard_normal(n)
    bd = torch.as_tensor(b).to(dev)
    xd = torch.zeros(n, dtype=torch.float64, device=dev)
    H.cycle_async(bd, xd, 2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    H.cycle_async(bd, xd, cycles)
    torch.cuda.synchronize()
    out["vcycle_ms"] = round((time.perf_counter() - t0) / cycles * 1e3, 4)
    hist = H.cycle(bd, torch.zeros_like(bd), 10)
    out["conv_factor_10"] = float((hist[-1] / hist[0]) ** (1 / 9))
    t0 = time.perf_counter()
    x, info = H.gmres(b, rtol=1e-8, restart=100, maxiter=1, return_info=True)
    out["gmres_s"] = round(time.perf_counter() - t0, 4)
    out["gmres_iters"] = info["inner_iters"]
    out["gmres_relres"] = float(np.linalg.norm(b - A @ x) / np.linalg.norm(b))
    if cpu:
        import scipy.linalg
        from oracle import restated as R
        rhos = [L.lam for L in H.levels]
        t0 = time.perf_counter()
        levels, Ac = R.pyamg_sa_setup(A, rhos=rhos)
        pinv = scipy.linalg.pinv(Ac.toarray())
        out["cpu_setup_s_given_rho"] = round(time.perf_counter() - t0, 4)
        x = np.zeros(n)
        k = max(2, min(cycles, 5))
        t0 = time.perf_counter()
        for _ in range(k):
            R.pyamg_sa_vcycle(levels, pinv, b, x)
        out["cpu_vcycle_ms"] = round((time.perf_counter() - t0) / k * 1e3, 3)
        out["cpu_kind"] = "port (oracle restatement: scipy + C amg_core loops, 1 thread)"
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", action="append", default=[])
    ap.add_argument("--out", default=None)
    ap.add_argument("--no-cpu", action="store_true")
    a = ap.parse_args()
    res = []
    for c in a.case or ["poisson2d:512"]:
        r = run(c, cpu=not a.no_cpu)
        print(json.dumps(r), flush=True)
        res.append(r)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
