"""Throughput of the V-cycle on every BASELINE.json configuration (1 GPU), next to the oracle's
scipy cycle on the host (1 thread) — the per-config table of DESIGN.md §7.

  python tools/bench_configs.py [--steps 50] [--cpu-cycles 5] [--out gpurun_out/configs.json]

Configs: C1 1D N=1024 two-level (tiny; GPU launch-bound), C2 2D 5-point
1024^2, C3 P1 on cylflow-highres refined x4^3 (817k DoF), C4 3D 7-point 216^3, C5 Voronoi jump
coefficients on a 1024^2 grid. One line of JSON per config plus a summary file.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "ml-amg_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def matrices():
    from mlamg import mesh, problems
    m = mesh.load_npz(os.path.join(ROOT, "tests", "golden", "cylflow_highres_mesh.npz"))
    yield "C1", "1D Poisson N=1024", lambda: problems.poisson_1d(1024), 64
    yield "C2", "2D 5-point 1024^2", lambda: problems.poisson_2d_5pt(1024), 2000
    yield ("C3", "P1 Laplacian, cylflow-highres x4^3 (red refinement)",
           lambda: mesh.poisson_dirichlet(mesh.refine(mesh.refine(mesh.refine(m))))[0], 2000)
    yield "C4", "3D 7-point 216^3", lambda: problems.poisson_3d_7pt(216), 2000
    yield ("C5", "Voronoi jump coefficients, 1024^2 grid",
           lambda: problems.jump_2d(1024, problems.voronoi_jumps(np.random.RandomState(0))), 2000)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--cpu-cycles", type=int, default=5)
    ap.add_argument("--only", default="")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "configs.json"))
    ap.add_argument("--aggregation", default="reference", choices=("reference", "bellman_ford"))
    ap.add_argument("--done-ab", action="store_true",
                    help="also time every config with the per-kernel stop-flag test forced on "
                         "(mlamg_hier_set_done_check 1; interleaved with the default)")
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()
    from mlamg.hierarchy import Hierarchy
    from bench import cpu_baseline
    rows = []
    for key, desc, make, max_coarse in matrices():
        if args.only and key not in args.only.split(","):
            continue
        A = make()
        n = A.shape[0]
        H = Hierarchy.build(A, alpha=0.1, max_coarse=max_coarse, aggregation=args.aggregation,
                            coarse_order="sorted")
        x0 = np.random.RandomState(0).randn(n)
        x0 /= np.linalg.norm(x0)
        b = torch.zeros(n, dtype=torch.float64, device="cuda")
        x = torch.as_tensor(x0).cuda()
        hist = H.cycle(b, x, 10)
        H.cycle_async(b, x, 5)
        torch.cuda.synchronize()
        from mlamg._lib import call

        def timed():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            H.cycle_async(b, x, args.steps)
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) / args.steps

        ab = {}
        if args.done_ab:
            # interleaved A/B, best of 3 each (same hierarchy, same graph shape)
            ts = {0: [], 1: []}
            for _ in range(3):
                for mode in (1, 0):
                    call("mlamg_hier_set_done_check", H.handle, mode)
                    H.cycle_async(b, x, 3)
                    ts[mode].append(timed())
            call("mlamg_hier_set_done_check", H.handle, 0)
            ab = {"done_check_always_ms": round(min(ts[1]) * 1e3, 4),
                  "done_check_notol_ms": round(min(ts[0]) * 1e3, 4)}
            dt = min(ts[0])
        else:
            dt = timed()
        cps = (float("nan") if args.no_cpu
               else cpu_baseline(H, np.zeros(n), x0, args.cpu_cycles)[0])
        row = {"config": key, "workload": desc, "n": n, "nnz": int(A.nnz),
               "levels": H.n_levels, "operator_complexity": round(H.operator_complexity(), 3),
               "setup_s": round(H.timings["total"], 3), "gpu_vcycles_per_s": round(1 / dt, 2),
               "ms_per_cycle": round(dt * 1e3, 4),
               "cycle_hbm_frac": round(H.cycle_bytes(stored=True) / dt / 1e9 / 8000.0, 4),
               "cycle_csr_equivalent_GBps": round(H.cycle_bytes() / dt / 1e9, 1),
               "conv_factor_10cycles": round(float((hist[-1] / hist[-4]) ** (1 / 3)), 5),
               "cpu_vcycles_per_s_1thread": round(cps, 3),
               "gpu_over_cpu": round((1 / dt) / cps, 1),
               "formats": [{k: v[0] for k, v in f.items()} for f in H.formats()],
               "aggregation": args.aggregation, **ab}
        print(json.dumps(row), flush=True)
        rows.append(row)
        del H
        torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(rows, fh, indent=1)


if __name__ == "__main__":
    main()
