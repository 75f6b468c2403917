"""Device GMRES (Hierarchy.gmres, the PyAMG PC's Krylov loop) wall time per solve on a few
operators: inner steps, ms per solve, ms per inner step (host wall clock, after a warm-up).

  python tools/gmres_timing.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ml-amg_amd")]

import numpy as np  # noqa: E402


def main():
    import torch
    from mlamg import problems
    from mlamg.hierarchy import Hierarchy
    torch.cuda.set_device(0)
    for name, A in (("p2d_256", problems.poisson_2d_5pt(256)), ("p2d_1024", problems.poisson_2d_5pt(1024)),
                    ("p3d_48", problems.poisson_3d_7pt(48))):
        H = Hierarchy.build(A, alpha=0.1, max_coarse=500)
        b = torch.as_tensor(np.random.RandomState(7).randn(A.shape[0])).cuda()
        for rtol, restart in ((1e-6, 20), (1e-10, 100)):
            x, st = H.gmres(b, rtol=rtol, restart=restart, maxiter=1, return_info=True)
            torch.cuda.synchronize()
            reps = 5
            t0 = time.perf_counter()
            for _ in range(reps):
                x, st = H.gmres(b, rtol=rtol, restart=restart, maxiter=1, return_info=True)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / reps * 1e3
            it = st["inner_iters"]
            print(f"gmres {name} n={A.shape[0]} rtol={rtol:g} restart={restart}: {it} steps, "
                  f"{ms:.2f} ms/solve, {ms / max(it, 1):.3f} ms/step, "
                  f"presid[-1]={st['presid'][-1] if len(st['presid']) else 0:.3e}", flush=True)


if __name__ == "__main__":
    main()
