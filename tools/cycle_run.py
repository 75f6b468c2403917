"""Build one BASELINE configuration's hierarchy and replay its V-cycle (the workload of a
rocprofv3 kernel trace for tools/cycle_trace.py).

  python tools/cycle_run.py C2 [cycles=40]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ml-amg_amd"), os.path.join(ROOT, "tools")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from bench_configs import matrices
    from mlamg.hierarchy import Hierarchy
    key = sys.argv[1] if len(sys.argv) > 1 else "C2"
    cycles = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    torch.cuda.set_device(0)
    for k, desc, make, max_coarse in matrices():
        if k != key:
            continue
        A = make()
        H = Hierarchy.build(A, alpha=0.1, max_coarse=max_coarse, aggregation="reference",
                            coarse_order="sorted")
        if os.environ.get("MLAMG_FACTORED_P0") == "1":
            H.set_factored_prolong(0)  # opt-in factored level-0 prolongation
        n = A.shape[0]
        x0 = np.random.RandomState(0).randn(n)
        x0 /= np.linalg.norm(x0)
        b = torch.zeros(n, dtype=torch.float64, device="cuda")
        x = torch.as_tensor(x0).cuda()
        H.cycle_async(b, x, 5)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        H.cycle_async(b, x, cycles)
        e1.record()
        torch.cuda.synchronize()
        print(f"cycle_run {key} ({desc}): levels {H.n_levels} "
              f"rows {[L.A.shape[0] for L in H.levels] + [H.Ac.shape[0]]} "
              f"formats {H.formats()} {e0.elapsed_time(e1) * 1e3 / cycles:.1f} us/cycle",
              flush=True)


if __name__ == "__main__":
    main()
