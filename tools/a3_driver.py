"""The level-3 Galerkin operator A_3 of the bench hierarchy (C4 216^3, 10,078 rows, ~709 entries
per row, CSR-vector family) applied 20 times: the workload of counter passes on the vector kernel.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ml-amg_amd")]


def main():
    import torch
    from mlamg import problems
    from mlamg.hierarchy import Hierarchy
    torch.cuda.set_device(0)
    lvl = int(os.environ.get("A3_LEVEL", "3"))
    op = os.environ.get("A3_OP", "A")
    H = Hierarchy.build(problems.poisson_3d_7pt(216), alpha=0.1, strength_mode="invabs",
                        max_coarse=2000)
    M = getattr(H.levels[lvl], op)
    x = torch.randn(M.shape[1], dtype=torch.float64, device="cuda")
    y = torch.empty(M.shape[0], dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        M.matvec(x, out=y)
    e1.record()
    torch.cuda.synchronize()
    print(f"a3_driver: level {lvl} {op} format {M.get_format()} bytes {M.format_bytes():.0f} "
          f"us {e0.elapsed_time(e1) * 1e3 / 20:.2f}", flush=True)


if __name__ == "__main__":
    main()
