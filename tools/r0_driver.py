"""Restriction R_0 r of the bench hierarchy (C4 216^3) launched repeatedly on its own stream
position: the workload of tools/pmc_r0.py's counter passes. Prints the format bytes.
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
    A = problems.poisson_3d_7pt(216)
    H = Hierarchy.build(A, alpha=0.1, strength_mode="invabs", max_coarse=2000)
    R = H.levels[0].R
    r = torch.randn(R.shape[1], dtype=torch.float64, device="cuda")
    y = torch.empty(R.shape[0], dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    for _ in range(20):
        R.matvec(r, out=y)
    torch.cuda.synchronize()
    print(f"r0_driver: format {R.get_format()} bytes {R.format_bytes():.0f} rows {R.shape[0]} "
          f"nnz {R.nnz}", flush=True)


if __name__ == "__main__":
    main()
