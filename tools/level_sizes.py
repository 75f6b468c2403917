"""Rows, nonzeros, format and stored bytes of every operator of the bench hierarchy (C4 216^3).

  python tools/level_sizes.py [n]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ml-amg_amd")]


def main():
    import torch
    from mlamg import problems
    from mlamg.hierarchy import Hierarchy
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 216
    torch.cuda.set_device(0)
    A = problems.poisson_3d_7pt(n)
    H = Hierarchy.build(A, alpha=0.1, strength_mode="invabs", max_coarse=2000)
    for l, L in enumerate(H.levels):
        for name in ("A", "P", "R"):
            M = getattr(L, name, None)
            if M is None:
                continue
            r, c = M.shape
            nnz = M.nnz if hasattr(M, "nnz") else None
            print(f"level {l} {name}: {r} x {c}, nnz {nnz}, nnz/row {nnz / max(r, 1):.1f}, "
                  f"format {M.get_format()}, bytes {M.format_bytes() / 1e6:.2f} MB", flush=True)
    print("coarse", H.coarse_n if hasattr(H, "coarse_n") else "?")


if __name__ == "__main__":
    main()
