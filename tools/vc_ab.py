"""A/B of the sorted format's value codes on C4's A_1 (VERDICT r04 Next #3): cold time of the
residual epilogue (the cycle's A_1 pass) in 'sorted' (fp64 values) and 'sorted' + value codes,
plus how many of the most frequent values cover the entries (the LDS-staged hot table).

  MLAMG_LIB=<variant.so> python tools/vc_ab.py [--n 216]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ml-amg_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=216)
    ap.add_argument("--tag", default=os.environ.get("MLAMG_LIB", "default"))
    args = ap.parse_args()
    from mlamg import problems
    from mlamg.hierarchy import Hierarchy
    A = problems.poisson_3d_7pt(args.n)
    H = Hierarchy.build(A, alpha=0.1, max_coarse=2000, aggregation="reference",
                        coarse_order="sorted", finalize=False)
    M = H.levels[1].A
    dev = torch.device("cuda")
    flush = torch.ones(Hierarchy.FLUSH_BYTES // 8, dtype=torch.float64, device=dev)
    x = torch.randn(M.shape[1], dtype=torch.float64, device=dev)
    y = torch.zeros(M.shape[0], dtype=torch.float64, device=dev)
    out = {"tag": os.path.basename(args.tag), "rows": M.shape[0], "nnz": M.nnz}
    for fmt, arg in (("sorted", 0), ("sorted", 2), ("sorted", 0), ("sorted", 2)):
        t = Hierarchy._time_format(M, fmt, arg, x, y, reps=9, kind="A", flush=flush)
        out.setdefault(f"{fmt}/{arg}_us", []).append(round(t, 2))
        out[f"{fmt}/{arg}_bytes"] = M.format_bytes()
    v = M.to_scipy().data
    _, cnt = np.unique(v.view(np.uint64), return_counts=True)
    c = np.cumsum(np.sort(cnt)[::-1]) / v.size
    out["top_k_coverage"] = {k: round(float(c[min(k, c.size) - 1]), 4)
                             for k in (64, 256, 512, 1024, 2048, 4096, 16384, 61440)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
