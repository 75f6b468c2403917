"""Distinct-value statistics of the C4 hierarchy's coarse operators (VERDICT r04 Weak #3 / Next
#3): for A_1, A_2 (and A_3): nnz, distinct values, how many of the most frequent values cover
50/90/99/99.9/100 % of the entries, and per-block distinct counts (blocks of 4096 consecutive
stored entries, the sorted format's streaming order is CSR order here), plus the column-offset
range |j - i| (bits an index delta needs).

  python tools/value_stats.py [--n 216] [--out profiles/r05/value_stats.json]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "ml-amg_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402


def stats(M, block=4096):
    v = M.data
    nnz = v.size
    u, inv, cnt = np.unique(v.view(np.uint64), return_inverse=True, return_counts=True)
    order = np.sort(cnt)[::-1]
    cum = np.cumsum(order) / nnz
    cover = {f"{int(q * 1000) / 10}%": int(np.searchsorted(cum, q) + 1)
             for q in (0.5, 0.9, 0.99, 0.999)}
    cover["100%"] = int(u.size)
    nb = (nnz + block - 1) // block
    per_block = np.empty(nb, dtype=np.int64)
    for b in range(nb):
        per_block[b] = np.unique(inv[b * block:(b + 1) * block]).size
    rows = np.repeat(np.arange(M.shape[0]), np.diff(M.indptr))
    off = np.abs(M.indices.astype(np.int64) - rows)
    return {"rows": int(M.shape[0]), "nnz": int(nnz), "distinct": int(u.size),
            "distinct_frac": round(u.size / nnz, 5), "top_values_covering": cover,
            "block": block, "block_distinct_mean": round(float(per_block.mean()), 1),
            "block_distinct_max": int(per_block.max()),
            "col_offset_max": int(off.max()),
            "col_offset_le_32767_frac": round(float(np.mean(off <= 32767)), 6),
            "row_len_mean": round(nnz / M.shape[0], 2), "row_len_max": int(np.diff(M.indptr).max())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=216)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "value_stats.json"))
    args = ap.parse_args()
    from mlamg import problems
    from mlamg.hierarchy import Hierarchy
    A = problems.poisson_3d_7pt(args.n)
    H = Hierarchy.build(A, alpha=0.1, max_coarse=2000, aggregation="reference",
                        coarse_order="sorted", finalize=False)
    res = {"config": f"C4 {args.n}^3, aggregation='reference' (sorted coarse order)"}
    for l in range(1, len(H.levels)):
        M = H.levels[l].A.to_scipy()
        res[f"A{l}"] = stats(M)
        print(l, json.dumps(res[f"A{l}"]), flush=True)
        Pm = H.levels[l].P.to_scipy()
        res[f"P{l}"] = {"nnz": int(Pm.nnz), "distinct": int(np.unique(Pm.data).size)}
        del M, Pm
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
