"""Level-0 aggregate agreement: the hierarchy's order-independent Bellman-Ford rule vs the
reference's push-order sweeps (ns/lib/graph.py:40-51, the "dumb" recipe of
utils/evaluate_dataset.py:80-90), at full size on C2, C4 and C5 (VERDICT r04 Next #1).

For each config: strength C = invabs(A), seeds = RandomState(0).permutation(n)
[:ceil(0.1 n)]; the device runs both rules from the same seeds (mlamg_bellman_ford_canon and
mlamg_bellman_ford); reported: the fraction of nodes whose aggregate seed agrees, the number of
aggregates that are the same node set under both rules, sweeps and wall times; and, for the
push order, a bitwise check of (distance, nearest seed) against the oracle's C transcription of
the reference loop (oracle/oracle.c ref_bellman_ford_torch, pinned to the reference's own
modified_bellman_ford output in tests/golden/reference_vectors.npz).

  python tools/agg_agreement.py [--only C2,C4,C5] [--out profiles/r05/agg_agreement.json]
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "ml-amg_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def configs():
    from mlamg import problems
    yield "C2", "2D 5-point 1024^2", lambda: problems.poisson_2d_5pt(1024)
    yield "C4", "3D 7-point 216^3", lambda: problems.poisson_3d_7pt(216)
    yield ("C5", "Voronoi jump coefficients, 1024^2 grid",
           lambda: problems.jump_2d(1024, problems.voronoi_jumps(np.random.RandomState(0))))


def same_sets(lab_a, lab_b):
    """Aggregates (seed -> node set) identical under both labelings."""
    n = lab_a.size
    # an aggregate is identical iff every node of it under a has the same label under b and
    # the sizes agree
    ok_node = lab_a == lab_b
    k_a = np.bincount(lab_a[lab_a >= 0], minlength=n)
    k_b = np.bincount(lab_b[lab_b >= 0], minlength=n)
    bad = np.zeros(n, dtype=bool)
    bad[lab_a[~ok_node & (lab_a >= 0)]] = True
    bad[lab_b[~ok_node & (lab_b >= 0)]] = True
    seeds = np.nonzero(k_a > 0)[0]
    return int(np.sum(~bad[seeds] & (k_a[seeds] == k_b[seeds]))), int(seeds.size)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    ap.add_argument("--alpha", type=float, default=0.1)
    ap.add_argument("--no-oracle", action="store_true")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "agg_agreement.json"))
    args = ap.parse_args()
    from mlamg.graph import bellman_ford_device, modified_bellman_ford_device
    from mlamg.hierarchy import strength
    from mlamg.sparse import DeviceCSR
    rows = []
    for key, desc, make in configs():
        if args.only and key not in args.only.split(","):
            continue
        A = make()
        n = A.shape[0]
        Ad = DeviceCSR.from_scipy(A, check=False)
        C = strength(Ad, "invabs")
        k = int(math.ceil(args.alpha * n))
        seeds = np.random.RandomState(0).permutation(n)[:k]
        sd = torch.as_tensor(seeds.astype(np.int32)).cuda()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dr, lr, sw_r = modified_bellman_ford_device(C, sd)
        torch.cuda.synchronize()
        t_ref = time.perf_counter() - t0
        t0 = time.perf_counter()
        dc, lc, sw_c = bellman_ford_device(C, torch.as_tensor(np.sort(seeds).astype(np.int32)).cuda())
        torch.cuda.synchronize()
        t_can = time.perf_counter() - t0
        lab_r, lab_c = lr.cpu().numpy(), lc.cpu().numpy()
        d_r, d_c = dr.cpu().numpy(), dc.cpu().numpy()
        n_same, n_agg = same_sets(lab_r, lab_c)
        row = {"config": key, "workload": desc, "n": n, "nnz": int(A.nnz), "seeds": k,
               "strength": "invabs", "seed_rule": "RandomState(0).permutation(n)[:ceil(0.1 n)]",
               "label_agreement": round(float(np.mean(lab_r == lab_c)), 6),
               "nodes_differing": int(np.sum(lab_r != lab_c)),
               "aggregates_identical": n_same, "aggregates": n_agg,
               "aggregates_identical_frac": round(n_same / max(n_agg, 1), 6),
               "distances_bitwise_equal": bool(np.array_equal(d_r, d_c)),
               "push_order_sweeps": sw_r, "canonical_sweeps": sw_c,
               "push_order_device_s": round(t_ref, 3), "canonical_device_s": round(t_can, 3),
               "unreached_nodes": int(np.sum(lab_r < 0))}
        if not args.no_oracle:
            from oracle import restated as orc
            t0 = time.perf_counter()
            d_o, near_o, sw_o = orc.modified_bellman_ford(C.to_scipy(), seeds)
            row["oracle_push_s"] = round(time.perf_counter() - t0, 3)
            row["device_push_vs_oracle_bitwise"] = bool(
                np.array_equal(d_o, d_r) and np.array_equal(near_o, lab_r.astype(np.int64))
                and sw_o == sw_r)
        print(json.dumps(row), flush=True)
        rows.append(row)
        del C, Ad, dr, lr, dc, lc
        torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(rows, fh, indent=1)


if __name__ == "__main__":
    main()
