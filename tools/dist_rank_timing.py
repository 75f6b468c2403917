"""One rank's device work in the distributed C4 cycle at world W, timed on a single GPU with the
timing-only communicator (mlamg.distributed.NullComm: halos, allgather and all-reduce skipped,
so results are invalid): the compute floor of the W-GPU cycle, before any communication cost.

    python tools/dist_rank_timing.py [--n 216] [--worlds 1,2,4,8] [--steps 50]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ml-amg_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mlamg import problems  # noqa: E402
from mlamg.distributed import DistributedHierarchy, NullComm  # noqa: E402
from mlamg.hierarchy import Hierarchy  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=216)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--min-rows", default="50000", help="comma list of dist_min_rows values")
    ap.add_argument("--overlap", default="1", help="comma list: halo/interior overlap off (0) / on (1)")
    ap.add_argument("--overlap-min-rows", default="2000000",
                    help="comma list of DistributedHierarchy overlap_min_rows values (-1: none)")
    ap.add_argument("--ranks", default="", help="comma list of ranks (default: first, middle, "
                                                "last)")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    A = problems.poisson_3d_7pt(a.n)
    # the bench's hierarchy (bench.py defaults): reference aggregation, coarse rows in seed order
    H = Hierarchy.build(A, alpha=0.1, strength_mode="invabs", max_coarse=2000,
                        aggregation="reference", coarse_order="sorted")
    n = A.shape[0]
    xd = torch.zeros(n, dtype=torch.float64, device="cuda")
    bd = torch.zeros(n, dtype=torch.float64, device="cuda")
    H.cycle(bd, xd, 3)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    H.cycle_async(bd, xd, a.steps)
    torch.cuda.synchronize()
    single = (time.perf_counter() - t0) / a.steps
    out = {"n": n, "single_gpu_ms_per_cycle": round(single * 1e3, 4), "ranks": []}
    print(json.dumps(out), flush=True)
    for w, mr, omr in [(w, mr, omr) for w in map(int, a.worlds.split(","))
                       for mr in map(int, a.min_rows.split(","))
                       for omr in map(int, a.overlap_min_rows.split(","))]:
        ranks = ([int(x) for x in a.ranks.split(",") if int(x) < w] if a.ranks
                 else sorted({0, w // 2, w - 1}))
        for r in ranks:
            c = NullComm(w, r)
            D = DistributedHierarchy(H, c, min_rows=mr, A_host=A,
                                     overlap_min_rows=None if omr < 0 else omr)
            for ov in map(int, a.overlap.split(",")):
                D.set_overlap(ov)
                D.set_cycle_graph(True)
                x = D.new_x(torch.zeros(D.n_own, dtype=torch.float64))
                b = torch.zeros(D.n_own, dtype=torch.float64, device="cuda")
                D.cycle(b, x, 3, history=False)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                D.cycle(b, x, a.steps, history=False)
                torch.cuda.synchronize()
                t = (time.perf_counter() - t0) / a.steps
                row = {"world": w, "rank": r, "min_rows": mr, "overlap_min_rows": omr,
                       "K": D.K, "rows": D.n_own,
                       "overlap": ov, "splits": [(s["level"], s["op"]) for s in D.splits],
                       "compute_ms_per_cycle": round(t * 1e3, 4),
                       "compute_bound_cycles_per_s": round(1.0 / t, 1),
                       "local_formats": [x["chosen"] for x in D.tuning],
                       "partition_s": {k: round(v, 3) for k, v in D.setup_times.items()}}
                out["ranks"].append(row)
                print(json.dumps(row), flush=True)
            del D
            c.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
