"""Per-rank local operators of the C4 partition on ONE GPU (no RCCL): for world W and a few
ranks, build the partition maps (mlamg.partition.build_levels), upload every rank's local A/P/R,
autotune their kernels (mlamg.distributed.tune_local) and report the chosen formats and the
local kernel times — the device work one rank of the W-GPU cycle does, without the exchanges.

    python tools/dist_local_ops.py [--n 216] [--world 8] [--ranks 0,4]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ml-amg_amd")]

import torch  # noqa: E402

from mlamg import partition, problems  # noqa: E402
from mlamg.distributed import tune_local  # noqa: E402
from mlamg.hierarchy import Hierarchy  # noqa: E402
from mlamg.sparse import DeviceCSR  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=216)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--ranks", default="0,4")
    ap.add_argument("--min-rows", type=int, default=50000)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    A = problems.poisson_3d_7pt(a.n)
    H = Hierarchy.build(A, alpha=0.1, strength_mode="invabs", max_coarse=1000)
    K = 1
    while K < len(H.levels) and H.levels[K].A.shape[0] >= a.min_rows:
        K += 1
    As = [A] + [H.levels[l].A.to_scipy() for l in range(1, K)]
    Ps = [H.levels[l].P.to_scipy() for l in range(K)]
    seeds = [H.levels[l].seeds for l in range(K)]
    out = {"n": A.shape[0], "world": a.world, "K": K, "global": H.formats(), "ranks": {}}
    for r in map(int, a.ranks.split(",")):
        t0 = time.perf_counter()
        parts = partition.build_levels(As, Ps, seeds, a.world, r)
        tp = time.perf_counter() - t0
        rows = []
        for l, p in enumerate(parts):
            row = {"rows": p["hi"] - p["lo"]}
            for kind, key, Mg in (("A", "A_loc", H.levels[l].A), ("P", "P_loc", H.levels[l].P),
                                  ("R", "R_own", H.levels[l].R)):
                M = DeviceCSR.from_scipy(p[key], check=False)
                _, t = tune_local(Mg, M, kind)
                fixed, _ = tune_local(Mg, DeviceCSR.from_scipy(p[key], check=False), kind,
                                      autotune=False)
                row[kind] = {"chosen": t["chosen"], "us": t.get("us"),
                             "global_format_would_be": "/".join(map(str, fixed.get_format()[:2]))}
            rows.append(row)
        out["ranks"][r] = {"partition_s": round(tp, 1), "levels": rows}
        print(json.dumps({r: out["ranks"][r]}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
