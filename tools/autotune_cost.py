"""Wall time of the format autotune per operator and candidate (format build + timed launches)
on the C4 hierarchy: where the setup's `formats` phase goes.

  python tools/autotune_cost.py [--n 216] [--out FILE]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ml-amg_amd")]

import torch  # noqa: E402

from mlamg import problems  # noqa: E402
from mlamg.hierarchy import Hierarchy  # noqa: E402
from mlamg.sparse import DeviceCSR  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=216)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    A = problems.poisson_3d_7pt(a.n)
    H = Hierarchy.build(A, alpha=0.1, max_coarse=2000, aggregation="reference",
                        coarse_order="sorted", finalize=False)
    rows = []
    orig_set, orig_time = DeviceCSR.set_format, Hierarchy._time_format
    cur = {}

    def set_format(self, fmt, vec_width=0):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = orig_set(self, fmt, vec_width)
        torch.cuda.synchronize()
        cur["build_s"] = cur.get("build_s", 0.0) + time.perf_counter() - t0
        return r

    def time_format(M, fmt, arg, x, y, reps=5, kind="A", flush=None):
        cur.clear()
        t0 = time.perf_counter()
        row = {"kind": kind, "rows": M.shape[0], "nnz": M.nnz, "cand": f"{fmt}/{arg}"}
        try:
            us = orig_time(M, fmt, arg, x, y, reps=reps, kind=kind, flush=flush)
        except Exception as e:  # a refused format: its build time is what it cost
            torch.cuda.synchronize()
            row.update(refused=str(e)[:80], wall_s=round(time.perf_counter() - t0, 4))
            rows.append(row)
            raise
        row.update(us=round(us, 2), wall_s=round(time.perf_counter() - t0, 4),
                   build_s=round(cur.get("build_s", 0.0), 4))
        rows.append(row)
        return us

    DeviceCSR.set_format = set_format
    Hierarchy._time_format = staticmethod(time_format)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    H.apply_formats("autotune", "auto")
    torch.cuda.synchronize()
    total = time.perf_counter() - t0
    DeviceCSR.set_format, Hierarchy._time_format = orig_set, staticmethod(orig_time)
    for r in rows:
        print(r)
    print({"apply_formats_s": round(total, 3),
           "timed_candidates_s": round(sum(r["wall_s"] for r in rows if "us" in r), 3),
           "refused_s": round(sum(r["wall_s"] for r in rows if "refused" in r), 3)})
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"apply_formats_s": total, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
