"""Distributed setup (mlamg/dsetup.py) vs the replicated build at C4, on ONE GPU (run on the
GPU box): world 1 with the world-1 transport, and worlds 2 / 4 / 8 with the ranks as threads
taking turns on the device — each rank's own work (ThreadComm.busy_s: the time it held the
device, its waits excluded) is what one GPU of a world-W job would spend, minus the transfers.

  python tools/dsetup_timing.py [--n 216] [--worlds 1,2,4,8] [--aggregation reference]
Prints one JSON line per configuration."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ml-amg_amd"), ROOT]
import torch  # noqa: E402
from mlamg import dsetup, partition, problems  # noqa: E402
from mlamg.hierarchy import Hierarchy  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=216)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--aggregation", default="reference")
    ap.add_argument("--min-rows", type=int, default=50000)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    A = problems.poisson_3d_7pt(a.n)
    n = A.shape[0]
    kw = dict(alpha=0.1, strength_mode="invabs", max_coarse=2000, aggregation=a.aggregation)
    # the replicated path: the whole build, then one rank's maps (build_levels_torch)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    H = Hierarchy.build(A, coarse_order="sorted", **kw)
    torch.cuda.synchronize()
    t_build = time.perf_counter() - t0
    K = 1
    while K < len(H.levels) and H.levels[K].A.shape[0] >= a.min_rows:
        K += 1

    def tc(M):
        crow, col, val = M.to_torch()
        return partition.TCSR(crow, col, val, M.shape)

    t1 = time.perf_counter()
    partition.build_levels_torch([tc(H.levels[l].A) for l in range(K)],
                                 [tc(H.levels[l].P) for l in range(K)],
                                 [tc(H.levels[l].R) for l in range(K)],
                                 [H.levels[l].seeds for l in range(K)], 8, 0)
    torch.cuda.synchronize()
    print(json.dumps({"path": "replicated", "n": n, "build_s": round(t_build, 3),
                      "build_phases": {k: round(v, 3) for k, v in H.timings.items()},
                      "maps_rank0_of_8_s": round(time.perf_counter() - t1, 3),
                      "lams": [L.lam for L in H.levels[:K]]}), flush=True)
    lams_ref = [L.lam for L in H.levels]
    del H
    torch.cuda.empty_cache()
    for w in [int(x) for x in a.worlds.split(",")]:
        def fn(comm):
            S = dsetup.build_distributed(dsetup.split_rows(A, w, comm.rank), n, comm,
                                         A0_global=A if a.aggregation == "reference" else None,
                                         min_rows=a.min_rows, **kw)
            return S.times, S.lams, len(S.parts), S.bf_sweeps, S.lanczos_iters
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if w == 1:
            out = [fn(dsetup.SoloComm())]
            busy = [time.perf_counter() - t0]
        else:
            comms = []

            def fn2(comm):
                comms.append(comm)
                return fn(comm)
            out = dsetup.run_threads(w, fn2)
            busy = [c.busy_s for c in sorted(comms, key=lambda c: c.rank)]
        wall = time.perf_counter() - t0
        rel = max(abs(x - y) / abs(y) for x, y in zip(out[0][1], lams_ref))
        print(json.dumps({"path": "distributed", "world": w, "wall_s_all_ranks": round(wall, 3),
                          "rank_busy_s": [round(b, 3) for b in busy],
                          "rank0_phases": out[0][0], "partitioned_levels": out[0][2],
                          "bf_sweeps": out[0][3], "lanczos_iters": out[0][4],
                          "lam_max_rel_diff_vs_single": rel}), flush=True)
        del out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
