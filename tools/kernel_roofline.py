"""Per-operator roofline table of the C4 V-cycle (GPU box): every level's A (residual and
weighted-Jacobi epilogues), P (prolongation x += P e) and R (restriction) in the formats the
autotune chose, plus the dense coarse solve, timed with HIP events on torch's stream, next to the
bytes each launch must move (mlamg_csr_format_bytes: the matrix as stored + x once + y once, plus
the epilogue's extra vectors) and the fraction of the 8 TB/s HBM3E peak.

  python tools/kernel_roofline.py [n=216] [--out gpurun_out/kernel_roofline.json]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "ml-amg_amd")):
    sys.path.insert(0, p)

PEAK = 8000.0  # GB/s, MI355X HBM3E spec (/opt/skills/guides/MI355X_MICROARCH.md)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("n", nargs="?", type=int, default=216)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "kernel_roofline.json"))
    args = ap.parse_args()
    import torch
    from mlamg import problems
    from mlamg._lib import call, ptr, stream_ptr
    from mlamg.hierarchy import Hierarchy

    H = Hierarchy.build(problems.poisson_3d_7pt(args.n), alpha=0.1, max_coarse=2000)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / args.reps * 1e3  # us

    rows = []
    s = stream_ptr()
    for l, L in enumerate(H.levels):
        n, nc = L.A.shape[0], L.P.shape[1]
        x = torch.randn(n, dtype=torch.float64, device="cuda")
        b = torch.randn(n, dtype=torch.float64, device="cuda")
        r = torch.empty_like(x)
        t = torch.empty_like(x)
        e = torch.randn(nc, dtype=torch.float64, device="cuda")
        rc = torch.empty(nc, dtype=torch.float64, device="cuda")
        fa, fp, fr = L.A.format_bytes(), L.P.format_bytes(), L.R.format_bytes()
        dinv_attached = L.A.get_format()[0] == "rowpat"
        ops = [
            ("A residual r = b - A x", L.A, fa + 8.0 * n,
             lambda: call("mlamg_residual", L.A.handle, ptr(b), ptr(x), ptr(r), None, s)),
            # two sweeps (ping-pong, no copy-back); bytes of one: + b, + dinv unless attached
            ("A Jacobi x' = x + D(b - A x)", L.A, fa + 8.0 * n + (0.0 if dinv_attached else 8.0 * n),
             lambda: call("mlamg_jacobi", L.A.handle, ptr(L.dinv), ptr(b), ptr(x), ptr(t), 2, s)),
            ("P prolongation x += P e", L.P, fp + 8.0 * n,
             lambda: call("mlamg_prolong_add", L.P.handle, ptr(e), ptr(x), s)),
            ("R restriction r_c = R r", L.R, fr,
             lambda: call("mlamg_restrict", L.R.handle, ptr(r), ptr(rc), s)),
        ]
        for name, M, nbytes, fn in ops:
            us = timed(fn)
            if name.startswith("A Jacobi"):
                us /= 2.0
            fmt, arg, _ = M.get_format()
            gbs = nbytes / us / 1e3
            rows.append({"level": l, "op": name, "format": f"{fmt}/{arg}", "rows": M.shape[0],
                         "nnz": M.nnz, "bytes": nbytes, "us": round(us, 2),
                         "GBps": round(gbs, 1), "frac_of_peak": round(gbs / PEAK, 3)})
    nc = H.Ac.shape[0]
    bc = torch.randn(nc, dtype=torch.float64, device="cuda")
    xc = torch.empty_like(bc)
    us = timed(lambda: call("mlamg_dense_solve", H.dense, ptr(bc), ptr(xc), s))
    nbytes = 8.0 * nc * nc + 16.0 * nc
    rows.append({"level": len(H.levels), "op": "dense coarse x = A_c^-1 b (GEMV)", "format": "dense",
                 "rows": nc, "nnz": nc * nc, "bytes": nbytes, "us": round(us, 2),
                 "GBps": round(nbytes / us / 1e3, 1), "frac_of_peak": round(nbytes / us / 1e3 / PEAK, 3)})
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(rows, fh, indent=1)
    print("| level | operation | format | rows | nnz | MB | µs | GB/s | % of 8 TB/s |")
    print("|---|---|---|---|---|---|---|---|---|")
    for r in rows:
        print(f"| {r['level']} | {r['op']} | {r['format']} | {r['rows']:,} | {r['nnz']:,} | "
              f"{r['bytes'] / 1e6:.0f} | {r['us']:.1f} | {r['GBps']:.0f} | "
              f"{100 * r['frac_of_peak']:.0f} |", flush=True)


if __name__ == "__main__":
    main()
