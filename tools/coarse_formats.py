"""A/B of the SpMV kernels on the coarse operators of the C4 hierarchy (GPU box): every level's
A (residual epilogue, as in the cycle), P (x += P e) and R (y = R r) in each format, HIP events
on torch's stream, plus a bitwise check of every scipy-order format against CSR-stream.

  python tools/coarse_formats.py [n=216] [--levels 1 2 3] [--out gpurun_out/coarse_formats.json]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "ml-amg_amd")):
    sys.path.insert(0, p)

FORMATS = (("csr_stream", 0), ("sorted", 0), ("long", 0), ("vector", 64), ("vector", 128),
           ("vector", 256), ("vector", 512))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("n", nargs="?", type=int, default=216)
    ap.add_argument("--levels", type=int, nargs="*", default=None)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "coarse_formats.json"))
    args = ap.parse_args()
    import torch
    from mlamg import problems
    from mlamg._lib import MLAMG_EUNSUPPORTED, MlamgError, call, ptr, stream_ptr
    from mlamg.hierarchy import Hierarchy

    H = Hierarchy.build(problems.poisson_3d_7pt(args.n), alpha=0.1, max_coarse=2000,
                        fine_format="csr_stream")
    s = stream_ptr()

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / args.reps * 1e3

    out = []
    levels = args.levels if args.levels is not None else range(1, len(H.levels))
    for l in levels:
        L = H.levels[l]
        for name, M in (("A", L.A), ("P", L.P), ("R", L.R)):
            x = torch.randn(M.shape[1], dtype=torch.float64, device="cuda")
            y0 = torch.randn(M.shape[0], dtype=torch.float64, device="cuda")
            y = torch.empty_like(y0)
            if name == "A":
                def op():
                    call("mlamg_residual", M.handle, ptr(y0), ptr(x), ptr(y), None, s)
            elif name == "P":
                def op():
                    y.copy_(y0)
                    call("mlamg_prolong_add", M.handle, ptr(x), ptr(y), s)
            else:
                def op():
                    M.matvec(x, out=y)
            row = {"level": l, "op": name, "rows": M.shape[0], "nnz": M.nnz, "us": {},
                   "bitwise_vs_csr_stream": {}}
            ref = None
            for fmt, arg in FORMATS:
                try:
                    M.set_format(fmt, arg)
                except MlamgError as e:
                    if e.code != MLAMG_EUNSUPPORTED:
                        raise
                    continue
                key = f"{fmt}/{arg}"
                op()
                torch.cuda.synchronize()
                res = y.clone()
                if ref is None:
                    ref = res
                else:
                    row["bitwise_vs_csr_stream"][key] = bool(torch.equal(res, ref))
                if name == "P":
                    t = timed(op) - timed(lambda: y.copy_(y0))
                else:
                    t = timed(op)
                row["us"][key] = round(t, 2)
                row.setdefault("bytes", {})[key] = M.format_bytes()
            print(json.dumps(row), flush=True)
            out.append(row)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
