"""Time the C4 fine-level operator's kernels in one storage format (default rowpat): y = A x,
r = b - A x with the norm, two weighted-Jacobi sweeps (attached weights when rowpat), for A/B runs
of kernel variants (MLAMG_LIB=<variant .so>, MLAMG_FMT). GPU box only.

  python tools/rowpat_ops.py [n=216] [reps=30]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "ml-amg_amd")):
    sys.path.insert(0, p)


def main():
    import torch
    from mlamg import problems
    from mlamg._lib import call, ptr, stream_ptr
    from mlamg.sparse import DeviceCSR

    n1 = int(sys.argv[1]) if len(sys.argv) > 1 else 216
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    fmt = os.environ.get("MLAMG_FMT", "rowpat")
    A = DeviceCSR.from_scipy(problems.poisson_3d_7pt(n1), check=False).set_format(fmt)
    n = A.shape[0]
    d = A.diag_inv(2.0 / 3.0)
    attached = A.attach_dinv(d) if fmt == "rowpat" else False
    x = torch.randn(n, dtype=torch.float64, device="cuda")
    b = torch.randn(n, dtype=torch.float64, device="cuda")
    y = torch.empty_like(x)
    t = torch.empty_like(x)
    nrm = torch.zeros(1, dtype=torch.float64, device="cuda")
    ops = {
        "spmv": lambda: A.matvec(x, out=y),
        "resid+norm": lambda: call("mlamg_residual", A.handle, ptr(b), ptr(x), ptr(y), ptr(nrm),
                                   stream_ptr()),
        "2 jacobi": lambda: call("mlamg_jacobi", A.handle, ptr(d), ptr(b), ptr(x), ptr(t), 2,
                                 stream_ptr()),
    }
    out = []
    for name, fn in ops.items():
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        out.append(f"{name} {e0.elapsed_time(e1) / reps * 1e3:.1f} us")
    print(f"rowpat_ops[{os.path.basename(os.environ.get('MLAMG_LIB', 'default'))}, fmt={fmt}, "
          f"attached={attached}]: " + ", ".join(out), flush=True)


if __name__ == "__main__":
    main()
