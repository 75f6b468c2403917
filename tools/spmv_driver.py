"""Run only the fine-level C4 SpMV (the roofline kernel) `reps` times — the program profiled by
tools/pmc_traffic.py and tools/profile.sh under rocprofv3."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "ml-amg_amd")):
    sys.path.insert(0, p)


def main():
    import torch
    from mlamg import problems
    from mlamg.sparse import DeviceCSR

    n1 = int(os.environ.get("MLAMG_N", "216"))
    reps = int(os.environ.get("MLAMG_REPS", "20"))
    fmt = os.environ.get("MLAMG_FMT", "auto_exact")  # bench.py's autotune picks sell for C4
    A = DeviceCSR.from_scipy(problems.poisson_3d_7pt(n1), check=False).set_format(fmt)
    x = torch.randn(A.shape[1], dtype=torch.float64, device="cuda")
    y = torch.empty(A.shape[0], dtype=torch.float64, device="cuda")
    A.matvec(x, out=y)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        A.matvec(x, out=y)
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    print(f"spmv_driver: n={A.shape[0]} nnz={A.nnz} reps={reps} format={A.get_format()} "
          f"avg {us:.1f} us format_bytes={A.format_bytes():.0f}")


if __name__ == "__main__":
    main()
