"""The C4 fine operator (216^3 7-point) in the row-pair pattern format, y = A x 20 times: the
workload of counter passes on k_rowpair / k_rowpair_win (MLAMG_RP_WIN=0/1 picks the kernel)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ml-amg_amd")]


def main():
    import torch
    from mlamg import problems
    from mlamg.sparse import DeviceCSR
    torch.cuda.set_device(0)
    n = int(os.environ.get("RP_N", "216"))
    A = DeviceCSR.from_scipy(problems.poisson_3d_7pt(n)).set_format("rowpat")
    x = torch.randn(A.shape[1], dtype=torch.float64, device="cuda")
    y = torch.empty(A.shape[0], dtype=torch.float64, device="cuda")
    A.matvec(x, out=y)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        A.matvec(x, out=y)
    e1.record()
    torch.cuda.synchronize()
    print(f"rowpat_driver: n={n} win={os.environ.get('MLAMG_RP_WIN', '1')} "
          f"us {e0.elapsed_time(e1) * 1e3 / 20:.2f}", flush=True)


if __name__ == "__main__":
    main()
