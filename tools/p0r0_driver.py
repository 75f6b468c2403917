"""Run the C4 level-0 prolongation (x += P0 e) and restriction (r_c = R0 r) 30 times each in the
sorted format, after building the hierarchy without autotune: the program profiled by
tools/p0r0_pmc.sh (rocprofv3 --pmc passes). GPU box only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "ml-amg_amd")):
    sys.path.insert(0, p)


def main():
    import torch
    from mlamg import problems
    from mlamg._lib import call, ptr, stream_ptr
    from mlamg.hierarchy import Hierarchy
    H = Hierarchy.build(problems.poisson_3d_7pt(216), alpha=0.1, max_coarse=2000,
                        fine_format="csr_stream", finalize=False)
    L = H.levels[0]
    L.P.set_format("sorted")
    L.R.set_format("sorted")
    e = torch.randn(L.P.shape[1], dtype=torch.float64, device="cuda")
    x = torch.randn(L.P.shape[0], dtype=torch.float64, device="cuda")
    rc = torch.empty_like(e)
    s = stream_ptr()
    for _ in range(30):
        call("mlamg_prolong_add", L.P.handle, ptr(e), ptr(x), s)
    for _ in range(30):
        call("mlamg_restrict", L.R.handle, ptr(x), ptr(rc), s)
    torch.cuda.synchronize()
    print(f"p0r0_driver: P0 {L.P.format_bytes():.0f} B + y read {8.0 * L.P.shape[0]:.0f}; "
          f"R0 {L.R.format_bytes():.0f} B", flush=True)


if __name__ == "__main__":
    main()
