"""C4 level-0 prolongation (x += P0 e) and restriction (r_c = R0 r) in the sorted format: HIP
event time per launch over 30 launches each (A/B of lab variants via MLAMG_LIB). GPU box only."""
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
    tag = os.path.basename(os.environ.get("MLAMG_LIB", "default"))
    for name, fn, nbytes in (
            ("P0", lambda: call("mlamg_prolong_add", L.P.handle, ptr(e), ptr(x), s),
             L.P.format_bytes() + 8.0 * L.P.shape[0]),
            ("R0", lambda: call("mlamg_restrict", L.R.handle, ptr(x), ptr(rc), s),
             L.R.format_bytes())):
        for _ in range(5):
            fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(30):
            fn()
        b.record()
        torch.cuda.synchronize()
        us = a.elapsed_time(b) / 30 * 1e3
        print(f"{tag} {name}: {us:.1f} us, {nbytes / us / 1e3:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
