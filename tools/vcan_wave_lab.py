"""CSR-vector kernels on the C4 bench hierarchy (216^3): k_csr_vcan (MLAMG_VCAN_WAVE=0) against
the wave-per-row k_vcan_wave with x in LDS (1) and without (2), per coarse operator, in the
cycle's cache state (a 512 MB read before every timed launch) and back to back; outputs compared
bitwise across the kernels. Also times the vector family on the exact-family operators of
levels >= 1 (A_2: 187 entries per row) to place the family rule.

  python tools/vcan_wave_lab.py > gpurun_out/vcan_wave_lab.log
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ml-amg_amd")]


def main():
    import torch
    from mlamg import problems
    from mlamg.hierarchy import Hierarchy
    from mlamg._lib import call, ptr, stream_ptr
    torch.cuda.set_device(0)
    H = Hierarchy.build(problems.poisson_3d_7pt(216), alpha=0.1, strength_mode="invabs",
                        max_coarse=2000, fine_format="autotune")
    dev = torch.device("cuda", 0)
    flush = torch.ones((512 << 20) // 8, dtype=torch.float64, device=dev)
    sink = torch.empty((), dtype=torch.float64, device=dev)
    out = []
    for i, L in enumerate(H.levels):
        if i == 0:
            continue
        for name in ("A", "P", "R"):
            M = getattr(L, name)
            fmt0 = M.get_format()
            g = torch.Generator(device="cpu").manual_seed(1)
            x = torch.randn(M.shape[1], dtype=torch.float64, generator=g).to(dev)
            b = torch.randn(M.shape[0], dtype=torch.float64, generator=g).to(dev)
            y = torch.zeros(M.shape[0], dtype=torch.float64, device=dev)

            def op():
                if name == "A":
                    call("mlamg_residual", M.handle, ptr(b), ptr(x), ptr(y), None, stream_ptr())
                else:
                    M.matvec(x, out=y)

            def timed(cold, reps=7):
                s = torch.cuda.current_stream()
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                      for _ in range(reps)]
                op()
                for e0, e1 in ev:
                    if cold:
                        torch.sum(flush, dim=0, out=sink)
                    e0.record(s)
                    op()
                    e1.record(s)
                ev[-1][1].synchronize()
                return round(statistics.median(a.elapsed_time(c) for a, c in ev) * 1e3, 2)

            rec = {"level": i, "op": name, "rows": M.shape[0], "cols": M.shape[1], "nnz": M.nnz,
                   "format": list(fmt0[:2]), "us": {}}
            if fmt0[0] != "vector":
                rec["us"][f"{fmt0[0]}"] = [timed(True), timed(False)]
                M.set_format("vector", 64)
            ref = None
            for mode in ("0", "1", "2"):
                os.environ["MLAMG_VCAN_WAVE"] = mode
                rec["us"][f"vec_mode{mode}"] = [timed(True), timed(False)]
                op()
                torch.cuda.synchronize()
                cur = y.clone()
                if ref is None:
                    ref = cur
                else:
                    rec[f"bitwise_mode{mode}"] = bool(torch.equal(ref.view(torch.int64),
                                                                  cur.view(torch.int64)))
            os.environ.pop("MLAMG_VCAN_WAVE")
            M.set_format(fmt0[0], int(fmt0[1]))
            out.append(rec)
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
