"""A/B of the uniform row-pair stencil kernel (k_rowpat_uni) against k_rowpair on the C4 (216^3)
and C2 (1024^2) fine operators: every epilogue the V-cycle uses, outputs compared bitwise, device
times cold (a 512 MB read before each launch) and back to back (HIP events, 20 launches each).

  python tools/rpuni_ab.py [n3=216] [n2=1024]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ml-amg_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def timed(fn, flush, reps=20):
    s = torch.cuda.current_stream()
    sink = torch.empty((), dtype=torch.float64, device="cuda")
    fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for e0, e1 in ev:
        torch.sum(flush, dim=0, out=sink)
        e0.record(s)
        fn()
        e1.record(s)
    torch.cuda.synchronize()
    cold = float(np.mean([a.elapsed_time(b) for a, b in ev])) * 1e3
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return cold, e0.elapsed_time(e1) * 1e3 / reps


def main():
    from mlamg import problems
    from mlamg._lib import call, ptr, stream_ptr
    from mlamg.sparse import DeviceCSR
    torch.cuda.set_device(0)
    n3 = int(sys.argv[1]) if len(sys.argv) > 1 else 216
    n2 = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    flush = torch.ones(64 << 20, dtype=torch.float64, device="cuda")
    for name, A in (("C4", problems.poisson_3d_7pt(n3)), ("C2", problems.poisson_2d_5pt(n2))):
        n = A.shape[0]
        mats = {}
        for tag, env in (("pair", "0"), ("uni", "1")):
            os.environ["MLAMG_RP_UNI"] = env
            M = DeviceCSR.from_scipy(A).set_format("rowpat")
            d = M.diag_inv(2.0 / 3.0)
            att = M.attach_dinv(d)
            mats[tag] = (M, d, att)
        rs = np.random.RandomState(0)
        x = torch.as_tensor(rs.randn(n)).cuda()
        b = torch.as_tensor(rs.randn(n)).cuda()
        outs = {}
        for tag, (M, d, att) in mats.items():
            y = torch.empty(n, dtype=torch.float64, device="cuda")
            r = torch.empty_like(y)
            nrm = torch.zeros(1, dtype=torch.float64, device="cuda")
            xt = torch.empty_like(y)
            xj = x.clone()
            s = stream_ptr()
            ops = {
                "spmv": lambda: M.matvec(x, out=y),
                "resid+norm": lambda: call("mlamg_residual", M.handle, ptr(b), ptr(x), ptr(r),
                                           ptr(nrm), s),
                "jacobi(xin=x)": lambda: call("mlamg_jacobi", M.handle, ptr(d), ptr(b), ptr(xj),
                                              ptr(xt), 1, s),
            }
            res = {}
            for op, fn in ops.items():
                xj.copy_(x)
                fn()
                torch.cuda.synchronize()
                val = {"spmv": y, "resid+norm": r, "jacobi(xin=x)": xj}[op].cpu().numpy().copy()
                cold, warm = timed(fn, flush)
                res[op] = (val, cold, warm)
            outs[tag] = res
            print(f"{name} {tag}: format {M.get_format()} dinv attached {att} "
                  f"bytes {M.format_bytes():.0f}", flush=True)
        for op in outs["pair"]:
            vp, cp, wp = outs["pair"][op]
            vu, cu, wu = outs["uni"][op]
            same = np.array_equal(vp.view(np.int64), vu.view(np.int64))
            print(f"{name} {op:15s} k_rowpair cold {cp:7.2f} warm {wp:7.2f} us | k_rowpat_uni "
                  f"cold {cu:7.2f} warm {wu:7.2f} us | bitwise {same}", flush=True)


if __name__ == "__main__":
    main()
