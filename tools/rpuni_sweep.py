"""Launch-shape sweep of the uniform stencil kernel (k_rowpat_uni) on the C4 fine operator:
chunks per workgroup (MLAMG_RPU_CH) and an LDS pad that caps workgroups per CU
(MLAMG_RPU_LDSPAD), and the plane-marching form (rpm=0|1, mch=2|4 chunks, seg planes per
segment; MLAMG_RPM*), y = A x timed cold by its dispatch packet (mlamg_timer_*, a 512 MB read
before each launch) and back to back; outputs compared bitwise with the first configuration.

  python tools/rpuni_sweep.py [n3=216] ch=4,pad=0 ch=2,pad=0 ...
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ml-amg_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from mlamg import problems
    from mlamg._lib import call
    from mlamg.sparse import DeviceCSR
    torch.cuda.set_device(0)
    args = sys.argv[1:]
    n3 = int(args.pop(0)) if args and args[0].isdigit() else 216
    cfgs = args or ["ch=4,pad=0"]
    A = problems.poisson_3d_7pt(n3)
    n = A.shape[0]
    flush = torch.ones(64 << 20, dtype=torch.float64, device="cuda")
    sink = torch.empty((), dtype=torch.float64, device="cuda")
    x = torch.as_tensor(np.random.RandomState(0).randn(n)).cuda()
    y = torch.empty_like(x)
    tm = ctypes.c_void_p()
    call("mlamg_timer_create", ctypes.byref(tm))
    ms = ctypes.c_float()
    ref = None
    for cfg in cfgs:
        kv = dict(t.split("=") for t in cfg.split(","))
        os.environ["MLAMG_RPU_CH"] = kv.get("ch", "4")
        os.environ["MLAMG_RPU_LDSPAD"] = kv.get("pad", "0")
        os.environ["MLAMG_RPM"] = kv.get("rpm", "1")        # plane-marching form
        os.environ["MLAMG_RPM_CH"] = kv.get("mch", "4")
        os.environ["MLAMG_RPM_SEG"] = kv.get("seg", "0")
        os.environ["MLAMG_RPM_PF"] = kv.get("pf", "1")
        M = DeviceCSR.from_scipy(A, check=False).set_format("rowpat")
        M.matvec(x, out=y)
        torch.cuda.synchronize()
        out = y.cpu().numpy().view(np.int64).copy()
        if ref is None:
            ref = out
        cold = []
        for _ in range(20):
            torch.sum(flush, dim=0, out=sink)
            call("mlamg_timer_arm", tm)
            M.matvec(x, out=y)
            call("mlamg_timer_elapsed_ms", tm, ctypes.byref(ms))
            cold.append(ms.value * 1e3)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            M.matvec(x, out=y)
        e1.record()
        e1.synchronize()
        warm = e0.elapsed_time(e1) * 1e3 / 50
        fb = M.format_bytes()
        print(f"{cfg:18s} cold mean {np.mean(cold):6.2f} median {np.median(cold):6.2f} us "
              f"({fb / np.mean(cold) / 1e3 / 8e3:.3f} of 8 TB/s) warm {warm:6.2f} us "
              f"bitwise {np.array_equal(out, ref)}", flush=True)
        del M
    call("mlamg_timer_destroy", tm)


if __name__ == "__main__":
    main()
