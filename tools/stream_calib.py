"""Streaming calibration for the roofline kernel: what plain HBM streams of the same size reach
from a cold cache on this box, next to the C4 fine-level SpMV (k_rowpat_uni). Every launch
follows a 512 MB read and sits between a pair of stream events (so each figure carries the same
event + dispatch overhead); the SpMV is also timed by its own dispatch packet (mlamg_timer_*).

  python tools/stream_calib.py [n3=216]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ml-amg_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def cold_events(fn, flush, sink, reps=20):
    s = torch.cuda.current_stream()
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
    return float(np.mean([a.elapsed_time(b) for a, b in ev])) * 1e3


def main():
    from mlamg import problems
    from mlamg._lib import call
    from mlamg.sparse import DeviceCSR
    torch.cuda.set_device(0)
    n3 = int(sys.argv[1]) if len(sys.argv) > 1 else 216
    A = problems.poisson_3d_7pt(n3)
    n = A.shape[0]
    flush = torch.ones(64 << 20, dtype=torch.float64, device="cuda")
    sink = torch.empty((), dtype=torch.float64, device="cuda")
    x = torch.randn(n, dtype=torch.float64, device="cuda")
    z = torch.randn(n, dtype=torch.float64, device="cuda")
    y = torch.empty_like(x)
    M = DeviceCSR.from_scipy(A, check=False).set_format("rowpat")
    fb = M.format_bytes()
    rows = [
        ("copy y = x", lambda: y.copy_(x), 16.0 * n),
        ("add y = x + z", lambda: torch.add(x, z, out=y), 24.0 * n),
        ("read sum(x)", lambda: torch.sum(x, dim=0, out=sink), 8.0 * n),
        ("SpMV y = A x (rowpat)", lambda: M.matvec(x, out=y), fb),
    ]
    for name, fn, nbytes in rows:
        us = cold_events(fn, flush, sink)
        print(f"{name:24s} {nbytes / 1e6:7.1f} MB  cold (stream events) {us:6.2f} us  "
              f"{nbytes / us / 1e6:5.2f} TB/s", flush=True)
    tm = ctypes.c_void_p()
    call("mlamg_timer_create", ctypes.byref(tm))
    ms = ctypes.c_float()
    ts = []
    for _ in range(20):
        torch.sum(flush, dim=0, out=sink)
        call("mlamg_timer_arm", tm)
        M.matvec(x, out=y)
        call("mlamg_timer_elapsed_ms", tm, ctypes.byref(ms))
        ts.append(ms.value * 1e3)
    call("mlamg_timer_destroy", tm)
    print(f"{'SpMV (dispatch packet)':24s} {fb / 1e6:7.1f} MB  cold {np.mean(ts):6.2f} us  "
          f"{fb / np.mean(ts) / 1e6:5.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
