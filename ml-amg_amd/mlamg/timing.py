"""Kernel timing for the roofline lines of bench.py (single GPU and every rank of a distributed
run): warm back-to-back launches, and cold launches timed by their own dispatch packet."""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from ._lib import call

_FLUSH = None


def time_kernel(fn, reps=50):
    """Average device time (s) of fn() (one kernel launch on torch's current stream), launches
    back to back between two HIP events: operands may stay cache-resident (warm)."""
    s = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / 1000.0 / reps


def time_kernel_cold(fn, reps=20):
    """Device time of fn() (one SpMV-family kernel launch on torch's current stream) from a cold
    cache: each launch follows a read of a 512 MB buffer (twice the 256 MB MALL, so no operand
    survives in any cache level — what the autotune does before its timings,
    mlamg/hierarchy.py). The kernel is timed by the events of its own dispatch packet
    (mlamg_timer_*, hipExtLaunchKernel): its execution alone, which is what rocprofv3's kernel
    trace reports for the same launches (tools/rocprof_roofline.py). A second round brackets each
    call with a pair of stream events instead (event packet + dispatch + kernel), reported beside
    it. Returns (mean, median, stream-event mean) in s."""
    global _FLUSH
    if _FLUSH is None:
        _FLUSH = torch.ones(64 << 20, dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    sink = torch.empty((), dtype=torch.float64, device="cuda")
    tm = ctypes.c_void_p()
    call("mlamg_timer_create", ctypes.byref(tm))
    ts = []
    try:
        ms = ctypes.c_float()
        for _ in range(reps):
            torch.sum(_FLUSH, dim=0, out=sink)
            call("mlamg_timer_arm", tm)
            try:
                fn()
            finally:
                call("mlamg_timer_disarm")  # fn() that launched nothing timed leaves it unarmed
            call("mlamg_timer_elapsed_ms", tm, ctypes.byref(ms))
            ts.append(ms.value / 1000.0)
    finally:
        call("mlamg_timer_destroy", tm)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for e0, e1 in ev:
        torch.sum(_FLUSH, dim=0, out=sink)
        e0.record(s)
        fn()
        e1.record(s)
    torch.cuda.synchronize()
    te = [e0.elapsed_time(e1) / 1000.0 for e0, e1 in ev]
    return float(np.mean(ts)), float(np.median(ts)), float(np.mean(te))
