"""Practical HBM ceilings on this device for the fine-level SpMV's traffic shape: a cold read of
80 MB plus a write of 80 MB (y = f(x) elementwise, the bytes of the C4 fine SpMV without the
stencil), a cold read-only pass and a cold write-only pass, each after a 512 MB flush read, timed
with events. Context for the roofline fraction (the guide's 8 TB/s is the peak, not what a
read+write stream reaches).

  python tools/copy_ceiling.py [--n 10077696] [--reps 20] [--out FILE]
"""
import argparse
import json
import statistics

import torch


def timed(fn, flush, reps):
    s = torch.cuda.current_stream()
    sink = torch.empty((), dtype=flush.dtype, device=flush.device)
    out = []
    for _ in range(reps):
        torch.sum(flush, dim=0, out=sink)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        fn()
        e1.record(s)
        e1.synchronize()
        out.append(e0.elapsed_time(e1) * 1e3)
    return statistics.median(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10077696)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    x = torch.randn(a.n, dtype=torch.float64, device=dev)
    y = torch.empty_like(x)
    flush = torch.ones(512 << 17, dtype=torch.float64, device=dev)
    nb = 8 * a.n
    res = {}
    us = timed(lambda: y.copy_(x), flush, a.reps)
    res["copy_read_write"] = {"us": us, "bytes": 2 * nb, "GBps": 2 * nb / us / 1e3}
    us = timed(lambda: torch.mul(x, 1.5, out=y), flush, a.reps)
    res["scale_read_write"] = {"us": us, "bytes": 2 * nb, "GBps": 2 * nb / us / 1e3}
    sink = torch.empty((), dtype=torch.float64, device=dev)
    us = timed(lambda: torch.sum(x, dim=0, out=sink), flush, a.reps)
    res["read_only"] = {"us": us, "bytes": nb, "GBps": nb / us / 1e3}
    us = timed(lambda: y.fill_(1.0), flush, a.reps)
    res["write_only"] = {"us": us, "bytes": nb, "GBps": nb / us / 1e3}
    for k, v in res.items():
        v["frac_of_8TBps"] = v["GBps"] / 8000.0
        print(k, {kk: round(vv, 3) for kk, vv in v.items()})
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
