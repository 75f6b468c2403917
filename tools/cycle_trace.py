"""Per-kernel breakdown of the V-cycle from a rocprofv3 kernel trace (host-side analysis).

  python tools/cycle_trace.py gpurun_out/prof/bench_kernel_trace.csv [n_cycles] [must_contain]

Cycles are delimited by the end-of-cycle norm kernel (k_finalize_norm). Over the last n_cycles
cycles (default 10) that launch the same kernel sequence as the last one, prints each
position's median duration and median idle gap before it, then the median span and busy time
(a single cycle's numbers scatter by a few microseconds per kernel). must_contain: only cycles
launching a kernel whose name contains it (bench.py also runs a variable-coefficient cycle).
"""
import csv
import statistics
import sys


def cycles(rows):
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    fused = not any("k_finalize_norm" in r["Kernel_Name"] for r in rows)
    # the cycle ends with k_finalize_norm, or, with the norm finished inside its pass, with the
    # end-of-cycle residual pass (the only RESID launch with NORM: "<1, true")
    idx = [i for i, r in enumerate(rows)
           if ("<1, true" in r["Kernel_Name"] if fused else "k_finalize_norm" in r["Kernel_Name"])]
    return [rows[a + 1:b + 1] for a, b in zip(idx, idx[1:])]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    cyc = cycles(rows)
    if len(sys.argv) > 3:
        cyc = [c for c in cyc if any(sys.argv[3] in r["Kernel_Name"] for r in c)]
    names = [r["Kernel_Name"] for r in cyc[-1]]
    same = [c for c in cyc if [r["Kernel_Name"] for r in c] == names][-n:]
    durs, gaps, spans, busys = [], [], [], []
    for c in same:
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in c]
        g = [0.0] + [(int(c[i]["Start_Timestamp"]) - int(c[i - 1]["End_Timestamp"])) / 1e3
                     for i in range(1, len(c))]
        durs.append(d)
        gaps.append(g)
        spans.append((int(c[-1]["End_Timestamp"]) - int(c[0]["Start_Timestamp"])) / 1e3)
        busys.append(sum(d))
    for i, name in enumerate(names):
        md = statistics.median(d[i] for d in durs)
        mg = statistics.median(g[i] for g in gaps)
        print(f"{mg:7.2f} {md:8.2f}  {name[:100]}")
    print(f"cycles {len(same)}  kernels {len(names)}  median span {statistics.median(spans):.1f} us"
          f"  busy {statistics.median(busys):.1f} us")


if __name__ == "__main__":
    main()
