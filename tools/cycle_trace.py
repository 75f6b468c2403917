"""Per-kernel breakdown of one V-cycle from a rocprofv3 kernel trace (host-side analysis).

  python tools/cycle_trace.py gpurun_out/prof/bench_kernel_trace.csv [cycle_index_from_end]

Cycles are delimited by the end-of-cycle norm kernel (k_finalize_norm); prints each kernel's
duration and the idle gap before it, then the cycle's span and busy time.
"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "k_finalize_norm" in r["Kernel_Name"]]
    i0, i1 = idx[-k - 1], idx[-k]
    seg = rows[i0 + 1:i1 + 1]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
    prev = None
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev else 0.0
        print(f"{gap:7.2f} {(e - s) / 1e3:8.2f}  {r['Kernel_Name'][:100]}")
        prev = e
    print(f"kernels {len(seg)}  span {(t1 - t0) / 1e3:.1f} us  busy {busy / 1e3:.1f} us")


if __name__ == "__main__":
    main()
