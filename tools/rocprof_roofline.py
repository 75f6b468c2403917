"""The roofline kernel's launches in a rocprofv3 kernel trace of bench.py, against bench.py's own
HIP-event figure (host-side analysis).

  python tools/rocprof_roofline.py <kernel_trace.csv> <bench.json line file> [out_stats.csv]

bench.py times the fine-level SpMV cold: 20 launches, each right after a 512 MB torch.sum (the
cache flush) and timed by its own dispatch packet's events, then 20 more between stream events. Those launches are found in the trace as the kernels that start right after a
torch reduce kernel and whose name is the roofline kernel's (the first one launched after a
flush); their mean duration is what bench.py's avg_launch_us measures. Writes a rocprofv3-style
stats row for exactly those launches and prints the agreement.
"""
import csv
import json
import statistics
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    line = [ln for ln in open(sys.argv[2]) if ln.startswith("{")][-1]
    bench = json.loads(line)["roofline"]
    picked = []
    for a, b in zip(rows, rows[1:]):
        if "reduce_kernel" in a["Kernel_Name"] and "mlamg::" in b["Kernel_Name"]:
            picked.append(b)
    names = {r["Kernel_Name"] for r in picked}
    # the roofline window: the last 20 flush-preceded launches of the fine level's plain SpMV
    # (y = A x: epilogue 0, no norm) in the bench's format — the autotune flushes before its
    # timings too, earlier, and the variable-coefficient line after it uses other formats
    fam = {"rowpat": ("k_rowpat_uni<0, false", "k_rowpair<0, false"), "sell": ("k_sell<0, false",),
           "sell_dict": ("k_sell_dict<0, false",), "sorted": ("k_sorted<0, false",),
           "csr_stream": ("k_csr_stream<0, false",)}
    fmt = bench["kernel"].split("(")[1].split()[0]
    keys = fam.get(fmt, ("<0, false",))
    cand = [r for r in picked if any(k in r["Kernel_Name"] for k in keys)]
    name = cand[-1]["Kernel_Name"]
    # bench.py times 20 launches by their dispatch packets, then 20 between stream events
    same = [r for r in cand if r["Kernel_Name"] == name][-40:-20]
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in same]
    mean_us = statistics.mean(d) / 1e3
    med_us = statistics.median(d) / 1e3
    b_us = bench["avg_launch_us"]
    print(f"kernel: {name[:110]}")
    print(f"flush-preceded launches found: {len(picked)} ({len(names)} kernel names); window {len(d)}")
    print(f"rocprof mean {mean_us:.2f} us, median {med_us:.2f} us; bench avg_launch_us {b_us:.2f}"
          f" -> rocprof/bench = {mean_us / b_us:.4f}")
    frac = bench["algorithmic_bytes_per_launch"] / (mean_us * 1e-6) / 8e12
    print(f"frac from the rocprof mean: {frac:.4f} (bench {bench['frac']})")
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w", newline="") as fh:
            w = csv.writer(fh, quoting=csv.QUOTE_NONNUMERIC)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MedianNs", "MinNs",
                        "MaxNs", "StdDev", "BenchAvgLaunchNs", "RocprofOverBench"])
            w.writerow([name, len(d), sum(d), statistics.mean(d), statistics.median(d), min(d),
                        max(d), statistics.pstdev(d), b_us * 1e3, mean_us / b_us])


if __name__ == "__main__":
    main()
