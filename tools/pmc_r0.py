"""HBM traffic of the restriction R_0 (the bench hierarchy's fine-level R = P_0^T, gather-sorted
format) from rocprofv3 PMC counters, as tools/pmc_traffic.py does for the fine SpMV: separate
FETCH_SIZE and WRITE_SIZE passes (counters only), reads doubled per the gfx950 note
(MI355X_MICROARCH.md §HBM; an upper bound for 4/8-byte-per-lane streams), the R_0 dispatches
picked as the k_sorted<0,...> launches of the largest grid, the first (cold) one skipped.

  python tools/pmc_r0.py r03   ->  gpurun_out/pmc/r0_pmc.json
"""
import csv
import glob
import json
import os
import shutil
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out", "pmc")


def run_pass(counter):
    d = os.path.join(OUT, f"r0_{counter}")
    shutil.rmtree(d, ignore_errors=True)
    os.makedirs(d, exist_ok=True)
    cmd = ["rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "run", "--",
           sys.executable, os.path.join(ROOT, "tools", "r0_driver.py")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        raise RuntimeError(f"rocprofv3 failed:\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}")
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if "k_sorted<0" in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                    rows.append((int(row.get("Grid_Size", 0)), int(row.get("Dispatch_Id", 0)),
                                 float(row["Counter_Value"])))
    gmax = max(g for g, _, _ in rows)
    vals = [v for g, _, v in sorted(rows, key=lambda t: t[1]) if g == gmax]
    drv = [ln for ln in r.stdout.splitlines() if ln.startswith("r0_driver:")]
    return vals, gmax, (drv[-1] if drv else "")


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r03"
    fetch, grid, drv = run_pass("FETCH_SIZE")
    write, _, _ = run_pass("WRITE_SIZE")
    f = statistics.median(fetch[1:] or fetch) * 1024.0  # KiB -> bytes
    w = statistics.median(write[1:] or write) * 1024.0
    fmt_bytes = float(drv.split("bytes")[1].split()[0]) if "bytes" in drv else None
    rec = {"kernel": "R_0 = P_0^T (k_sorted<0,...>)", "round": tag, "grid": grid,
           "dispatches": len(fetch), "fetch_bytes_raw": f, "fetch_bytes_x2": 2 * f,
           "write_bytes": w, "traffic_bytes": 2 * f + w, "format_bytes": fmt_bytes,
           "traffic_over_format": (2 * f + w) / fmt_bytes if fmt_bytes else None,
           "driver": drv}
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, "r0_pmc.json"), "w") as fh:
        json.dump(rec, fh, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
