"""HBM traffic of the roofline kernel from rocprofv3 PMC counters (run on the GPU box).

Two separate passes (FETCH_SIZE costs 3 TCC slots, WRITE_SIZE 2: they cannot share one pass),
counters only, no tracing domains. Both report KiB per dispatch. gfx950 correction
(/opt/skills/guides/MI355X_MICROARCH.md §HBM): FETCH_SIZE counts exactly half the bytes of a
wide coalesced streaming read, so reads are doubled; WRITE_SIZE is exact for streaming stores.
This parent process never touches the GPU (rocprofv3 runs the driver as a child).

Usage: pmc_traffic.py <round> [csr_stream|sell]. Writes gpurun_out/pmc/spmv_c4_pmc_<fmt>.json
and the raw counter CSVs (only gpurun_out/ comes back from the GPU box); they are then committed
as profiles/spmv_c4_pmc_<fmt>.json (read by bench.py as roofline.traffic for the format the
fine-level autotune chose) and profiles/<round>/.
"""
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out", "pmc")
KERNELS = {"csr_stream": "k_csr_stream", "sell": "k_sell<", "sorted": "k_sorted",
           "sell_dict": "k_sell_dict", "rowpat": "k_rowpa"}


def run_pass(counter, fmt, tag=""):
    d = os.path.join(OUT, f"{counter.replace(' ', '+')}_{fmt}{tag}")
    shutil.rmtree(d, ignore_errors=True)
    os.makedirs(d, exist_ok=True)
    cmd = ["rocprofv3", "--pmc", *counter.split(), "--output-format", "csv", "-d", d, "-o", "run", "--",
           sys.executable, os.path.join(ROOT, "tools", "spmv_driver.py")]
    env = dict(os.environ, MLAMG_FMT=fmt)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    if r.returncode != 0:
        raise RuntimeError(f"rocprofv3 failed:\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}")
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise RuntimeError(f"no counter_collection.csv under {d}")
    vals = []
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if KERNELS[fmt] in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                    vals.append(float(row["Counter_Value"]))
                elif (" " in counter and KERNELS[fmt] in row.get("Kernel_Name", "")
                      and row.get("Counter_Name") in counter.split()):
                    vals.append((row["Counter_Name"], float(row["Counter_Value"])))
    drv = [ln for ln in r.stdout.splitlines() if ln.startswith("spmv_driver:")]
    return vals, files, (drv[-1] if drv else "")


def main():
    round_tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    fmt = sys.argv[2] if len(sys.argv) > 2 else "sell"
    # PMC_TAG names a variant run (e.g. MLAMG_RP_UNI=0 in the environment: the general row-pair
    # kernel); PMC_L2=1 adds a third pass with the L2 hit / miss counts
    tag = os.environ.get("PMC_TAG", "")
    fetch, f1, drv = run_pass("FETCH_SIZE", fmt, tag)
    write, f2, _ = run_pass("WRITE_SIZE", fmt, tag)
    l2 = {}
    if os.environ.get("PMC_SQ") == "1":  # where the waves' time goes (quad-cycle units)
        names = ("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY "
                 "SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS")
        v, _, _ = run_pass(names, fmt, tag)
        for name in names.split():
            xs = sorted(x for nm, x in v if nm == name)
            if xs:
                l2[name + "_median"] = xs[len(xs) // 2]
    if os.environ.get("PMC_L2") == "1":
        v, _, _ = run_pass("TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum", fmt, tag)
        for name in ("TCC_HIT_sum", "TCC_MISS_sum", "TCC_EA0_RDREQ_sum"):
            xs = sorted(x for nm, x in v if nm == name)
            if xs:
                l2[name + "_median"] = xs[len(xs) // 2]
    if not fetch or not write:
        raise RuntimeError("no dispatches of the SpMV kernel found in the counter CSVs")
    # skip the first (cold) dispatch
    fk = sorted(fetch[1:] or fetch)
    wk = sorted(write[1:] or write)
    fetch_kib = fk[len(fk) // 2]
    write_kib = wk[len(wk) // 2]
    read_bytes = 2.0 * fetch_kib * 1024.0
    write_bytes = write_kib * 1024.0
    n = 216 ** 3
    nnz = 70263936
    csr_algo = 12.0 * nnz + 4.0 * (n + 1) + 8.0 * n + 8.0 * n
    algo = float(drv.split("format_bytes=")[1].split()[0]) if "format_bytes=" in drv else csr_algo
    res = {
        "kernel": f"{KERNELS[fmt]}<EPI_AXPBY> (fine-level SpMV, C4 216^3, format {fmt})",
        "format": fmt,
        "fetch_size_kib_median": fetch_kib,
        "write_size_kib_median": write_kib,
        "correction": "reads = 2 x FETCH_SIZE (gfx950 wide-read under-count), writes = WRITE_SIZE",
        "hbm_read_bytes_per_launch": read_bytes,
        "hbm_write_bytes_per_launch": write_bytes,
        "hbm_bytes_per_launch": read_bytes + write_bytes,
        "algorithmic_bytes_per_launch": algo,
        "csr_algorithmic_bytes_per_launch": csr_algo,
        "driver": drv,
        "traffic_over_algorithmic": (read_bytes + write_bytes) / algo,
        "dispatches": len(fetch),
        **l2,
    }
    with open(os.path.join(OUT, f"spmv_c4_pmc_{fmt}{tag}.json"), "w") as fh:
        json.dump(res, fh, indent=1)
    for f, ctr in ((f1[0], "FETCH_SIZE"), (f2[0], "WRITE_SIZE")):
        shutil.copy(f, os.path.join(OUT, f"spmv_c4_pmc_{fmt}{tag}_{ctr}_{round_tag}.csv"))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
