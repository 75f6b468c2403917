"""PMC counter study of single SpMV operators (run on the GPU box; never touches the GPU itself).

  python tools/pmc_probe.py DIR OUT.json OP:FMT[:VW] [OP:FMT[:VW] ...]

For each operator and each counter pass in PASSES, runs
  rocprofv3 --pmc <counters> -- python tools/level_driver.py run DIR OP FMT VW
and records the median per-dispatch value of every counter for the SpMV kernel (first, cold
dispatch dropped). Counter passes only, no tracing domains.
"""
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PASSES = [
    "FETCH_SIZE",
    "TCC_HIT_sum TCC_MISS_sum",
    "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum",
    "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY "
    "SQ_INSTS_VMEM_RD SQ_INSTS_LDS",
    "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum",
]
KERNELS = ("k_csr_stream", "k_sell", "k_csr_vec")


def one(d, op, fmt, vw, counters, work):
    os.makedirs(work, exist_ok=True)
    cmd = ["rocprofv3", "--pmc"] + counters.split() + ["--output-format", "csv", "-d", work,
                                                      "-o", "run", "--", sys.executable,
                                                      os.path.join(ROOT, "tools", "level_driver.py"),
                                                      "run", d, op, fmt, str(vw)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        return {"error": (r.stderr or r.stdout)[-800:]}
    files = glob.glob(os.path.join(work, "**", "*counter_collection.csv"), recursive=True)
    vals = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if any(k in row.get("Kernel_Name", "") for k in KERNELS):
                    vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    shutil.rmtree(work, ignore_errors=True)
    out = {}
    for k, v in vals.items():
        v = sorted(v[1:] or v)
        out[k] = v[len(v) // 2]
    out["driver"] = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else ""
    return out


def main():
    d, out_path = sys.argv[1], sys.argv[2]
    res = {}
    for spec in sys.argv[3:]:
        parts = spec.split(":")
        op, fmt = parts[0], parts[1]
        vw = int(parts[2]) if len(parts) > 2 else 0
        row = {}
        for i, counters in enumerate(PASSES):
            row.update({f"pass{i}:{k}" if k == "error" else k: v
                        for k, v in one(d, op, fmt, vw, counters,
                                        os.path.join("/tmp", f"pmc_probe_{os.getpid()}_{i}")).items()})
        res[spec] = row
        print(spec, json.dumps(row), flush=True)
    with open(out_path, "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
