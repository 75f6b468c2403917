"""Per-launch roofline of the bench's C4 V-cycle (VERDICT r05 Next #3).

  run:   python tools/cycle_roofline.py run OUTDIR [--cycles K] [--eager] [--n 216]
         (on the GPU box, under `rocprofv3 --kernel-trace` or `--pmc ...`): builds the bench's
         hierarchy (bench.py defaults: C4, reference aggregation, sorted coarse order), writes
         OUTDIR/launch_bytes.json — one entry per launch of a fused V(1,1) cycle in launch order,
         with the bytes that launch must move as its operands are stored (the model of
         csrc/hier.hip cycle_bytes, launch by launch) — then runs K cycles with b = 0 (NULL).
  table: python tools/cycle_roofline.py table OUTDIR TRACE_CSV [--fetch CSV] [--write CSV]
         (host side): aligns the rocprof kernel trace with launch_bytes.json (cycles end at
         k_finalize_norm; per position the median duration over the last 15 cycles) and prints
         the table — format bytes, µs, fraction of the 8 TB/s peak and of the measured
         elementwise ceiling — plus, from PMC counter CSVs of separate FETCH_SIZE / WRITE_SIZE
         passes, the HBM bytes per launch (gfx950 correction: FETCH_SIZE counts half of a
         wide streaming read, so it is doubled; /opt/skills/guides/MI355X_MICROARCH.md).
"""
import argparse
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "ml-amg_amd")):
    sys.path.insert(0, p)

PEAK = 8000.0      # GB/s, HBM3E peak (MI355X_MICROARCH.md)
CEILING = 5310.0   # GB/s, measured elementwise ceiling (profiles/r05/final/copy_ceiling.json)


def launch_list(H, zero_rhs=True):
    """The fused V(1,1) cycle's launches (csrc/hier.hip cycle_top / cycle_coarse) with the bytes
    each must move as stored: operator format bytes (matrix + x once + y once) + epilogue
    vectors."""
    out = []
    L = H.levels
    nl = len(L)

    def fb(M):
        return float(M.format_bytes())

    def dv(l):
        return 0.0 if L[l].A.get_format()[0] == "rowpat" else 8.0 * L[l].A.shape[0]

    def bb(l):
        return 0.0 if (l == 0 and zero_rhs) else 8.0 * L[l].A.shape[0]

    for l in range(nl):
        n = L[l].A.shape[0]
        out.append({"op": f"A{l} residual r = b - A x", "level": l, "bytes": fb(L[l].A) + bb(l)})
        if l + 1 < nl:
            n1 = L[l + 1].A.shape[0]
            out.append({"op": f"R{l} restriction (+ x{l + 1} = D b{l + 1})", "level": l,
                        "bytes": fb(L[l].R) + 16.0 * n1})
        else:
            out.append({"op": f"R{l} restriction", "level": l, "bytes": fb(L[l].R)})
    nc = H.Ac.shape[0]
    out.append({"op": f"coarse dense GEMV (n={nc})", "level": nl,
                "bytes": 8.0 * nc * nc + 16.0 * nc})
    for l in range(nl - 1, -1, -1):
        n = L[l].A.shape[0]
        out.append({"op": f"P{l} prolongation x += P e", "level": l,
                    "bytes": fb(L[l].P) + 8.0 * n})
        out.append({"op": f"A{l} Jacobi post-smoothing", "level": l,
                    "bytes": fb(L[l].A) + bb(l) + dv(l)})
    out.append({"op": "A0 end residual + norm partials + next pre-sweep", "level": 0,
                "bytes": fb(L[0].A) + bb(0) + dv(0)})
    out.append({"op": "norm finalize", "level": 0, "bytes": 0.0})
    return out


def run(args):
    import numpy as np
    import torch
    from mlamg import problems
    from mlamg.hierarchy import Hierarchy
    os.makedirs(args.outdir, exist_ok=True)
    A = problems.poisson_3d_7pt(args.n)
    H = Hierarchy.build(A, alpha=0.1, strength_mode="invabs", max_coarse=2000,
                        aggregation="reference", coarse_order="sorted")
    launches = launch_list(H)
    rows = [{"level": l, "n": L.A.shape[0], "A": L.A.get_format()[:2], "A_nnz": L.A.nnz,
             "P": L.P.get_format()[:2], "P_nnz": L.P.nnz, "R": L.R.get_format()[:2]}
            for l, L in enumerate(H.levels)]
    with open(os.path.join(args.outdir, "launch_bytes.json"), "w") as fh:
        json.dump({"launches": launches, "levels": rows,
                   "cycle_format_bytes": H.cycle_bytes(stored=True)}, fh, indent=1)
    n = A.shape[0]
    x0 = np.random.RandomState(0).randn(n)
    x0 /= np.linalg.norm(x0)
    b = torch.zeros(n, dtype=torch.float64, device="cuda")
    x = torch.as_tensor(x0).cuda()
    H.cycle_async(b, x, 3, use_graph=not args.eager)
    torch.cuda.synchronize()
    H.cycle_async(b, x, args.cycles, use_graph=not args.eager)
    torch.cuda.synchronize()
    print(f"cycle_roofline: {len(launches)} launches per cycle, {args.cycles} cycles run",
          flush=True)


def is_cycle_end(name, fused):
    """The cycle's last launch: k_finalize_norm, or — with the norm finished inside the pass
    (no finalize launch) — the end-of-cycle residual pass, the only RESID launch with NORM."""
    return "k_finalize_norm" in name if not fused else "<1, true" in name


def fused_norm(names):
    return not any("k_finalize_norm" in n for n in names)


def cycles_of(rows, key_start, key_end, key_name):
    rows = sorted(rows, key=lambda r: int(r[key_start]))
    fused = fused_norm(r[key_name] for r in rows)
    idx = [i for i, r in enumerate(rows) if is_cycle_end(r[key_name], fused)]
    return [rows[a + 1:b + 1] for a, b in zip(idx, idx[1:])]


def pmc_per_position(path, names, counter):
    """Median counter value per cycle position from a counter_collection CSV."""
    rows = [r for r in csv.DictReader(open(path)) if r.get("Counter_Name") == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    fused = fused_norm(r["Kernel_Name"] for r in rows)
    idx = [i for i, r in enumerate(rows) if is_cycle_end(r["Kernel_Name"], fused)]
    cyc = [rows[a + 1:b + 1] for a, b in zip(idx, idx[1:])]
    cyc = [c for c in cyc if len(c) == len(names)]
    if not cyc:
        return None
    return [statistics.median(float(c[i]["Counter_Value"]) for c in cyc)
            for i in range(len(names))]


def counters(args):
    """Per-position medians of every counter in the given counter_collection CSVs."""
    meta = json.load(open(os.path.join(args.outdir, "launch_bytes.json")))
    launches = meta["launches"]
    res = {}
    for path in args.csv:
        rows = list(csv.DictReader(open(path)))
        if fused_norm(r["Kernel_Name"] for r in rows):
            launches = [L for L in meta["launches"] if L["op"] != "norm finalize"]
        for name in sorted({r["Counter_Name"] for r in rows}):
            v = pmc_per_position(path, launches, name)
            if v is not None:
                res[name] = v
    names = sorted(res)
    print("| # | launch | " + " | ".join(names) + " |")
    print("|---|---|" + "---|" * len(names))
    for i, L in enumerate(launches):
        print(f"| {i} | {L['op']} | " + " | ".join(f"{res[k][i]:.4g}" for k in names) + " |")
    with open(os.path.join(args.outdir, "cycle_counters.json"), "w") as fh:
        json.dump({"positions": [L["op"] for L in launches], "counters": res}, fh, indent=1)


def table(args):
    meta = json.load(open(os.path.join(args.outdir, "launch_bytes.json")))
    launches = meta["launches"]
    rows = list(csv.DictReader(open(args.trace)))
    if fused_norm(r["Kernel_Name"] for r in rows):  # the norm is finished inside its pass
        launches = [L for L in launches if L["op"] != "norm finalize"]
    cyc = cycles_of(rows, "Start_Timestamp", "End_Timestamp", "Kernel_Name")
    cyc = [c for c in cyc if len(c) == len(launches)][-15:]
    if not cyc:
        raise SystemExit("no traced cycle has the expected number of launches")
    names = [r["Kernel_Name"] for r in cyc[-1]]
    us = [statistics.median((int(c[i]["End_Timestamp"]) - int(c[i]["Start_Timestamp"])) / 1e3
                            for c in cyc) for i in range(len(names))]
    span = statistics.median((int(c[-1]["End_Timestamp"]) - int(c[0]["Start_Timestamp"])) / 1e3
                             for c in cyc)
    fetch = pmc_per_position(args.fetch, names, "FETCH_SIZE") if args.fetch else None
    write = pmc_per_position(args.write, names, "WRITE_SIZE") if args.write else None
    out = []
    for i, (L, name, t) in enumerate(zip(launches, names, us)):
        gbs = L["bytes"] / t / 1e3 if t > 0 else 0.0
        row = {"pos": i, "op": L["op"], "kernel": name.split("(")[0].replace("void ", ""),
               "bytes": L["bytes"], "us": round(t, 2), "GBps": round(gbs, 1),
               "frac_peak": round(gbs / PEAK, 3), "frac_ceiling": round(gbs / CEILING, 3)}
        if fetch and write:
            hbm = 2.0 * fetch[i] * 1024 + write[i] * 1024  # KiB; reads doubled (gfx950)
            row["pmc_hbm_bytes"] = hbm
            row["pmc_over_format"] = round(hbm / L["bytes"], 3) if L["bytes"] else None
        out.append(row)
    tot_b = sum(L["bytes"] for L in launches)
    busy = sum(us)
    res = {"rows": out, "span_us": round(span, 1), "busy_us": round(busy, 1),
           "cycle_bytes": tot_b, "cycle_GBps": round(tot_b / span / 1e3, 1),
           "levels": meta["levels"], "cycles_used": len(cyc)}
    with open(os.path.join(args.outdir, "cycle_roofline.json"), "w") as fh:
        json.dump(res, fh, indent=1)
    pm = fetch and write
    print("| # | launch | kernel | MB | µs | GB/s | of 8 TB/s | of 5.31 TB/s |"
          + (" PMC MB | PMC / format |" if pm else ""))
    print("|---|---|---|---|---|---|---|---|" + ("---|---|" if pm else ""))
    for r in out:
        line = (f"| {r['pos']} | {r['op']} | `{r['kernel']}` | {r['bytes'] / 1e6:.1f} | "
                f"{r['us']:.1f} | {r['GBps']:.0f} | {r['frac_peak']:.2f} | "
                f"{r['frac_ceiling']:.2f} |")
        if pm:
            line += f" {r['pmc_hbm_bytes'] / 1e6:.1f} | {r['pmc_over_format']} |"
        print(line)
    print(f"\ncycle: {tot_b / 1e6:.1f} MB, span {span:.1f} µs (busy {busy:.1f}), "
          f"{tot_b / span / 1e3:.0f} GB/s = {tot_b / span / 1e3 / PEAK:.3f} of peak; "
          f"{len(cyc)} cycles")


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("outdir")
    r.add_argument("--cycles", type=int, default=30)
    r.add_argument("--eager", action="store_true")
    r.add_argument("--n", type=int, default=216)
    t = sub.add_parser("table")
    t.add_argument("outdir")
    t.add_argument("trace")
    t.add_argument("--fetch")
    t.add_argument("--write")
    c = sub.add_parser("counters")
    c.add_argument("outdir")
    c.add_argument("csv", nargs="+")
    args = ap.parse_args()
    {"run": run, "table": table, "counters": counters}[args.cmd](args)


if __name__ == "__main__":
    main()
