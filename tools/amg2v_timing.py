"""End-to-end time of the reference's own call pattern — two-level amg_2_v (GS smoother, res_tol)
on small grids, the per-problem unit of the training/evaluation loops (utils/common.py:77,106,
utils/evaluate_dataset.py:96) — device vs the oracle's CPU restatement (scipy factorized + the
C Gauss-Seidel sweep). Run on the GPU box:

  python tools/amg2v_timing.py [--out gpurun_out/amg2v_timing.json]

1. single calls at 32^2 .. 128^2: fused one-launch solver (engine='auto'), per-operation
   hierarchy engine, CPU restatement (1 core);
2. the task farm: 48 grids 32^2..64^2 — CPU restatement sequential (1 core) and over a process
   pool on every CPU this process may use (bench.host_cores), device amg_2_v_batch (one launch)
   and its threaded hierarchy engine.
The CPU pool runs before anything touches the GPU (fork).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ml-amg_amd")]
import numpy as np  # noqa: E402

from mlamg import problems  # noqa: E402
from oracle import restated as orc  # noqa: E402

_PROBS = None


def _cpu_solve(i):
    A, P, b, x0 = _PROBS[i]
    return orc.amg_2_v(A, P, b, x0, res_tol=1e-10)[3]


def make_farm(count=48):
    out = []
    for i in range(count):
        m = 32 + 16 * (i % 3)
        A = problems.poisson_2d_5pt(m)
        P, _ = orc.smoothed_aggregation_jacobi(A, problems.box_aggregates_2d(m, m, 3),
                                               omega=2.0 / 3.0)
        out.append((A, P, np.zeros(A.shape[0]), np.random.RandomState(i).randn(A.shape[0])))
    return out


def main():
    global _PROBS
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "amg2v_timing.json"))
    args = ap.parse_args()
    from bench import host_cores
    threads, cores_desc = host_cores()
    rec = {"host": cores_desc, "pool_processes": threads, "single": [], "farm": {}}
    _PROBS = make_farm()
    # ---- CPU: sequential and process pool (before any GPU call)
    for A, P, b, x0 in _PROBS[:3]:
        orc.amg_2_v(A, P, b, x0, res_tol=1e-10)
    t0 = time.perf_counter()
    for i in range(len(_PROBS)):
        _cpu_solve(i)
    t_seq = time.perf_counter() - t0
    import multiprocessing as mp
    with mp.get_context("fork").Pool(threads) as pool:
        pool.map(_cpu_solve, range(threads))  # warm the workers
        t0 = time.perf_counter()
        pool.map(_cpu_solve, range(len(_PROBS)), chunksize=1)
        t_pool = time.perf_counter() - t0
    rec["farm"]["cpu_sequential_ms"] = round(t_seq * 1e3, 2)
    rec["farm"]["cpu_pool_ms"] = round(t_pool * 1e3, 2)
    # the same pool over a 256-grid farm
    _PROBS = make_farm(256)
    with mp.get_context("fork").Pool(threads) as pool:
        pool.map(_cpu_solve, range(threads))
        t0 = time.perf_counter()
        pool.map(_cpu_solve, range(len(_PROBS)), chunksize=1)
        rec["farm"]["cpu_pool256_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
    _PROBS = make_farm()
    print(f"48 grids: CPU restatement sequential {t_seq*1e3:.1f} ms ({t_seq/48*1e3:.2f} ms/grid); "
          f"pool of {threads} processes {t_pool*1e3:.1f} ms", flush=True)
    # ---- GPU
    import torch
    torch.cuda.set_device(0)
    from mlamg import multigrid
    for m in (32, 48, 64, 96, 128):
        A = problems.poisson_2d_5pt(m)
        P, _ = orc.smoothed_aggregation_jacobi(A, problems.box_aggregates_2d(m, m, 3),
                                               omega=2.0 / 3.0)
        n = A.shape[0]
        x0 = np.random.RandomState(0).randn(n)
        b = np.zeros(n)
        row = {"grid": f"{m}^2", "n": n, "n_c": P.shape[1]}
        for eng in ("auto", "fused", "hierarchy"):
            multigrid.amg_2_v(A, P, b, x0, res_tol=1e-10, engine=eng)  # warm
            reps = 5
            t0 = time.perf_counter()
            for _ in range(reps):
                x, conv, err, it = multigrid.amg_2_v(A, P, b, x0, res_tol=1e-10, engine=eng)
            row[f"device_{eng}_ms"] = round((time.perf_counter() - t0) / reps * 1e3, 3)
            row[f"iters_{eng}"] = it
        t0 = time.perf_counter()
        for _ in range(3):
            xr, convr, errr, itr = orc.amg_2_v(A, P, b, x0, res_tol=1e-10)
        row["cpu_1core_ms"] = round((time.perf_counter() - t0) / 3 * 1e3, 3)
        row["iters_cpu"] = itr
        row["conv"] = [float(conv), float(convr)]
        print(json.dumps(row), flush=True)
        rec["single"].append(row)
    probs = _PROBS
    multigrid.amg_2_v_batch(probs[:6], res_tol=1e-10)
    torch.cuda.synchronize()
    # first call at this batch size (host and device buffers grow inside it), then the steady
    # state of a loop over a dataset (buffers reused): best of 5
    t0 = time.perf_counter()
    out = multigrid.amg_2_v_batch(probs, res_tol=1e-10)
    rec["farm"]["device_fused_batch_first_call_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
    t_f = 1e9
    for _ in range(5):
        t0 = time.perf_counter()
        out = multigrid.amg_2_v_batch(probs, res_tol=1e-10)
        t_f = min(t_f, time.perf_counter() - t0)
    its = [o[3] for o in out]
    ref_its = [orc.amg_2_v(*p, res_tol=1e-10)[3] for p in probs]
    rec["farm"]["device_fused_batch_ms"] = round(t_f * 1e3, 2)
    rec["farm"]["iterations_match_cpu"] = its == ref_its
    t0 = time.perf_counter()
    multigrid.amg_2_v_batch(probs, workers=16, res_tol=1e-10, engine="hierarchy")
    t_h = time.perf_counter() - t0
    rec["farm"]["device_threaded_hierarchy_ms"] = round(t_h * 1e3, 2)
    rec["farm"]["speedup_vs_cpu_pool"] = round(t_pool / t_f, 2)
    print(json.dumps(rec["farm"]), flush=True)
    # a dataset-sized farm: 256 grids (one launch fills more of the 256 CUs)
    big = make_farm(256)
    t0 = time.perf_counter()
    out = multigrid.amg_2_v_batch(big, res_tol=1e-10)
    t_first = time.perf_counter() - t0
    t_b = 1e9
    for _ in range(3):
        t0 = time.perf_counter()
        out = multigrid.amg_2_v_batch(big, res_tol=1e-10)
        t_b = min(t_b, time.perf_counter() - t0)
    rec["farm256"] = {"device_fused_batch_first_call_ms": round(t_first * 1e3, 2),
                      "device_fused_batch_ms": round(t_b * 1e3, 2),
                      "cpu_pool_ms": rec["farm"].get("cpu_pool256_ms")}
    if rec["farm256"]["cpu_pool_ms"]:
        rec["farm256"]["speedup_vs_cpu_pool"] = round(rec["farm256"]["cpu_pool_ms"] / (t_b * 1e3), 2)
    print(json.dumps(rec["farm256"]), flush=True)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(rec, fh, indent=1)


if __name__ == "__main__":
    main()
