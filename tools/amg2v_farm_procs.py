"""The unchanged callers' real shape (VERDICT r04 Weak #6 / Next #6): P worker processes, each
making the reference's single calls amg_2_v(A, P, b, x, res_tol=1e-10) (utils/evaluate_dataset.py:96;
the pool of ns/parallel/pool.py:139-186 splits the grids cyclically over its workers), all
sharing ONE GPU — against the same P-process pool running the CPU restatement of the reference
(oracle.amg_2_v: scipy factorized + the Gauss-Seidel sweep).

  python tools/amg2v_farm_procs.py [--procs 1,4,8,16] [--grids 80] [--out ...json]

The parent never touches the GPU: it starts each worker (python this_file --worker), waits for
every worker's READY (problems built, device warmed by one call), releases them together and
takes the wall time until the last one reports. Grids: 2D 5-point m^2, m cycling over
32, 48, 64, 96, 128; SA prolongator of 3x3 box aggregates (omega 2/3); x0 RandomState(i).
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ml-amg_amd")]

SIZES = (32, 48, 64, 96, 128)
BROKER_DIR = os.path.join(ROOT, "gpurun_out", "broker")


def make_problem(i):
    import numpy as np
    from mlamg import problems
    from oracle import restated as orc
    m = SIZES[i % len(SIZES)]
    A = problems.poisson_2d_5pt(m)
    P, _ = orc.smoothed_aggregation_jacobi(A, problems.box_aggregates_2d(m, m, 3),
                                           omega=2.0 / 3.0)
    return A, P, np.zeros(A.shape[0]), np.random.RandomState(i).randn(A.shape[0])


def worker(rank, nprocs, ngrids, device, kw):
    """One pool worker: its cyclic share of the grids, one amg_2_v call per grid."""
    mine = [make_problem(i) for i in range(rank, ngrids, nprocs)]
    if device == "broker":  # unchanged single calls, MLAMG_BROKER=1: this process never
        from mlamg import multigrid  # touches the GPU, the shared broker runs the solves
        solve = multigrid.amg_2_v
        solve(*make_problem(rank), **kw)  # connects (the first worker starts it)
    elif device == "gpu":
        import torch
        torch.cuda.set_device(0)
        from mlamg import multigrid
        solve = multigrid.amg_2_v
        solve(*make_problem(rank), **kw)  # context, library, caches
    else:
        from threadpoolctl import threadpool_limits
        threadpool_limits(1)
        from oracle import restated as orc
        solve = orc.amg_2_v
        solve(*make_problem(rank), **kw)
    print("READY", flush=True)
    sys.stdin.readline()
    t0 = time.perf_counter()
    its = [int(solve(*p, **kw)[3]) for p in mine]
    dt = time.perf_counter() - t0
    print(json.dumps({"rank": rank, "s": dt, "iters": its}), flush=True)


def stop_broker():
    """Shut the farm's broker down (a socket message: this parent never touches the GPU) and
    wait until it has exited."""
    os.environ["MLAMG_BROKER_DIR"] = BROKER_DIR
    from mlamg import broker
    broker.shutdown()
    for _ in range(600):
        if not os.path.exists(broker.socket_path()):
            break
        time.sleep(0.05)
    time.sleep(0.5)  # the process releases the GPU after it removed its socket


def run_farm(nprocs, ngrids, device, mode):
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    if device == "broker":
        env["MLAMG_BROKER"] = "1"
        env["MLAMG_BROKER_DIR"] = BROKER_DIR
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--worker", str(r),
                               "--procs", str(nprocs), "--grids", str(ngrids), "--device", device,
                              "--mode", mode],
                              stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, env=env)
             for r in range(nprocs)]
    try:
        for p in procs:
            line = p.stdout.readline()
            if line.strip() != "READY":
                raise RuntimeError(f"worker failed to start: {line!r}")
        t0 = time.perf_counter()
        for p in procs:
            p.stdin.write("GO\n")
            p.stdin.flush()
        outs = [json.loads(p.stdout.readline()) for p in procs]
        wall = time.perf_counter() - t0
        for p in procs:
            p.wait(timeout=60)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return wall, outs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", default="1,4,8,16")
    ap.add_argument("--grids", type=int, default=80)
    ap.add_argument("--device", default="both")
    ap.add_argument("--mode", default="res", choices=("res", "err"),
                    help="res: res_tol=1e-10 (utils/evaluate_dataset.py:96); err: error_tol=1e-6 "
                         "(utils/train_dataset.py:114)")
    ap.add_argument("--worker", type=int, default=-1)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "amg2v_farm_procs.json"))
    args = ap.parse_args()
    if args.worker >= 0:
        kw = {"res_tol": 1e-10} if args.mode == "res" else {"error_tol": 1e-6}
        return worker(args.worker, int(args.procs), args.grids, args.device, kw)
    rows = []
    devices = {"both": ("cpu", "gpu"), "all": ("cpu", "gpu", "broker")}.get(args.device,
                                                                            (args.device,))
    os.makedirs(BROKER_DIR, exist_ok=True)
    for pn in [int(p) for p in args.procs.split(",")]:
        row = {"procs": pn, "grids": args.grids, "sizes": [f"{m}^2" for m in SIZES],
               "call": "amg_2_v(..., res_tol=1e-10)" if args.mode == "res"
               else "amg_2_v(..., error_tol=1e-6)"}
        for device in devices:
            wall, outs = run_farm(pn, args.grids, device, args.mode)
            if device == "broker":  # stop it now: the next GPU farm's P processes plus a live
                stop_broker()       # broker would exceed the box's 16 GPU processes
            row[f"{device}_wall_s"] = round(wall, 3)
            row[f"{device}_grids_per_s"] = round(args.grids / wall, 2)
            row[f"{device}_iters"] = [it for o in sorted(outs, key=lambda o: o["rank"])
                                      for it in o["iters"]]
        if "gpu_wall_s" in row and "cpu_wall_s" in row:
            row["gpu_over_cpu"] = round(row["cpu_wall_s"] / row["gpu_wall_s"], 2)
            row["iters_match"] = row["cpu_iters"] == row["gpu_iters"]
        if "broker_wall_s" in row and "cpu_wall_s" in row:
            row["broker_over_cpu"] = round(row["cpu_wall_s"] / row["broker_wall_s"], 2)
            row["broker_iters_match"] = row["cpu_iters"] == row["broker_iters"]
        for d in ("cpu", "gpu", "broker"):
            row.pop(f"{d}_iters", None)
        print(json.dumps(row), flush=True)
        rows.append(row)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump({"note": "P processes, each single amg_2_v(res_tol=1e-10) calls on its cyclic "
                           "share of the grids; GPU: all P on one MI355X; CPU: the oracle's "
                           "restatement, 1 thread per process", "rows": rows}, fh, indent=1)


if __name__ == "__main__":
    main()
