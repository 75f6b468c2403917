"""Per-operator SpMV driver for counter studies of the C4 hierarchy (run on the GPU box).

  python tools/level_driver.py dump DIR            build the 216^3 hierarchy, save its operators
  python tools/level_driver.py run DIR OP FMT [VW] run OP (A0, P0, R0, A1, ...) REPS times in FMT

`run` is the program profiled by tools/pmc_probe.py under rocprofv3 (it touches no other kernel
between the upload and the timed launches, so per-dispatch counters isolate the operator).
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "ml-amg_amd")):
    sys.path.insert(0, p)


def dump(d):
    import numpy as np
    from mlamg import problems
    from mlamg.hierarchy import Hierarchy
    n1 = int(os.environ.get("MLAMG_N", "216"))
    H = Hierarchy.build(problems.poisson_3d_7pt(n1), alpha=0.1, max_coarse=2000,
                        fine_format="csr_stream")
    os.makedirs(d, exist_ok=True)
    for i, L in enumerate(H.levels):
        for name, M in (("A", L.A), ("P", L.P), ("R", L.R)):
            S = M.to_scipy()
            np.savez(os.path.join(d, f"{name}{i}.npz"), indptr=S.indptr, indices=S.indices,
                     data=S.data, shape=np.array(S.shape))
            base = os.path.join(d, f"{name}{i}")  # raw arrays for tools/spmv_lab.hip
            S.indptr.astype(np.int32).tofile(base + ".indptr.bin")
            S.indices.astype(np.int32).tofile(base + ".indices.bin")
            S.data.astype(np.float64).tofile(base + ".data.bin")
            np.array(S.shape, dtype=np.int64).tofile(base + ".shape.bin")
    print("dumped", [f for f in sorted(os.listdir(d))])


def run(d, op, fmt, vw=0):
    import numpy as np
    import scipy.sparse as sp
    import torch
    from mlamg.sparse import DeviceCSR
    z = np.load(os.path.join(d, f"{op}.npz"))
    S = sp.csr_matrix((z["data"], z["indices"], z["indptr"]), shape=tuple(z["shape"]))
    M = DeviceCSR.from_scipy(S, check=False).set_format(fmt, vw)
    reps = int(os.environ.get("MLAMG_REPS", "20"))
    x = torch.randn(M.shape[1], dtype=torch.float64, device="cuda")
    y = torch.empty(M.shape[0], dtype=torch.float64, device="cuda")
    M.matvec(x, out=y)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        M.matvec(x, out=y)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    B = 12.0 * M.nnz + 4.0 * (M.shape[0] + 1) + 8.0 * M.shape[1] + 8.0 * M.shape[0]
    print(f"{op} {fmt}/{vw}: n={M.shape[0]} m={M.shape[1]} nnz={M.nnz} {dt * 1e6:.1f} us "
          f"{B / dt / 1e9:.0f} GB/s (algorithmic {B / 1e6:.1f} MB)")


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        run(sys.argv[2], sys.argv[3], sys.argv[4], int(sys.argv[5]) if len(sys.argv) > 5 else 0)
