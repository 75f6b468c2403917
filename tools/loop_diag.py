"""Diagnostics for the loopback distributed executor: per (world, K) bitwise check + partition
sizes per level (run on the GPU box)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ml-amg_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mlamg import problems, partition  # noqa: E402
from mlamg.hierarchy import Hierarchy  # noqa: E402
import test_gpu_distributed_loopback as T  # noqa: E402

A = problems.poisson_3d_7pt(int(sys.argv[1]) if len(sys.argv) > 1 else 36)
H = Hierarchy.build(A, alpha=0.1, max_coarse=200)
n = A.shape[0]
print("levels", [L.A.shape[0] for L in H.levels], "coarse", H.Ac.shape[0])
x0 = np.random.RandomState(0).randn(n)
b = np.random.RandomState(1).randn(n)
xd = torch.as_tensor(x0).cuda()
h_ref = H.cycle(torch.as_tensor(b).cuda(), xd, 6, use_graph=False)
x_ref = xd.cpu().numpy()
for world in (2, 4, 5, 8):
    for K in (1, 2, 3):
        if K > len(H.levels):
            continue
        Ds, out = T._run(A, H, world, 0, b=b, x0=x0, K=K)
        ok = [np.array_equal(xo, x_ref[D.lo:D.hi]) for D, (xo, h) in zip(Ds, out)]
        own = [[p["hi"] - p["lo"] for p in D.parts] for D in Ds]
        cown = [int(D.c_hi[D.comm.rank] - D.c_lo[D.comm.rank]) for D in Ds]
        err = max(float(np.abs(xo - x_ref[D.lo:D.hi]).max()) for D, (xo, h) in zip(Ds, out))
        print(f"world {world} K {K}: bitwise per rank {ok} max|dx| {err:.2e}; rows per level {own}; owned coarse segment {cown}", flush=True)
