"""V-cycles of the pyamg-recipe hierarchy for a kernel trace (run under rocprofv3 --kernel-trace
--stats): python tools/pyamg_sa_trace.py poisson3d:64 [cycles]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ml-amg_amd"), os.path.join(ROOT, "tools")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mlamg.hierarchy import Hierarchy  # noqa: E402
from pyamg_sa_bench import problem  # noqa: E402

spec = sys.argv[1] if len(sys.argv) > 1 else "poisson3d:64"
cycles = int(sys.argv[2]) if len(sys.argv) > 2 else 5
A = problem(spec)
H = Hierarchy.pyamg_sa(A)
for i, L in enumerate(H.levels):
    print(f"level {i}: n={L.A.shape[0]} nnz={L.A.nnz} gs_levels={L.gs.n_levels}", flush=True)
b = torch.as_tensor(np.random.default_rng(0).standard_normal(A.shape[0])).to("cuda")
x = torch.zeros_like(b)
H.cycle_async(b, x, cycles, use_graph=False)
torch.cuda.synchronize()
print("done", flush=True)
