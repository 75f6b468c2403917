"""Device-wide inverse Cholesky factor of an SPD coarse-sized operator (2D Poisson, n = m^2):
mlamg_dense_create three times, for per-kernel timing under rocprofv3 --kernel-trace (A/B of lab
builds via MLAMG_LIB). GPU box only."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ml-amg_amd")]
import torch  # noqa: E402

from mlamg import problems, sparse  # noqa: E402
from mlamg._lib import call, stream_ptr  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 64
A = sparse.as_device(problems.poisson_2d_5pt(m))
tag = os.path.basename(os.environ.get("MLAMG_LIB", "default"))
for rep in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    h = ctypes.c_void_p()
    call("mlamg_dense_create", A.handle, ctypes.byref(h), stream_ptr())
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    call("mlamg_dense_destroy", h)
    print(f"{tag} n={m * m}: dense_create {t * 1e3:.1f} ms", flush=True)
