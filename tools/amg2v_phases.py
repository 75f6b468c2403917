import os, sys, time
ROOT = "/root/repo" if os.path.exists("/root/repo/bench.py") else os.getcwd()
sys.path[:0] = [ROOT, os.path.join(ROOT, "ml-amg_amd")]
import numpy as np, torch, ctypes
from mlamg import multigrid, problems, sparse, _lib
from mlamg.hierarchy import Hierarchy, Level
from mlamg.sparse import as_device, galerkin, to_device_vec
from oracle import restated as orc
torch.cuda.set_device(0)
def T(): torch.cuda.synchronize(); return time.perf_counter()
for m in (96, 128):
    A = problems.poisson_2d_5pt(m); Agg = problems.box_aggregates_2d(m, m, 3)
    P, _ = orc.smoothed_aggregation_jacobi(A, Agg, omega=2.0/3.0)
    n = A.shape[0]; x0 = np.random.RandomState(0).randn(n); b = np.zeros(n)
    multigrid.amg_2_v(A, P, b, x0, res_tol=1e-10)
    for rep in range(2):
        t = [T()]
        Ad = as_device(A); t.append(T())
        Pd = as_device(P); t.append(T())
        Rd = Pd.transpose(); t.append(T())
        Ac = galerkin(Rd, Ad, Pd); t.append(T())
        dinv = Ad.diag_inv(0.666); t.append(T())
        h = ctypes.c_void_p(); _lib.call("mlamg_dense_create", Ac.handle, ctypes.byref(h), _lib.stream_ptr()); t.append(T())
        gs = multigrid.GaussSeidel(Ad); t.append(T())
        H = Hierarchy.two_level(A, P, omega=0.666, smoother="gauss_seidel"); t.append(T())
        xd = to_device_vec(x0).clone(); bd = to_device_vec(b); t.append(T())
        err = H.cycle(bd, xd, 500, tol=1e-10); t.append(T())
        err = H.cycle(bd, to_device_vec(x0).clone(), 500, tol=1e-10); t.append(T())
        out = xd.cpu().numpy(); t.append(T())
        names = ["upA", "upP", "transpose", "galerkin", "diag_inv", "dense", "gs_create", "two_level(all)", "vecs", "cycle(first)", "cycle(2nd)", "download"]
        print(m, " ".join(f"{k}={1e3*(t[i+1]-t[i]):.2f}" for i, k in enumerate(names)), flush=True)
