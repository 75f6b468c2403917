import os, sys, time
os.environ["MLAMG_BATCH_TIMING"] = "1"
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path[:0] = [os.path.join(ROOT, "ml-amg_amd"), ROOT]
import torch
from mlamg import multigrid
from tools.amg2v_timing import make_farm
torch.cuda.set_device(0)
probs = make_farm()
for rep in range(3):
    t0 = time.perf_counter()
    multigrid.amg_2_v_batch(probs, res_tol=1e-10)
    print(f"rep {rep}: {1e3*(time.perf_counter()-t0):.2f} ms", flush=True)
