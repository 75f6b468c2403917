"""Wall time of FullAggNet.forward (ns/model/agg_interp.py:432-486) on the device at the
reference's default sizes (dim 64, AggNet 4 x 2 TAGConv layers, CNet 5 / PNet 4 internal NNConv
layers), per stage, on 2D Poisson grids. GPU box: python tools/gnn_timing.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ml-amg_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mlamg import gnn, problems  # noqa: E402


def main():
    torch.manual_seed(0)
    net = gnn.FullAggNet(dim=64, num_conv=2, iterations=4).cuda()
    out = []
    for m in (32, 64, 128):
        A = problems.poisson_2d_5pt(m)
        net.forward(A, 0.1)  # warm
        torch.cuda.synchronize()
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            net.forward(A, 0.1)
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / reps
        g = gnn.Graph(A)
        st = {}
        for name, fn in (("aggnet", lambda: net.AggNet.run(g, int(np.ceil(0.1 * A.shape[0])))),
                         ("cnet", lambda: net.CNet.run(g))):
            fn()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            st[name + "_ms"] = round((time.perf_counter() - t1) * 1e3, 3)
        row = {"grid": f"{m}^2", "n": A.shape[0], "edges": int(A.nnz),
               "forward_ms": round(t * 1e3, 3), **st}
        print(json.dumps(row), flush=True)
        out.append(row)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "gnn_timing.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
