"""Where the amg_2_v_batch farm spends its time, and which batch strategy is fastest for it.
MLAMG_BATCH_TIMING=1 prints the engine's host / device phases on stderr.

  python tools/farm_breakdown.py [count ...]

For each farm size (default 256 and 48 grids of 32^2/48^2/64^2, tools/amg2v_timing.make_farm)
and each engine variant (env knobs of csrc/batch.hip, set between calls): best of 4 wall times.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ml-amg_amd")]
sys.path.insert(0, os.path.join(ROOT, "tools"))
import numpy as np  # noqa: E402,F401
import torch  # noqa: E402

from amg2v_timing import make_farm  # noqa: E402

VARIANTS = ("", "MLAMG_BATCH_NO_PHASED_BATCH", "MLAMG_BATCH_NO_BATCH_EXT")


def main():
    counts = [int(a) for a in sys.argv[1:]] or [256, 48]
    torch.cuda.set_device(0)
    from mlamg import multigrid
    for count in counts:
        probs = make_farm(count)
        multigrid.amg_2_v_batch(probs[:6], res_tol=1e-10)
        for var in VARIANTS:
            for v in VARIANTS:
                os.environ.pop(v, None) if v else None
            if var:
                os.environ[var] = "1"
            best = 1e9
            for rep in range(4):
                t0 = time.perf_counter()
                out = multigrid.amg_2_v_batch(probs, res_tol=1e-10)
                best = min(best, time.perf_counter() - t0)
            print(f"{count} grids, variant {var or 'default'}: best {best*1e3:.2f} ms, iters "
                  f"{sorted(set(o[3] for o in out))}", flush=True)
        for v in VARIANTS:
            if v:
                os.environ.pop(v, None)


if __name__ == "__main__":
    main()
