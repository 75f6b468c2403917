"""mlamg — MI355X-native AMG V-cycle solve path of nicknytko/ml-amg.

Host side of libmlamg_hip.so (HIP kernels for gfx950 behind the C-ABI in include/mlamg.h).
Mirrors the reference modules on the hot path:

  mlamg.multigrid       <- ns/lib/multigrid.py   (jacobi, smoothed_aggregation_jacobi, amg_2_v)
  mlamg.graph           <- ns/lib/graph.py       (modified_bellman_ford, nearest_center_to_agg,
                                                  lloyd_aggregation)
  mlamg.sparse          <- ns/lib/sparse.py      (scipy <-> torch, device CSR handles)
  mlamg.strength        <- utils/common.py:25-31 (strength_measure_funcs; pyamg's evolution
                                                  strength of connection on the device)
  mlamg.preconditioner  <- ns/preconditioner     (MLAMG PC: initialize/update/apply)
  mlamg.gnn             <- ns/model/agg_interp.py (FullAggNet inference: AggNet, MPNN)
  mlamg.hierarchy       multilevel device hierarchy + V-cycle executor (precondition/solve)
  mlamg.distributed     fine level row-partitioned over GPUs (RCCL halo exchange)

Heavy submodules are imported lazily so `import mlamg` stays cheap.
"""
from __future__ import annotations

import importlib

__version__ = "0.1.0"

_SUBMODULES = ("multigrid", "graph", "sparse", "strength", "gnn", "hierarchy",
               "preconditioner", "problems", "gridio", "distributed", "_lib")


def __getattr__(name):
    if name in _SUBMODULES:
        return importlib.import_module(f"{__name__}.{name}")
    if name in ("solve", "precondition", "amg_2_v"):
        mg = importlib.import_module(f"{__name__}.multigrid")
        if name == "amg_2_v":
            return mg.amg_2_v
        pc = importlib.import_module(f"{__name__}.preconditioner")
        return getattr(pc, name)
    raise AttributeError(name)
