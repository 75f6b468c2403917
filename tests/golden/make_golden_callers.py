"""Golden vectors for the reference's CALLERS of the hot path and for tie-rich aggregation, made
by running the REFERENCE code (container-only: needs /root/reference).

* Tie-rich Lloyd: ns.lib.graph.lloyd_aggregation on constant-coefficient grids with 'unit'
  distances and on the default evaluation path (np.random.seed(0), olson measure, 'same',
  rand=0; utils/common.py:51-58) — the reference driver around the oracle's pyamg-order
  lloyd_cluster (oracle/oracle.c, canon=0).
* Callers: utils/common.py is exec'd from the reference file (its out-of-scope imports —
  ns.model.*, ns.ga.* — are empty stubs), and its evaluate_ref_conv (pyamg's own
  lloyd_aggregation, :84-111) and evaluate_dataset (model=None: ns.lib.graph.lloyd_aggregation,
  :40-82) are run on a small dataset; utils/evaluate_dataset.py's evaluate_dataset(ds, method)
  (:59-101, methods 'lloyd' and 'dumb') is taken out of that file with ast (its module level
  parses argv and loads a dataset) and run the same way. pyamg (absent) is the oracle's
  restatement: lloyd_cluster, gauss_seidel, evolution_strength_of_connection (seeded Arnoldi rho
  on the global generator) and pyamg 4.x aggregation.lloyd_aggregation. Every aggregate map the
  callers build (the Agg handed to smoothed_aggregation_jacobi) and every conv factor is stored.

Only inputs and outputs are stored (tests/golden/reference_callers.npz); no reference source.

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_callers.py
"""
import ast
import os
import sys
import types

import numpy as np
import scipy.sparse as sp

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(ROOT, "ml-amg_amd"))
from make_golden import REF, _stub, load_reference, orc  # noqa: E402


class Grid:
    def __init__(self, A):
        self.A = A


def dataset():
    """Small grids of the reference's families: constant-coefficient 2D (tie-rich), the
    reference's own demos/laplace_3d.grid, a 2D Voronoi jump-coefficient problem."""
    from mlamg import problems
    g = np.load(os.path.join(HERE, "laplace_3d_grid.npz"))
    A3 = sp.csr_matrix((g["data"], g["indices"], g["indptr"]))
    A3.sort_indices()
    mats = [problems.poisson_2d_5pt(20), problems.poisson_2d_5pt(28), A3,
            problems.jump_2d(24, problems.voronoi_jumps(np.random.RandomState(0)))]
    return [Grid(sp.csr_matrix(A)) for A in mats]


def install_caller_stubs():
    def esoc(A, *a, **kw):
        assert not a and not kw
        return orc.evolution_strength(A)

    sys.modules["pyamg"].strength = _stub("pyamg.strength", evolution_strength_of_connection=esoc)
    sys.modules["pyamg"].aggregation = _stub("pyamg.aggregation",
                                             lloyd_aggregation=orc.pyamg_lloyd_aggregation)
    for name in ("ns.model", "ns.ga"):
        sys.modules.setdefault(name, types.ModuleType(name))
    for name in ("ns.model.agg_interp", "ns.model.data", "ns.ga.parga", "ns.ga.torch"):
        _stub(name)


def load_common():
    path = os.path.join(REF, "utils", "common.py")
    mod = types.ModuleType("common")
    mod.__file__ = path
    with open(path) as fh:
        code = compile(fh.read(), path, "exec")
    exec(code, mod.__dict__)
    sys.modules["common"] = mod
    return mod


def load_evaluate_dataset(common):
    """evaluate_dataset() of utils/evaluate_dataset.py, compiled from its own def statement."""
    import numpy.linalg as la
    import torch
    path = os.path.join(REF, "utils", "evaluate_dataset.py")
    with open(path) as fh:
        tree = ast.parse(fh.read(), path)
    fn = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "evaluate_dataset"]
    code = compile(ast.Module(body=fn, type_ignores=[]), path, "exec")
    import ns.lib.graph  # noqa: F401
    import ns.lib.multigrid  # noqa: F401
    import ns.lib.sparse  # noqa: F401
    g = {"np": np, "la": la, "torch": torch, "pyamg": sys.modules["pyamg"], "common": common,
         "ns": sys.modules["ns"], "neumann_solve": False, "omega": 2. / 3., "alpha": 0.1,
         "model": None}
    exec(code, g)
    return g


def main():
    mg, gr, spm = load_reference()
    install_caller_stubs()
    out = {}
    g = dict(np.load(os.path.join(HERE, "reference_vectors.npz")))
    # ---------------------------------------------------------------- tie-rich Lloyd (driver)
    for k in ("p2d", "lap3d"):
        A = sp.csr_matrix((g[f"{k}_data"], g[f"{k}_indices"], g[f"{k}_indptr"]))
        C = sp.csr_matrix((np.ones_like(A.data), A.indices, A.indptr), A.shape)
        for rand in (0, 3):
            AggOp, roots, seeds = gr.lloyd_aggregation(C, ratio=0.1, distance='unit', rand=rand)
            out[f"{k}_unit{rand}_roots"], out[f"{k}_unit{rand}_seeds"] = roots, seeds
            out[f"{k}_unit{rand}_agg_indices"] = AggOp.indices
            out[f"{k}_unit{rand}_agg_indptr"] = AggOp.indptr
        np.random.seed(0)
        Cs = orc.strength_measure(A, "olson")
        AggOp, roots, seeds = gr.lloyd_aggregation(Cs, ratio=0.1, distance='same', rand=0)
        out[f"{k}_olson_roots"], out[f"{k}_olson_seeds"] = roots, seeds
        out[f"{k}_olson_agg_indices"] = AggOp.indices
        out[f"{k}_olson_agg_indptr"] = AggOp.indptr
    # ---------------------------------------------------------------- callers
    common = load_common()
    ed = load_evaluate_dataset(common)
    ds = dataset()
    for i, grid in enumerate(ds):
        A = grid.A
        out[f"ds{i}_indptr"], out[f"ds{i}_indices"], out[f"ds{i}_data"] = A.indptr, A.indices, A.data
    seen = []
    real_sa = mg.smoothed_aggregation_jacobi

    def spy_sa(A, Agg):
        Agg = sp.csr_matrix(Agg)
        seen.append(Agg)
        return real_sa(A, Agg)

    mg.smoothed_aggregation_jacobi = spy_sa
    runs = {
        "ref_conv": lambda: common.evaluate_ref_conv(ds, common.strength_measure_funcs['olson'],
                                                     alpha=0.1),
        "common_ed": lambda: common.evaluate_dataset(None, ds, alpha=0.1),
        "ed_lloyd": lambda: ed["evaluate_dataset"](ds, method='lloyd'),
        "ed_dumb": lambda: ed["evaluate_dataset"](ds, method='dumb'),
    }
    try:
        for name, run in runs.items():
            seen.clear()
            conv = run()
            out[f"{name}_conv"] = np.asarray(conv, dtype=np.float64)
            assert len(seen) == len(ds)
            for i, Agg in enumerate(seen):
                Agg = sp.csr_matrix(Agg)
                Agg.sort_indices()
                out[f"{name}{i}_agg_indptr"], out[f"{name}{i}_agg_indices"] = Agg.indptr, Agg.indices
            print(name, out[f"{name}_conv"])
    finally:
        mg.smoothed_aggregation_jacobi = real_sa
    path = os.path.join(HERE, "reference_callers.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}: {len(out)} arrays, {os.path.getsize(path)} bytes")


if __name__ == "__main__":
    main()
