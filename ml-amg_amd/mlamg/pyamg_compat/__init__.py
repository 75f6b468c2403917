"""The slice of pyamg (4.x; absent here, version unpinned by the reference's Dockerfile:5) that
the reference's hot-path callers import, backed by the MI355X kernels. Aliased as `pyamg` by
mlamg.compat.install() when the real package is missing (or on request):

  pyamg.aggregation.lloyd_aggregation   utils/common.py:91, utils/evaluate_dataset.py:77
  pyamg.graph.lloyd_cluster             ns/lib/graph.py:232
  pyamg.graph.bellman_ford              ns/model/agg_interp.py:475
  pyamg.strength.evolution_strength_of_connection   utils/common.py:27,30
  pyamg.relaxation.relaxation.gauss_seidel          ns/lib/multigrid.py:175,184
  pyamg.aggregation.smoothed_aggregation_solver     ns/preconditioner/PyAMG.py:94 (its default
      recipe: symmetric_strength_of_connection, standard_aggregation, fit_candidates,
      block_gauss_seidel, and the MultilevelSolver's solve / aspreconditioner / repr, :119,129)

Everything else of pyamg (gallery, krylov, other solvers) is not provided: the gallery is the
reference's input generator, which mlamg.mesh covers under its own names.
"""
from . import aggregation, graph, multilevel, relaxation, strength  # noqa: F401

__version__ = "4.2.3+mlamg"
