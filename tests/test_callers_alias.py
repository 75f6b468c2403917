"""CPU: the reference's callers resolve every hot-path name through mlamg.compat.install()
alone — with pyamg and torch_sparse absent. No GPU calls.

* The alias table: ns.lib.{multigrid, graph, sparse, sparse_tensor} and pyamg.{aggregation,
  graph, strength, relaxation.relaxation} resolve to this package, parents bound as attributes.
* ns.lib.sparse_tensor mirror (ns/lib/sparse_tensor.py:9-59) on CPU tensors against dense math.
* When the reference tree is present (this container, not the GPU box): utils/common.py is
  exec'd from the reference file, its out-of-scope imports (ns.model.agg_interp,
  ns.model.data, ns.ga.*: the GNN and the genetic algorithm) as empty stubs; every name its
  evaluate_dataset / evaluate_ref_conv bodies and utils/evaluate_dataset.py's evaluate_dataset
  load resolves, and the hot-path ones to this package's functions.
  tests/test_gpu_callers.py runs those call sequences on the device."""
import ast
import os
import sys
import types

import numpy as np
import pytest
import scipy.sparse as sp

REF = "/root/reference"


@pytest.fixture
def compat(monkeypatch):
    import mlamg.compat
    for name in list(sys.modules):
        if name == "ns" or name.startswith("ns.") or name == "pyamg" or name.startswith("pyamg."):
            monkeypatch.delitem(sys.modules, name)
    installed = mlamg.compat.install(pyamg=True)
    yield installed
    mlamg.compat.uninstall(installed)


def test_alias_table(compat):
    import mlamg.graph
    import mlamg.multigrid
    import mlamg.sparse
    import mlamg.sparse_tensor
    import mlamg.strength
    import ns.lib.graph
    import ns.lib.multigrid
    import ns.lib.sparse
    import ns.lib.sparse_tensor
    import pyamg
    import pyamg.aggregation
    import pyamg.graph
    import pyamg.relaxation.relaxation
    import pyamg.strength
    assert ns.lib.multigrid.amg_2_v is mlamg.multigrid.amg_2_v
    assert ns.lib.graph.modified_bellman_ford is mlamg.graph.modified_bellman_ford
    assert ns.lib.graph.lloyd_aggregation is mlamg.graph.lloyd_aggregation
    assert ns.lib.sparse.scipy_to_torch is mlamg.sparse.to_torch_sparse
    assert ns.lib.sparse_tensor.to_scipy is mlamg.sparse.to_scipy
    assert pyamg.aggregation.lloyd_aggregation is mlamg.graph.pyamg_lloyd_aggregation
    assert pyamg.graph.lloyd_cluster is mlamg.graph.lloyd_cluster
    assert pyamg.graph.bellman_ford is mlamg.graph.bellman_ford
    assert (pyamg.strength.evolution_strength_of_connection
            is mlamg.strength.evolution_strength_of_connection)
    assert callable(pyamg.relaxation.relaxation.gauss_seidel)
    # the PyAMG PC's solver (ns/preconditioner/PyAMG.py:94) and its pieces
    import mlamg.pyamg_compat.aggregation as agg
    assert pyamg.aggregation.smoothed_aggregation_solver is agg.smoothed_aggregation_solver
    assert callable(pyamg.aggregation.standard_aggregation)
    assert callable(pyamg.aggregation.fit_candidates)
    assert callable(pyamg.strength.symmetric_strength_of_connection)
    assert callable(pyamg.relaxation.relaxation.block_gauss_seidel)
    A = sp.identity(4, format="csr")
    for bad in ({"aggregate": "lloyd"}, {"smooth": "energy"}, {"strength": "classical"},
                {"coarse_solver": "splu"}, {"keep": True}):
        with pytest.raises(NotImplementedError):  # before any device call
            pyamg.aggregation.smoothed_aggregation_solver(A, **bad)


def test_sparse_tensor_mirror():
    import torch
    from mlamg import sparse_tensor as st
    rs = np.random.RandomState(0)
    A = (sp.random(9, 7, density=0.3, random_state=rs, format="coo") + sp.eye(9, 7)).tocoo()
    B = sp.random(7, 5, density=0.4, random_state=rs, format="coo")
    At = torch.sparse_coo_tensor(np.vstack([A.row, A.col]), A.data, A.shape).coalesce()
    Bt = torch.sparse_coo_tensor(np.vstack([B.row, B.col]), B.data, B.shape).coalesce()
    assert np.allclose(st.spspmm(At, Bt).to_dense().numpy(), (A @ B).toarray(), rtol=1e-14)
    X = rs.randn(7, 3)
    assert np.allclose(st.spmm(At, torch.as_tensor(X)).numpy(), A @ X, rtol=1e-14)
    assert np.array_equal(st.spT(At).to_dense().numpy(), A.toarray().T)
    d = st.diag(At)
    assert d.dtype == torch.float32 and d.shape == (7,)
    assert np.array_equal(d.numpy(), np.diag(A.toarray())[:7].astype(np.float32)
                          + np.where(np.diag(A.toarray())[:7] == 0, 1, 0))
    S = st.to_scipy(At)
    assert sp.isspmatrix_csr(S) and np.array_equal(S.toarray(), A.toarray())


def _names(code):
    out = set(code.co_names)
    for c in code.co_consts:
        if isinstance(c, types.CodeType):
            out |= _names(c)
    return out


def _resolve(ns, dotted):
    obj = ns[dotted[0]]
    for a in dotted[1:]:
        obj = getattr(obj, a)
    return obj


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present (GPU box)")
def test_reference_callers_resolve(compat, monkeypatch):
    import mlamg.graph
    import mlamg.multigrid
    import mlamg.sparse
    import mlamg.strength
    for name in ("ns.model", "ns.ga"):
        pkg = types.ModuleType(name)
        pkg.__path__ = []
        monkeypatch.setitem(sys.modules, name, pkg)
    for name in ("ns.model.agg_interp", "ns.model.data", "ns.ga.parga", "ns.ga.torch"):
        monkeypatch.setitem(sys.modules, name, types.ModuleType(name))
    path = os.path.join(REF, "utils", "common.py")
    common = types.ModuleType("common")
    with open(path) as fh:
        exec(compile(fh.read(), path, "exec"), common.__dict__)
    g = common.__dict__
    # every hot-path call of evaluate_dataset (:40-82) and evaluate_ref_conv (:84-111)
    hot = {
        ("ns", "lib", "graph", "lloyd_aggregation"): mlamg.graph.lloyd_aggregation,
        ("ns", "lib", "multigrid", "smoothed_aggregation_jacobi"):
            mlamg.multigrid.smoothed_aggregation_jacobi,
        ("ns", "lib", "multigrid", "amg_2_v"): mlamg.multigrid.amg_2_v,
        ("ns", "lib", "sparse_tensor", "to_scipy"): mlamg.sparse.to_scipy,
        ("pyamg", "aggregation", "lloyd_aggregation"): mlamg.graph.pyamg_lloyd_aggregation,
        ("pyamg", "strength", "evolution_strength_of_connection"):
            mlamg.strength.evolution_strength_of_connection,
    }
    for dotted, fn in hot.items():
        assert _resolve(g, dotted) is fn, dotted
    assert {"ns", "np"} <= _names(g["evaluate_dataset"].__code__)
    assert {"ns", "pyamg", "np"} <= _names(g["evaluate_ref_conv"].__code__)
    assert set(common.strength_measure_funcs) == {"abs", "evolution", "invabs", "unit", "olson"}
    # utils/evaluate_dataset.py's evaluate_dataset(dataset, method) (:59-101): its module level
    # parses argv and loads a dataset, so only the function is compiled, in a namespace holding
    # the script's own imports
    path = os.path.join(REF, "utils", "evaluate_dataset.py")
    with open(path) as fh:
        tree = ast.parse(fh.read(), path)
    imports = [n for n in tree.body if isinstance(n, (ast.Import, ast.ImportFrom))]
    fn = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "evaluate_dataset"]
    wanted = {"numpy", "numpy.linalg", "torch", "pyamg", "ns.lib.sparse", "ns.lib.sparse_tensor",
              "ns.lib.multigrid"}
    keep = [i for i in imports if isinstance(i, ast.Import)
            and all(a.name in wanted for a in i.names)]
    ns2 = {"common": common}
    exec(compile(ast.Module(body=keep + fn, type_ignores=[]), path, "exec"), ns2)
    import ns.lib.graph  # noqa: F401  (the script reaches ns.lib.graph through the ns package)
    code = ns2["evaluate_dataset"].__code__
    for dotted, fn_ in {
        ("ns", "lib", "graph", "modified_bellman_ford"): mlamg.graph.modified_bellman_ford,
        ("ns", "lib", "graph", "nearest_center_to_agg"): mlamg.graph.nearest_center_to_agg,
        ("ns", "lib", "sparse", "scipy_to_torch"): mlamg.sparse.to_torch_sparse,
        ("ns", "lib", "sparse", "torch_to_scipy"): mlamg.sparse.to_scipy,
        ("ns", "lib", "sparse_tensor", "to_scipy"): mlamg.sparse.to_scipy,
        ("pyamg", "aggregation", "lloyd_aggregation"): mlamg.graph.pyamg_lloyd_aggregation,
        ("ns", "lib", "multigrid", "amg_2_v"): mlamg.multigrid.amg_2_v,
        ("common", "strength_measure_funcs"): common.strength_measure_funcs,
    }.items():
        assert _resolve(ns2, dotted) is fn_, dotted
    assert {"ns", "np", "torch", "pyamg", "common", "la"} <= _names(code)


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present (GPU box)")
def test_reference_pyamg_pc_resolves(compat, monkeypatch):
    """ns/preconditioner/PyAMG.py exec'd from the reference file with Firedrake / PETSc /
    matplotlib stubs: its `pyamg.aggregation.smoothed_aggregation_solver` (:94) is this package's
    (tests/test_gpu_pyamg_sa.py runs that solver's :119 / :129 calls on the device)."""
    import mlamg.pyamg_compat.aggregation as agg
    fd = types.ModuleType("firedrake")

    class PCBase:  # the python-PC base class the PC derives from
        pass

    fd.PCBase = PCBase
    fd.__all__ = ["PCBase"]
    petsc = types.ModuleType("firedrake.petsc")
    petsc.PETSc = types.SimpleNamespace()
    asm = types.ModuleType("firedrake.assemble")
    asm.allocate_matrix = asm.assemble = None
    mpl = types.ModuleType("matplotlib")
    mpl.__path__ = []
    for name, mod in (("firedrake", fd), ("firedrake.petsc", petsc), ("firedrake.assemble", asm),
                      ("matplotlib", mpl), ("matplotlib.pyplot", types.ModuleType("pyplot"))):
        monkeypatch.setitem(sys.modules, name, mod)
    path = os.path.join(REF, "ns", "preconditioner", "PyAMG.py")
    mod = types.ModuleType("PyAMG_ref")
    with open(path) as fh:
        exec(compile(fh.read(), path, "exec"), mod.__dict__)
    g = mod.__dict__
    assert _resolve(g, ("pyamg", "aggregation", "smoothed_aggregation_solver")) is \
        agg.smoothed_aggregation_solver
    assert "pyamg" in _names(mod.PyAMG._createAmgSolver.__code__)
    assert "solve" in _names(mod.PyAMG._apply.__code__)
