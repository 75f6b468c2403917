"""CPU: the mirror modules can replace the reference modules wholesale (INTEGRATION.md §2:
sys.modules["ns.lib.multigrid" / "ns.lib.graph" / "ns.lib.sparse"] = mlamg.*), i.e. every public
name of /root/reference/ns/lib/{multigrid,graph,sparse}.py resolves through the alias, and the
non-hot-path helpers reproduce the reference's own outputs (tests/golden/reference_mirrors.npz,
made by tests/golden/make_golden_mirrors.py from the reference functions). No GPU calls."""
import os
import sys

import numpy as np
import pytest
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden", "reference_mirrors.npz")

# every function / alias the reference modules define (ns/lib/multigrid.py:15,48,58,93,102,111,
# 213; ns/lib/graph.py:7,56,89,125,156; ns/lib/sparse.py:8,20,35,51,78,105,106)
PUBLIC = {
    "ns.lib.multigrid": ("jacobi", "jacobi_torch", "gauss_seidel", "gauss_seidel_torch",
                         "smoothed_aggregation_jacobi", "amg_2_v", "amg_2_v_torch"),
    "ns.lib.graph": ("modified_bellman_ford", "nearest_center_to_agg",
                     "num_connected_components", "check_aggregates_connected",
                     "lloyd_aggregation"),
    "ns.lib.sparse": ("col_normalize_csr", "to_torch_sparse", "get_diagonal", "triu", "tril",
                      "scipy_to_torch", "torch_to_scipy"),
}


@pytest.fixture(scope="module")
def g():
    return dict(np.load(GOLD, allow_pickle=False))


@pytest.fixture
def alias(monkeypatch):
    import mlamg.graph
    import mlamg.multigrid
    import mlamg.sparse
    for name, mod in (("ns.lib.multigrid", mlamg.multigrid), ("ns.lib.graph", mlamg.graph),
                      ("ns.lib.sparse", mlamg.sparse)):
        monkeypatch.setitem(sys.modules, name, mod)
    return sys.modules


def test_every_public_name_through_the_alias(alias):
    import importlib
    for mod, names in PUBLIC.items():
        m = importlib.import_module(mod)
        missing = [n for n in names if not callable(getattr(m, n, None))]
        assert not missing, (mod, missing)


def test_col_normalize_csr(alias, g):
    spm = alias["ns.lib.sparse"]
    M = sp.csr_matrix((g["M_data"], g["M_indices"], g["M_indptr"]), shape=(40, 30))
    for o in (1, 2):
        N = spm.col_normalize_csr(M, ord=o)
        assert np.array_equal(N.indptr, g[f"colnorm{o}_indptr"])
        assert np.array_equal(N.indices, g[f"colnorm{o}_indices"])
        assert np.array_equal(N.data, g[f"colnorm{o}_data"])


def test_diag_triu_tril(alias, g):
    import torch
    spm = alias["ns.lib.sparse"]
    T = torch.sparse_coo_tensor(torch.as_tensor(np.vstack([g["S_row"], g["S_col"]])),
                                torch.as_tensor(g["S_val"]), (25, 25)).coalesce()
    assert np.array_equal(spm.get_diagonal(T).numpy(), g["diag_vec"])
    for d in (-2, 0, 1):
        for fn in ("triu", "tril"):
            R = getattr(spm, fn)(T, d).coalesce()
            assert np.array_equal(R.indices().numpy(), g[f"{fn}{d}_idx"])
            assert np.array_equal(R.values().numpy(), g[f"{fn}{d}_val"])


def test_graph_helpers(alias, g):
    gr = alias["ns.lib.graph"]
    G = sp.csr_matrix((g["G_data"], g["G_indices"], g["G_indptr"]), shape=(16, 16))
    assert gr.num_connected_components(G.tocsc()) == int(g["ncc"]) == 3
    grid = sp.csr_matrix((g["grid_data"], g["grid_indices"], g["grid_indptr"]), shape=(36, 36))
    for name in ("ok", "bad"):
        a = g[f"agg_{name}"]
        Agg = sp.csr_matrix((np.ones(36), (np.arange(36), a)))
        assert gr.check_aggregates_connected(grid, Agg) == bool(g[f"aggconn_{name}"])


def test_torch_variants(alias, g):
    import torch
    mg = alias["ns.lib.multigrid"]
    n = 64
    A = sp.diags([-1, 2, -1], [-1, 0, 1], shape=(n, n)).tocoo()
    AT = torch.sparse_coo_tensor(torch.as_tensor(np.vstack([A.row, A.col])),
                                 torch.as_tensor(A.data, dtype=torch.float64), A.shape).coalesce()
    x = mg.jacobi_torch(AT, torch.as_tensor(g["jt_b"]), torch.as_tensor(g["jt_x0"].copy()), nu=3)
    assert np.array_equal(x.numpy(), g["jt_x"])
    PT = torch.sparse_coo_tensor(torch.as_tensor(np.vstack([g["P_row"], g["P_col"]])),
                                 torch.as_tensor(g["P_val"]), (n, 16)).coalesce()
    conv = mg.amg_2_v_torch(AT, PT, torch.zeros(n, dtype=torch.float64),
                            torch.as_tensor(g["jt_x0"].copy()), max_iter=12)
    # torch.lu/lu_solve (reference) vs torch.linalg.lu_factor/lu_solve (same LAPACK getrf/getrs)
    assert abs(float(conv) - float(g["a2vt_conv"])) <= 1e-12 * abs(float(g["a2vt_conv"]))
    # gauss_seidel_torch: the reference's (1, n) right-hand side raises (recorded); the mirror
    # solves tril(A) x = b - triu(A, 1) x as a column: one forward Gauss-Seidel sweep
    assert bool(g["gst_raises"])
    b = torch.as_tensor(g["jt_b"])
    xg = mg.gauss_seidel_torch(AT, b, torch.as_tensor(g["jt_x0"].copy()), nu=1)
    Ad = A.toarray()
    ref = np.linalg.solve(np.tril(Ad), g["jt_b"] - np.triu(Ad, 1) @ g["jt_x0"])
    assert np.allclose(xg.numpy(), ref, rtol=1e-13, atol=1e-13)
