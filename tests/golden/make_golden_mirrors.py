"""Golden vectors for the non-hot-path helpers of the three mirrored reference modules
(ns/lib/sparse.py col_normalize_csr / get_diagonal / triu / tril, ns/lib/graph.py
num_connected_components / check_aggregates_connected, ns/lib/multigrid.py jacobi_torch /
amg_2_v_torch), produced by running the REFERENCE functions (imported with the stubs of
make_golden.py) on seeded CPU inputs. Only inputs and outputs are stored
(tests/golden/reference_mirrors.npz). ns.lib.multigrid.gauss_seidel_torch is not recorded: as
written it passes a (1, n) right-hand side to torch.linalg.solve_triangular with an (n, n)
matrix and raises for n > 1 (checked here); the mirror solves the evident column form instead.

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_mirrors.py
"""
import os
import sys

import numpy as np
import scipy.sparse as sp

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import load_reference  # noqa: E402

import torch  # noqa: E402


def coo_arrays(T):
    T = T.coalesce()
    return T.indices().numpy(), T.values().numpy()


def main():
    mg, gr, spm = load_reference()
    out = {}
    rs = np.random.RandomState(7)
    # ---- sparse helpers
    M = sp.random(40, 30, density=0.15, random_state=rs, format="csr") + \
        sp.eye(40, 30, format="csr")
    for o in (1, 2):
        N = spm.col_normalize_csr(M, ord=o)
        out[f"colnorm{o}_data"] = N.data
        out[f"colnorm{o}_indices"] = N.indices
        out[f"colnorm{o}_indptr"] = N.indptr
    out["M_data"], out["M_indices"], out["M_indptr"] = M.data, M.indices, M.indptr
    S = sp.random(25, 25, density=0.2, random_state=rs, format="coo") + sp.eye(25)
    S = S.tocoo()
    T = torch.sparse_coo_tensor(torch.as_tensor(np.vstack([S.row, S.col])),
                                torch.as_tensor(S.data), S.shape).coalesce()
    out["S_row"], out["S_col"], out["S_val"] = S.row, S.col, S.data
    out["diag_vec"] = spm.get_diagonal(T).numpy()
    for d in (-2, 0, 1):
        i, v = coo_arrays(spm.triu(T, d))
        out[f"triu{d}_idx"], out[f"triu{d}_val"] = i, v
        i, v = coo_arrays(spm.tril(T, d))
        out[f"tril{d}_idx"], out[f"tril{d}_val"] = i, v
    # ---- graph helpers: 3 components (two paths and a cycle), and aggregates
    blocks = [sp.diags([1, 1], [-1, 1], shape=(m, m)) for m in (5, 7, 4)]
    G = sp.block_diag(blocks).tocsr()
    perm = rs.permutation(G.shape[0])
    G = G[perm][:, perm].tocsr()
    out["G_data"], out["G_indices"], out["G_indptr"] = G.data, G.indices, G.indptr
    out["ncc"] = np.array(gr.num_connected_components(G.tocsc()))
    grid = sp.diags([1, 1, 1, 1], [-1, 1, -6, 6], shape=(36, 36)).tocsr()
    out["grid_data"], out["grid_indices"], out["grid_indptr"] = grid.data, grid.indices, grid.indptr
    agg_ok = np.arange(36) // 6                                 # rows of the 6x6 grid
    agg_bad = np.where(np.arange(36) % 2 == 0, 0, 1)            # checkerboard-ish split
    for name, a in (("ok", agg_ok), ("bad", agg_bad)):
        Agg = sp.csr_matrix((np.ones(36), (np.arange(36), a)))
        out[f"agg_{name}"] = a
        out[f"aggconn_{name}"] = np.array(gr.check_aggregates_connected(grid, Agg))
    # ---- torch variants
    n = 64
    A = sp.diags([-1, 2, -1], [-1, 0, 1], shape=(n, n)).tocoo()
    AT = torch.sparse_coo_tensor(torch.as_tensor(np.vstack([A.row, A.col])),
                                 torch.as_tensor(A.data, dtype=torch.float64), A.shape).coalesce()
    b = torch.as_tensor(rs.randn(n))
    x0 = rs.randn(n)
    out["jt_b"], out["jt_x0"] = b.numpy(), x0
    out["jt_x"] = mg.jacobi_torch(AT, b, torch.as_tensor(x0.copy()), nu=3).numpy()
    Agg = sp.csr_matrix((np.ones(n), (np.arange(n), np.arange(n) // 4)))
    Pd = (sp.eye(n) - 0.5 * sp.diags(1 / A.tocsr().diagonal()) @ A.tocsr()) @ Agg
    Pd = Pd.tocoo()
    PT = torch.sparse_coo_tensor(torch.as_tensor(np.vstack([Pd.row, Pd.col])),
                                 torch.as_tensor(Pd.data, dtype=torch.float64), Pd.shape).coalesce()
    out["P_row"], out["P_col"], out["P_val"] = Pd.row, Pd.col, Pd.data
    out["a2vt_conv"] = np.array(float(mg.amg_2_v_torch(AT, PT, torch.zeros(n, dtype=torch.float64),
                                                       torch.as_tensor(x0.copy()), max_iter=12)))
    try:
        mg.gauss_seidel_torch(AT.to_dense(), b, torch.as_tensor(x0.copy()), nu=1)
        out["gst_raises"] = np.array(False)
    except Exception:
        out["gst_raises"] = np.array(True)
    np.savez_compressed(os.path.join(HERE, "reference_mirrors.npz"), **out)
    print("wrote reference_mirrors.npz:", sorted(out))


if __name__ == "__main__":
    main()
