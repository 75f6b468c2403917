"""Generate the golden vectors in tests/golden/*.npz by running the REFERENCE functions.

Container-only (needs /root/reference, which does not exist on the GPU box). The reference's
hot-path modules import packages that are absent here (pyamg, torch_sparse, firedrake, ...);
they are replaced by empty stub modules in sys.modules before the import, exactly as recorded in
SURVEY.md §8c. Where the reference calls into pyamg (gauss_seidel in amg_2_v, lloyd_cluster in
lloyd_aggregation) the stub delegates to the oracle's restatement (oracle/oracle.c), so those
vectors pin the reference's *driver* code around a restated pyamg kernel (pyamg itself:
parity unpinned). Nothing from the reference is copied: only inputs and outputs are stored.

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
"""
from __future__ import annotations

import bz2
import importlib
import os
import pickletools
import sys
import types

import numpy as np
import scipy.sparse as sp

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, ROOT)

from oracle import restated as orc  # noqa: E402  (the restated pyamg kernels for the stubs)


def _stub(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    sys.modules[name] = m
    return m


def install_stubs():
    def gs(A, x, b, iterations=1, sweep='forward'):
        assert sweep == 'forward'
        orc.gauss_seidel(A.tocsr(), x, b, iterations)

    def lloyd_cluster(G, seeds, maxiter=10):
        return orc.lloyd_cluster(G, seeds, maxiter=maxiter, canon=False)

    pyamg = _stub("pyamg")
    rel = _stub("pyamg.relaxation")
    relrel = _stub("pyamg.relaxation.relaxation", gauss_seidel=gs)
    rel.relaxation = relrel
    pyamg.relaxation = rel
    graph = _stub("pyamg.graph", lloyd_cluster=lloyd_cluster)
    pyamg.graph = graph
    _stub("torch_sparse")


def load_reference():
    install_stubs()
    sys.path.insert(0, REF)
    mg = importlib.import_module("ns.lib.multigrid")
    gr = importlib.import_module("ns.lib.graph")
    spm = importlib.import_module("ns.lib.sparse")
    return mg, gr, spm


def grid_arrays(path):
    """Pull the CSR arrays out of a .grid (bz2 pickle) WITHOUT unpickling: walk the opcodes with
    pickletools and rebuild only the raw ndarray payloads (see mlamg/gridio.py)."""
    sys.path.insert(0, os.path.join(ROOT, "ml-amg_amd"))
    from mlamg.gridio import parse_grid_bytes
    with bz2.open(path, "rb") as fh:
        return parse_grid_bytes(fh.read())


def mlamg_ref_instance(A, P, w=2.0 / 3.0, rtol=1e-8):
    """An MLAMG object (ns/preconditioner/MLAMG.py) with A, Dinv, A_H_lu set as _createAmgSolver
    would, built without firedrake: the class body is exec'd from the reference file with stub
    firedrake/torch_geometric modules, then amg_2_v/jacobi are called unmodified."""
    import scipy.sparse.linalg as spla

    class PCBase:  # firedrake.PCBase stand-in (only the base class is needed)
        pass

    fd = _stub("firedrake", PCBase=PCBase)
    fd.__all__ = ["PCBase"]
    _stub("firedrake.petsc", PETSc=None)
    _stub("firedrake.assemble", allocate_matrix=None, assemble=None)
    _stub("matplotlib")
    _stub("matplotlib.pyplot")
    _stub("ns.model.ali_interp", InterpolationNetwork=None)
    sys.modules.setdefault("ns.model", types.ModuleType("ns.model"))
    mod = importlib.import_module("ns.preconditioner.MLAMG")
    obj = object.__new__(mod.MLAMG)
    obj.A = A
    obj.Dinv = sp.diags(1.0 / A.diagonal()) * w
    obj.A_H = P.T @ A @ P
    obj.A_H_lu = spla.splu(obj.A_H.tocsc(), permc_spec='COLAMD')
    obj.amg_rtol = rtol
    return obj


def main():
    mg, gr, spm = load_reference()
    import torch

    out = {}
    rng = np.random.RandomState(0)
    # ---------------------------------------------------------------- matrices
    n1 = 1024
    A1 = (sp.eye(n1) * 2 - sp.eye(n1, k=-1) - sp.eye(n1, k=1)).tocsr()          # C1
    Agg1 = np.zeros((n1, (n1 + 2) // 3))
    for a in range(Agg1.shape[1]):
        Agg1[3 * a:3 * (a + 1), a] = 1.
    Agg1 = sp.csr_matrix(Agg1)
    m2 = 32
    T = (sp.eye(m2) * 2 - sp.eye(m2, k=-1) - sp.eye(m2, k=1))
    A2 = (sp.kron(sp.eye(m2), T) + sp.kron(T, sp.eye(m2))).tocsr()              # 2D 5-pt 32^2
    A2.sort_indices()
    g = grid_arrays(os.path.join(REF, "demos", "laplace_3d.grid"))
    A3 = sp.csr_matrix((g["data"], g["indices"], g["indptr"]))                   # 1331 aniso P1
    # random-coefficient SPD (tie-free graph weights)
    m4 = 24
    idx = np.arange(m4 * m4)
    xs, ys = idx % m4, idx // m4
    rows, cols, vals = [], [], []
    for (dx, dy) in ((1, 0), (0, 1)):
        ok = (xs + dx < m4) & (ys + dy < m4)
        i = idx[ok]
        j = i + dx + dy * m4
        w = rng.uniform(0.5, 2.0, len(i))
        rows += [i, j]
        cols += [j, i]
        vals += [-w, -w]
    W = sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                      shape=(m4 * m4, m4 * m4))
    A4 = (W + sp.diags(-np.asarray(W.sum(axis=1)).ravel() + 0.1)).tocsr()
    A4.sort_indices()
    mats = {"c1": A1, "p2d": A2, "lap3d": A3, "rnd": A4}
    for k, A in mats.items():
        out[f"{k}_indptr"] = A.indptr.astype(np.int32)
        out[f"{k}_indices"] = A.indices.astype(np.int32)
        out[f"{k}_data"] = A.data.astype(np.float64)
        out[f"{k}_shape"] = np.array(A.shape)
    # ---------------------------------------------------------------- SpMV / Jacobi (reference)
    for k, A in mats.items():
        n = A.shape[0]
        x = np.random.RandomState(1).randn(n)
        b = np.random.RandomState(2).randn(n)
        out[f"{k}_x"] = x
        out[f"{k}_b"] = b
        out[f"{k}_Ax"] = A @ x
        out[f"{k}_resid"] = b - A @ x
        for nu in (1, 2, 5):
            out[f"{k}_jacobi_nu{nu}"] = mg.jacobi(A, b, x.copy(), omega=0.666, nu=nu)
    # ---------------------------------------------------------------- SA prolongator + Galerkin
    for k, A, Agg in (("c1", A1, Agg1),):
        # record the eigenvalue ARPACK returns INSIDE the reference call (ARPACK's random start
        # makes separate calls differ in the last bits)
        import scipy.sparse.linalg as spla_mod
        seen = []
        real_eigs = spla_mod.eigs

        def spy_eigs(*a, **kw):
            v = real_eigs(*a, **kw)
            seen.append(v)
            return v

        mg.spla.eigs = spy_eigs
        try:
            P = mg.smoothed_aggregation_jacobi(A, Agg)
        finally:
            mg.spla.eigs = real_eigs
        out[f"{k}_omega"] = (4. / 3.) / np.abs(seen[0]).item()
        out[f"{k}_P_indptr"], out[f"{k}_P_indices"], out[f"{k}_P_data"] = P.indptr, P.indices, P.data
        AH = (P.T @ A @ P).tocsr()
        AH.sort_indices()
        out[f"{k}_AH_indptr"], out[f"{k}_AH_indices"], out[f"{k}_AH_data"] = AH.indptr, AH.indices, AH.data
        out[f"{k}_Agg_indptr"], out[f"{k}_Agg_indices"] = Agg.indptr, Agg.indices
    # ---------------------------------------------------------------- amg_2_v (reference driver)
    P1 = sp.csr_matrix((out["c1_P_data"], out["c1_P_indices"], out["c1_P_indptr"]), shape=Agg1.shape)
    x0 = np.random.RandomState(0).normal(0, 1, n1)
    b0 = np.zeros(n1)
    xr, conv, err, iters = mg.amg_2_v(A1, P1, b0, x0, error_tol=1e-10)
    out["c1_amg2v_err_x"], out["c1_amg2v_err_conv"], out["c1_amg2v_err_hist"] = xr, conv, err
    xr, conv, err, iters = mg.amg_2_v(A1, P1, b0, x0 / np.linalg.norm(x0), res_tol=1e-10)
    out["c1_amg2v_res_x"], out["c1_amg2v_res_conv"], out["c1_amg2v_res_hist"] = xr, conv, err
    # conv-factor quirks (multigrid.py:201-208): reference driver with max_iter = 1..7 and an
    # unreachable tolerance, so the history has exactly that many entries
    qs = []
    for L in range(1, 8):
        qs.append(float(mg.amg_2_v(A1, P1, b0, x0, error_tol=1e-300, max_iter=L)[1]))
    out["conv_quirk_values"] = np.array(qs)
    # ---------------------------------------------------------------- MLAMG.amg_2_v residual histories
    obj = mlamg_ref_instance(A1, P1)
    hist = []
    for k in range(1, 9):
        xk = obj.amg_2_v(P1, b0, x0.copy(), max_iter=k)
        hist.append(np.linalg.norm(b0 - A1 @ xk))
    out["c1_mlamg_hist"] = np.array(hist)
    out["c1_mlamg_x8"] = xk
    # ---------------------------------------------------------------- Bellman-Ford / aggregates
    for k, A, alpha in (("p2d", A2, 0.1), ("rnd", A4, 0.1), ("lap3d", A3, 0.1)):
        n = A.shape[0]
        C = sp.csr_matrix((1.0 / np.abs(A.data), A.indices, A.indptr), A.shape)
        seeds = np.random.RandomState(0).permutation(n)[:int(np.ceil(alpha * n))]
        seeds_T = torch.Tensor(seeds).long()
        dist, nearest = gr.modified_bellman_ford(spm.to_torch_sparse(C), seeds_T)
        out[f"{k}_bf_seeds"] = seeds
        out[f"{k}_bf_dist"] = dist.numpy()
        out[f"{k}_bf_nearest"] = nearest.numpy()
        agg = gr.nearest_center_to_agg(seeds_T, nearest)
        agg = agg.coalesce()
        out[f"{k}_agg_idx"] = agg.indices().numpy()
    # lloyd_aggregation driver (seeds / AggOp layout) around the restated lloyd_cluster
    C = sp.csr_matrix((1.0 / np.abs(A4.data), A4.indices, A4.indptr), A4.shape)
    AggOp, roots, seeds = gr.lloyd_aggregation(C, ratio=0.1, distance='same', rand=0)
    out["rnd_lloyd_roots"], out["rnd_lloyd_seeds"] = roots, seeds
    out["rnd_lloyd_agg_indptr"], out["rnd_lloyd_agg_indices"] = AggOp.indptr, AggOp.indices
    path = os.path.join(HERE, "reference_vectors.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}: {len(out)} arrays, {os.path.getsize(path)} bytes")


if __name__ == "__main__":
    main()
