"""TEST INFRASTRUCTURE ONLY — numpy/scipy restatement of the reference hot path.

Each function cites the reference lines it restates. scipy calls are the reference's own
arithmetic (the reference is scipy code), so wherever the reference uses scipy this module uses
the same scipy call. pyamg (absent here) is restated in oracle/oracle.c.
"""
from __future__ import annotations

import ctypes
import math
import os

import numpy as np
import numpy.linalg as la
import scipy.sparse as sp
import scipy.sparse.linalg as spla

from . import build as _build

_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        path = _build.OUT
        if not os.path.exists(path):
            path = _build.build()
        L = ctypes.CDLL(path)
        vp = ctypes.c_void_p
        i64 = ctypes.c_int64
        L.ref_csr_matvec.argtypes = [i64, vp, vp, vp, vp, vp]
        L.ref_gauss_seidel.argtypes = [i64, vp, vp, vp, vp, vp, ctypes.c_int]
        L.ref_bellman_ford_torch.argtypes = [i64, vp, vp, vp, vp, i64, vp, vp]
        L.ref_bellman_ford_torch.restype = ctypes.c_int
        L.canon_bellman_ford.argtypes = [i64, vp, vp, vp, vp, i64, vp, vp]
        for f in (L.pyamg_bellman_ford, L.pyamg_bellman_ford_f64):
            f.argtypes = [i64, vp, vp, vp, vp, i64, vp, vp]
            f.restype = ctypes.c_int
        L.vec_matvec.argtypes = [i64, vp, vp, vp, vp, vp]
        L.lloyd_cluster.argtypes = [i64, vp, vp, vp, ctypes.c_int32, vp, ctypes.c_int, vp, vp,
                                    ctypes.c_int]
        L.lloyd_cluster.restype = ctypes.c_int
        L.pyamg_symmetric_strength.argtypes = [i64, vp, vp, vp, ctypes.c_double, vp, vp, vp]
        L.pyamg_symmetric_strength.restype = i64
        L.pyamg_standard_aggregation.argtypes = [i64, vp, vp, vp, vp]
        L.pyamg_standard_aggregation.restype = i64
        L.pyamg_block_gauss_seidel.argtypes = [i64, vp, vp, vp, vp, vp, ctypes.c_int,
                                               ctypes.c_int]
        L.pyamg_gauss_seidel.argtypes = [i64, vp, vp, vp, vp, vp, ctypes.c_int, ctypes.c_int]
        L.pyamg_fit_candidates.argtypes = [i64, vp, i64, vp, ctypes.c_double, vp, vp]
        _LIB = L
    return _LIB


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _csr_arrays(A):
    A = A.tocsr()
    return (np.ascontiguousarray(A.indptr, dtype=np.int32),
            np.ascontiguousarray(A.indices, dtype=np.int32),
            np.ascontiguousarray(A.data, dtype=np.float64))


# ---------------------------------------------------------------- sparse primitives
def csr_matvec(A, x):
    """scipy csr_matvec (A@x), restated in C."""
    ip, ij, ax = _csr_arrays(A)
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.empty(A.shape[0])
    lib().ref_csr_matvec(A.shape[0], _p(ip), _p(ij), _p(ax), _p(x), _p(y))
    return y


def vec_matvec(A, x, vw=None):
    """The device CSR-vector summation order (oracle.c vec_matvec): one canonical order for
    every lane width (vw, 64..512, is accepted and checked but does not change the result)."""
    if vw is not None and vw not in (64, 128, 256, 512):
        raise ValueError(f"vector width must be 64, 128, 256 or 512, got {vw}")
    ip, ij, ax = _csr_arrays(A)
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.empty(A.shape[0])
    lib().vec_matvec(A.shape[0], _p(ip), _p(ij), _p(ax), _p(x), _p(y))
    return y


def mv(M, x, vw=0):
    """M@x in scipy's order (vw == 0) or the device's canonical vector order (vw > 0)."""
    return M @ x if not vw else vec_matvec(M, x)


def gauss_seidel(A, x, b, iterations=1):
    """pyamg.relaxation.relaxation.gauss_seidel(A, x, b, iterations) forward, in place
    (called at ns/lib/multigrid.py:175,184)."""
    ip, ij, ax = _csr_arrays(A)
    assert x.dtype == np.float64 and x.flags.c_contiguous
    b = np.ascontiguousarray(b, dtype=np.float64)
    lib().ref_gauss_seidel(A.shape[0], _p(ip), _p(ij), _p(ax), _p(x), _p(b), int(iterations))
    return x


def pyamg_gauss_seidel(A, x, b, iterations=1, sweep="forward"):
    """pyamg.relaxation.relaxation.gauss_seidel(A, x, b, iterations, sweep) in place: the
    forward arithmetic of gauss_seidel above, rows n-1..0 for 'backward', forward then backward
    per iteration for 'symmetric' (amg_core gauss_seidel with row_step -1). Parity unpinned
    (pyamg absent)."""
    ip, ij, ax = _csr_arrays(A)
    assert x.dtype == np.float64 and x.flags.c_contiguous
    b = np.ascontiguousarray(b, dtype=np.float64)
    lib().pyamg_gauss_seidel(A.shape[0], _p(ip), _p(ij), _p(ax), _p(x), _p(b), int(iterations),
                             _SWEEPS[sweep])
    return x


def jacobi_mg(A, b, x, Dinv=None, omega=0.666, nu=2):
    """ns/lib/multigrid.py:15-45."""
    if Dinv is None:
        Dinv = sp.diags(1.0 / A.diagonal())
    for _ in range(nu):
        x += omega * Dinv @ b - omega * Dinv @ A @ x
    return x


def jacobi_mlamg(A, Dinv_w, b, x, nu=2):
    """ns/preconditioner/MLAMG.py:143-146 with Dinv_w = sp.diags(1/diag)*w (MLAMG.py:104)."""
    for _ in range(nu):
        x += Dinv_w @ (b - A @ x)
    return x


def mlamg_dinv(A, w=2.0 / 3.0):
    """MLAMG.py:104."""
    return sp.diags(1.0 / A.diagonal()) * w


def smoothed_aggregation_jacobi(A, Agg, omega=None):
    """ns/lib/multigrid.py:102-108 (omega from ARPACK unless given)."""
    n = A.shape[0]
    Dinv = sp.diags([1.0 / A.diagonal()], [0])
    if omega is None:
        omega = (4. / 3.) / np.abs(spla.eigs(Dinv @ A, k=1, return_eigenvectors=False)).item()
    smoother = (sp.eye(n) - omega * Dinv @ A)
    P = smoother @ Agg
    return P, omega


def arpack_lambda_max(A):
    Dinv = sp.diags([1.0 / A.diagonal()], [0])
    return float(np.abs(spla.eigs(Dinv @ A, k=1, return_eigenvectors=False)).item())


def canonical(M):
    """CSR with sorted indices (values untouched) for array-level comparison."""
    M = sp.csr_matrix(M)
    M = M.copy()
    M.has_sorted_indices = False
    M.sort_indices()
    return M


def galerkin(A, P):
    """ns/lib/multigrid.py:165 `P.T@A@P` (scipy CSC path), as sorted CSR."""
    return canonical((P.T @ A @ P).tocsr())


# ---------------------------------------------------------------- drivers
def conv_factor(err):
    """ns/lib/multigrid.py:201-208."""
    if len(err) != 1:
        try:
            err_n = min(len(err) // 3, 10)
            conv_factor = (err[-1] / err[-err_n]) ** (1 / (err_n - 1))
        except Exception:
            conv_factor = 0
    else:
        conv_factor = 0
    return conv_factor


def amg_2_v(A, P, b, x, pre_smoothing_steps=1, post_smoothing_steps=1, jacobi_weight=0.666,
            res_tol=None, error_tol=None, max_iter=500, singular=False, smoother="gauss_seidel"):
    """ns/lib/multigrid.py:111-210; smoother='jacobi' swaps in the MLAMG.py:143-146 Jacobi form
    with weight jacobi_weight. singular=True: lsqr coarse solve (scipy defaults, :178-179) and
    mean removal after post-smoothing (:186-187), no factorization."""
    if res_tol is None and error_tol is None:
        raise RuntimeError('One of res_tol or error_tol must be set!')
    tol = res_tol if res_tol is not None else error_tol
    err = np.zeros(max_iter)
    A_H = P.T @ A @ P
    if singular:
        def coarse(r_H):
            return spla.lsqr(P.T @ A @ P, r_H)[0]
    else:
        try:
            coarse = spla.factorized(A_H)
        except Exception:
            return x, np.float64(1.), err, 0
    x = x.copy()
    if smoother == "jacobi":
        Dw = mlamg_dinv(A, jacobi_weight)

        def smooth(nu):
            jacobi_mlamg(A, Dw, b, x, nu)
    else:
        def smooth(nu):
            gauss_seidel(A, x, b, iterations=nu)
    for i in range(max_iter):
        smooth(pre_smoothing_steps)
        x += P @ coarse(P.T @ (b - A @ x))
        smooth(post_smoothing_steps)
        if singular:
            x -= np.mean(x)
        if res_tol is not None:
            e = la.norm(b - A @ x, 2)
        else:
            e = la.norm(x, 2)
        err[i] = e
        if e <= tol:
            err = err[:i + 1]
            break
    return x, conv_factor(err), err, len(err)


def mlamg_amg_2_v(A, P, Dinv_w, b, x, pre_smoothing_steps=1, post_smoothing_steps=1,
                  max_iter=500, amg_rtol=1e-8):
    """ns/preconditioner/MLAMG.py:148-197 (A_H_lu = splu(P^T A P, COLAMD), :121-122).
    Returns (x, residual-norm history)."""
    A_H = (P.T @ A @ P).tocsc()
    lu = spla.splu(A_H, permc_spec='COLAMD')
    hist = []
    x = x.copy()
    for i in range(max_iter):
        x = jacobi_mlamg(A, Dinv_w, b, x, nu=pre_smoothing_steps)
        x += P @ lu.solve(P.T @ (b - A @ x))
        x = jacobi_mlamg(A, Dinv_w, b, x, nu=post_smoothing_steps)
        r = la.norm(b - A @ x, 2)
        hist.append(r)
        if r <= amg_rtol:
            break
    return x, np.array(hist)


# ---------------------------------------------------------------- aggregation
def modified_bellman_ford(C, centers):
    """ns/lib/graph.py:7-53 on S_T = scipy_to_torch(C): fp32 sequential push over the
    coalesced COO (= sorted CSR) order. Returns (distance fp32, nearest_center int64, sweeps)."""
    C = canonical(C)
    ip, ij, _ = _csr_arrays(C)
    w = np.ascontiguousarray(C.data, dtype=np.float32)
    c = np.ascontiguousarray(centers, dtype=np.int64)
    n = C.shape[0]
    d = np.empty(n, dtype=np.float32)
    nc = np.empty(n, dtype=np.int64)
    sweeps = lib().ref_bellman_ford_torch(n, _p(ip), _p(ij), _p(w), _p(c), len(c), _p(d), _p(nc))
    return d, nc, sweeps


def canon_bellman_ford(C, seeds):
    """Same distances with the device's order-independent label rule; label -1 unreachable."""
    C = canonical(C)
    ip, ij, _ = _csr_arrays(C)
    w = np.ascontiguousarray(C.data, dtype=np.float32)
    s = np.ascontiguousarray(seeds, dtype=np.int32)
    n = C.shape[0]
    d = np.empty(n, dtype=np.float32)
    lab = np.empty(n, dtype=np.int32)
    lib().canon_bellman_ford(n, _p(ip), _p(ij), _p(w), _p(s), len(s), _p(d), _p(lab))
    return d, lab


def pyamg_bellman_ford(G, seeds, dtype=None):
    """pyamg 4.x graph.bellman_ford(G, seeds) as ns/model/agg_interp.py:471-475 calls it: G a
    scipy COO/CSR (asgraph -> csr_matrix: duplicates summed, rows sorted), amg_core sweeps in
    the graph's dtype (float32 for the CNet weights; dtype=np.float64 widens them first).
    Returns (distances, nearest_seed int32 seed node id or -1, sweeps)."""
    G = sp.csr_matrix(G)
    G.sum_duplicates()
    dt = np.dtype(dtype or (np.float64 if G.dtype == np.float64 else np.float32))
    ip = np.ascontiguousarray(G.indptr, dtype=np.int32)
    ij = np.ascontiguousarray(G.indices, dtype=np.int32)
    w = np.ascontiguousarray(G.data, dtype=dt)
    s = np.ascontiguousarray(seeds, dtype=np.int32)
    n = G.shape[0]
    d = np.empty(n, dtype=dt)
    z = np.empty(n, dtype=np.int32)
    f = lib().pyamg_bellman_ford_f64 if dt == np.float64 else lib().pyamg_bellman_ford
    sweeps = f(n, _p(ip), _p(ij), _p(w), _p(s), len(s), _p(d), _p(z))
    return d, z, sweeps


def nearest_center_to_agg(top_k, nearest_center):
    """ns/lib/graph.py:56-86 as a scipy CSR of ones (n x m)."""
    n, m = len(nearest_center), len(top_k)
    inv = {int(k): i for i, k in enumerate(top_k)}
    cols = np.array([inv[int(c)] for c in nearest_center], dtype=np.int64)
    return sp.csr_matrix((np.ones(n), (np.arange(n), cols)), shape=(n, m))


def lloyd_cluster(G, seeds, maxiter=10, canon=False):
    """pyamg 4.x graph.lloyd_cluster (ns/lib/graph.py:232). Returns (distances, clusters, seeds)."""
    ip, ij, ax = _csr_arrays(G)
    s = np.array(seeds, dtype=np.int32)
    n = G.shape[0]
    d = np.empty(n)
    c = np.empty(n, dtype=np.int32)
    lib().lloyd_cluster(n, _p(ip), _p(ij), _p(ax), len(s), _p(s), int(maxiter), _p(d), _p(c),
                        int(bool(canon)))
    return d, c, s


def lloyd_aggregation(C, ratio=0.03, distance='unit', maxiter=10, rand=None, canon=False):
    """ns/lib/graph.py:156-239 with the lloyd_cluster restatement."""
    if distance == 'unit':
        data = np.ones_like(C.data).astype(float)
    elif distance == 'abs':
        data = abs(C.data)
    elif distance == 'inv':
        data = 1.0 / abs(C.data)
    elif distance == 'same':
        data = C.data
    elif distance == 'min':
        data = C.data - C.data.min()
    else:
        raise ValueError(distance)
    if rand is None:
        rand = np.random
    elif isinstance(rand, int):
        rand = np.random.RandomState(rand)
    G = C.__class__((data, C.indices, C.indptr), shape=C.shape)
    if sp.isspmatrix_csc(G):
        G = sp.csr_matrix((G.data, G.indices, G.indptr), shape=G.shape)
    N = C.shape[0]
    num_seeds = int(np.ceil(ratio * N))
    seeds = rand.permutation(N)[:num_seeds]
    _, clusters, roots = lloyd_cluster(G, np.copy(seeds), maxiter=maxiter, canon=canon)
    row = (clusters >= 0).nonzero()[0]
    col = clusters[row]
    AggOp = sp.coo_matrix((np.ones(len(row), dtype='int8'), (row, col)),
                          shape=(G.shape[0], num_seeds)).tocsr()
    return AggOp, roots, seeds


def pyamg_lloyd_aggregation(C, ratio=0.03, distance='unit', maxiter=10):
    """pyamg 4.x pyamg.aggregation.lloyd_aggregation (absent here; restated from its published
    source — the reference's own graph.py:156-239 says it was adapted from it; parity unpinned
    w.r.t. pyamg itself), as utils/common.py:91 and utils/evaluate_dataset.py:77 call it:
    num_seeds = int(min(max(ratio*N, 1), N)); pyamg.graph.lloyd_cluster(G, num_seeds, maxiter)
    draws np.random.permutation(N)[:num_seeds] from the GLOBAL generator; returns (AggOp, seeds)."""
    if ratio <= 0 or ratio > 1:
        raise ValueError('ratio must be > 0.0 and <= 1.0')
    if not (sp.isspmatrix_csr(C) or sp.isspmatrix_csc(C)):
        raise TypeError('expected csr_matrix or csc_matrix')
    if distance == 'unit':
        data = np.ones_like(C.data).astype(float)
    elif distance == 'abs':
        data = abs(C.data)
    elif distance == 'inv':
        data = 1.0 / abs(C.data)
    elif distance == 'same':
        data = C.data
    elif distance == 'min':
        data = C.data - C.data.min()
    else:
        raise ValueError(distance)
    G = C.__class__((data, C.indices, C.indptr), shape=C.shape)
    if sp.isspmatrix_csc(G):
        G = sp.csr_matrix((G.data, G.indices, G.indptr), shape=G.shape)
    N = G.shape[0]
    num_seeds = int(min(max(ratio * N, 1), N))
    seeds = np.random.permutation(N)[:num_seeds].astype('intc')
    _, clusters, seeds = lloyd_cluster(G, seeds, maxiter=maxiter)
    row = (clusters >= 0).nonzero()[0]
    col = clusters[row]
    AggOp = sp.coo_matrix((np.ones(len(row), dtype='int8'), (row, col)),
                          shape=(N, num_seeds)).tocsr()
    return AggOp, seeds.astype('intc')


# ---------------------------------------------------------------- multilevel (device recipe)
STRENGTH = {
    "abs": lambda A: abs(A),
    "invabs": lambda A: sp.csr_matrix((1.0 / np.abs(A.data), A.indices, A.indptr), A.shape),
    "unit": lambda A: sp.csr_matrix((np.ones_like(A.data), A.indices, A.indptr), A.shape),
}


def reference_aggregates(C, n, alpha, seed=0):
    """utils/evaluate_dataset.py:80-90 ("dumb" method): seeds = RandomState(seed).permutation(N)
    [:ceil(alpha N)] (unsorted), modified_bellman_ford on C in fp32 (graph.py:7-53), Agg =
    nearest_center_to_agg(seeds, nearest_center) (graph.py:56-86: column t = seeds[t]).
    Returns (seeds, nearest_center int64, Agg CSR n x k)."""
    k = int(math.ceil(alpha * n))
    seeds = np.random.RandomState(seed).permutation(n)[:k]
    _, near, _ = modified_bellman_ford(C, seeds)
    pos = np.full(n, -1, dtype=np.int64)
    pos[seeds] = np.arange(k)
    col = pos[near]
    if (col < 0).any():  # the reference's dict lookup (graph.py:80-82) raises
        raise KeyError(int(near[col < 0][0]))
    Agg = sp.csr_matrix((np.ones(n), (np.arange(n), col)), shape=(n, k))
    return seeds, near, Agg


def build_hierarchy(A, alpha=0.1, strength_mode="invabs", seed=0, sort_seeds=True,
                    max_coarse=1000, max_levels=10, jacobi_weight=2.0 / 3.0, omegas=None,
                    rhos=None, aggregation="bellman_ford", coarse_order="seed"):
    """CPU restatement of mlamg.hierarchy.Hierarchy.build (aggregation='bellman_ford' or
    'reference': level 0 by reference_aggregates, columns in seed order or, with
    coarse_order='sorted', relabelled in ascending seed order).

    omegas: per-level SA weights to use (e.g. the device's); None -> ARPACK (multigrid.py:105).
    rhos: per-level rho(D^-1 A) for the evolution measures ('evolution', 'olson').
    Returns a list of level dicts and the coarsest matrix.
    """
    levels = []
    A = canonical(A)
    while A.shape[0] > max_coarse and len(levels) + 1 < max_levels:
        n = A.shape[0]
        if strength_mode in ("evolution", "olson"):
            C = strength_measure(A, strength_mode, rho=None if rhos is None else rhos[len(levels)])
        else:
            C = STRENGTH[strength_mode](A)
        k = int(math.ceil(alpha * n))
        if aggregation == "reference" and not levels:
            seeds, lab, Agg = reference_aggregates(C, n, alpha, seed)
            if coarse_order == "sorted":
                order = np.argsort(seeds)
                seeds = seeds[order]
                Agg = Agg[:, order].tocsr()
                Agg.sort_indices()
        else:
            seeds = np.random.RandomState(seed).permutation(n)[:k]
            if sort_seeds:
                seeds = np.sort(seeds)
            _, lab = canon_bellman_ford(C, seeds)
            pos = np.full(n, -1, dtype=np.int64)
            pos[seeds] = np.arange(k)
            col = np.where(lab >= 0, pos[np.maximum(lab, 0)], -1)
            rows = np.nonzero(col >= 0)[0]
            Agg = sp.csr_matrix((np.ones(len(rows)), (rows, col[rows])), shape=(n, k))
        om = None if omegas is None else omegas[len(levels)]
        P, om = smoothed_aggregation_jacobi(A, Agg, omega=om)
        P = P.tocsr()
        levels.append({"A": A, "P": P, "omega": om, "Dw": mlamg_dinv(A, jacobi_weight),
                       "Agg": Agg, "seeds": seeds, "labels": lab})
        A = galerkin(A, P)
    return levels, A


def make_cycle(levels, lu, nu_pre=1, nu_post=1):
    """cycle(l, b, x): one V-cycle at level l (x=None: zero guess), coarsest solved by lu."""

    def cycle(l, b, x):
        if l == len(levels):
            return lu(b)
        L = levels[l]
        A, P, Dw = L["A"], L["P"], L["Dw"]
        avw, pvw, rvw = L.get("A_vw", 0), L.get("P_vw", 0), L.get("R_vw", 0)
        if not (avw or pvw or rvw):
            if x is None:
                x = np.zeros(A.shape[0])
            x = jacobi_mlamg(A, Dw, b, x, nu_pre)
            xc = cycle(l + 1, P.T @ (b - A @ x), None)
            x += P @ xc
            x = jacobi_mlamg(A, Dw, b, x, nu_post)
            return x
        # device vector-order operators (coarse levels): same cycle, explicit R = P^T
        d = Dw.diagonal()
        R = L["R"]
        if x is None:
            x = np.zeros(A.shape[0])
        for _ in range(nu_pre):
            x = x + d * (b - mv(A, x, avw))
        xc = cycle(l + 1, mv(R, b - mv(A, x, avw), rvw), None)
        x = x + mv(P, xc, pvw)
        for _ in range(nu_post):
            x = x + d * (b - mv(A, x, avw))
        return x

    return cycle


def vcycle_solve(levels, Ac, b, x, n_cycles, tol=None, nu_pre=1, nu_post=1, lu=None):
    """Multilevel Jacobi V(nu_pre, nu_post) iteration in the device executor's order
    (mlamg hier.hip; each level = MLAMG.py:189-195 with the coarse solve recursing).
    Returns (x, residual history). lu: a pre-factorised coarse solve (spla.factorized)."""
    if lu is None:
        lu = spla.factorized(sp.csc_matrix(Ac))
    cycle = make_cycle(levels, lu, nu_pre, nu_post)
    x = x.copy()
    hist = []
    A0 = levels[0]["A"] if levels else Ac
    for _ in range(n_cycles):
        x = cycle(0, b, x) if levels else lu(b)
        r = la.norm(b - A0 @ x, 2)
        hist.append(r)
        if tol is not None and r <= tol:
            break
    return x, np.array(hist)


# ---------------------------------------------------------------- parallel CPU baseline
_OMP = None


def omp_lib(threads):
    """oracle/omp_cycle.c (OpenMP row-parallel kernels), `threads` OpenMP threads."""
    global _OMP
    if _OMP is None:
        path = _build.OUT_OMP if os.path.exists(_build.OUT_OMP) else _build.build_omp()
        L = ctypes.CDLL(path)
        vp, i64 = ctypes.c_void_p, ctypes.c_int64
        L.omp_set_threads.argtypes = [ctypes.c_int]
        for f in ("omp_resid", "omp_matvec", "omp_add_matvec"):
            getattr(L, f).argtypes = [i64, vp, vp, vp, vp, vp] + ([vp] if f == "omp_resid" else [])
        L.omp_jacobi.argtypes = [i64, vp, vp, vp, vp, vp, vp, vp]
        L.omp_scale.argtypes = [i64, vp, vp, vp]
        L.omp_gemv.argtypes = [i64, vp, vp, vp]
        L.omp_norm2.argtypes = [i64, vp]
        L.omp_norm2.restype = ctypes.c_double
        _OMP = L
    _OMP.omp_set_threads(int(threads))
    return _OMP


def vcycle_omp(levels, Ainv, b, x, n_cycles, threads):
    """BASELINE ONLY: the weighted-Jacobi V(1,1) cycle of the device executor (hier.hip: zero-guess
    first sweep on coarse levels, explicit R = P^T, dense-inverse coarse solve) with OpenMP
    row-parallel kernels on `threads` host threads. levels: dicts with CSR "A", "P" and the
    Jacobi weights "d" (ndarray); Ainv: the coarse inverse (dense ndarray). Returns (x, history)."""
    L = omp_lib(threads)
    P_ = _p
    lv = []
    for Lv in levels:
        A = Lv["A"].tocsr()
        R = Lv["P"].T.tocsr()
        R.sort_indices()
        P = Lv["P"].tocsr()
        n = A.shape[0]
        lv.append({"n": n, "A": _csr_arrays(A), "R": _csr_arrays(R), "P": _csr_arrays(P),
                   "nc": P.shape[1], "d": np.ascontiguousarray(Lv["d"], dtype=np.float64),
                   "x": np.zeros(n), "t": np.zeros(n), "r": np.zeros(n), "b": np.zeros(n)})
    nc = Ainv.shape[0]
    Ainv = np.ascontiguousarray(Ainv, dtype=np.float64)
    xc = np.zeros(nc)

    def csr(M):
        return P_(M[0]), P_(M[1]), P_(M[2])

    def cycle(l, bvec, x_in):
        if l == len(lv):
            L.omp_gemv(nc, P_(Ainv), P_(bvec), P_(xc))
            return xc
        v = lv[l]
        n = v["n"]
        cur = v["x"] if x_in is None else x_in
        if x_in is None:
            L.omp_scale(n, P_(v["d"]), P_(bvec), P_(cur))
        else:
            L.omp_jacobi(n, *csr(v["A"]), P_(v["d"]), P_(bvec), P_(cur), P_(v["t"]))
            cur[:] = v["t"]
        L.omp_resid(n, *csr(v["A"]), P_(bvec), P_(cur), P_(v["r"]))
        bn = lv[l + 1]["b"] if l + 1 < len(lv) else np.zeros(nc)
        L.omp_matvec(v["nc"], *csr(v["R"]), P_(v["r"]), P_(bn))
        e = cycle(l + 1, bn, None)
        L.omp_add_matvec(n, *csr(v["P"]), P_(e), P_(cur))
        L.omp_jacobi(n, *csr(v["A"]), P_(v["d"]), P_(bvec), P_(cur), P_(v["t"]))
        cur[:] = v["t"]
        return cur

    x = np.ascontiguousarray(x, dtype=np.float64).copy()
    b = np.ascontiguousarray(b, dtype=np.float64)
    hist = []
    r0 = np.zeros(x.shape[0])
    A0 = lv[0]["A"]
    for _ in range(n_cycles):
        cycle(0, b, x)
        L.omp_resid(x.shape[0], *csr(A0), P_(b), P_(x), P_(r0))
        hist.append(L.omp_norm2(x.shape[0], P_(r0)))
    return x, np.array(hist)


# --------------------------------------------------------------------------------------------
# Evolution strength of connection: pyamg.strength.evolution_strength_of_connection (pyamg 4.x/5.x,
# absent here: restated from its published algorithm; parity unpinned — no reference fixture
# pins it) at the reference's arguments (B=None -> ones, epsilon=4, k=2, proj_type 'l2',
# symmetrize_measure=True), as called by utils/common.py:27,30. The scipy steps are pyamg's own
# scipy calls; its three amg_core kernels are restated below.

def _pyamg_norm(x):
    """pyamg.util.linalg.norm: sqrt(inner(conj(x), x).real) of the raveled vector."""
    x = np.ravel(x)
    return np.sqrt(np.inner(x.conj(), x).real)


def approximate_spectral_radius(A, tol=0.01, maxiter=15, restart=5):
    """pyamg.util.linalg.approximate_spectral_radius(A) with its _approximate_eigenvalues
    (pyamg 4.x/5.x; symmetric=False is forced there): v0 = np.random.rand(n, 1) from the GLOBAL
    generator (n draws), Arnoldi with modified Gram-Schmidt (H[i, j] = dot(conj(v_i), w),
    breakdown below eps*1e6), scipy.linalg.eig of H[:m, :m], restart from the dominant Ritz
    vector (complex if eig returned complex vectors — pyamg keeps it complex) until
    |H[m, m-1] y_m| / |ev| < tol. A@v is scipy's csr_matvec. Returns |ev_max| (float)."""
    import scipy.linalg
    n = A.shape[0]
    v0 = np.random.rand(n, 1)
    maxiter = min(n, maxiter)
    breakdown = np.finfo(np.float64).eps * 1e6
    ev = None
    max_index = 0
    for _ in range(restart + 1):
        v0 = v0 / _pyamg_norm(v0)
        H = np.zeros((maxiter + 1, maxiter), dtype=np.result_type(v0.dtype, A.dtype))
        V = [v0]
        flag = False
        j = 0
        for j in range(maxiter):
            w = A @ V[-1]
            for i, vi in enumerate(V):
                H[i, j] = np.dot(np.conjugate(vi.ravel()), w.ravel())
                w = w - H[i, j] * vi
            H[j + 1, j] = _pyamg_norm(w)
            if H[j + 1, j] < breakdown:
                flag = True
                if H[j + 1, j] != 0:
                    w = w / H[j + 1, j]
                V.append(w)
                break
            w = w / H[j + 1, j]
            V.append(w)
        ev, evect = scipy.linalg.eig(H[:j + 1, :j + 1], left=False, right=True)
        nvecs = ev.shape[0]
        max_index = np.abs(ev).argmax()
        err = H[nvecs, nvecs - 1] * evect[-1, max_index]
        v0 = np.dot(np.hstack(V[:-1]), evect[:, max_index].reshape(-1, 1))
        if np.abs(err) / np.abs(ev[max_index]) < tol or flag:
            break
    return float(np.abs(ev[max_index]))


def _incomplete_mat_mult(T, mask):
    """amg_core incomplete_mat_mult_csr(T, T.tocsc(), mask): S_ij = sum_k T_ik T_kj on mask's
    pattern, ascending k — the order in which csr_matmat accumulates the same products, so the
    product restricted to the mask (x * 1.0, zeros dropped = eliminate_zeros) is bitwise it."""
    ones = mask.copy()
    ones.data[:] = 1.0
    S = (T @ T).multiply(ones).tocsr()
    S.sort_indices()
    return S


def _row_reduce(M, fn, init):
    out = np.full(M.shape[0], init)
    nz = np.diff(M.indptr) > 0
    if M.nnz:
        red = fn.reduceat(M.data, M.indptr[:-1][nz])
        out[nz] = red
    return out


def evolution_strength(A, rho=None, epsilon=4.0):
    """pyamg evolution_strength_of_connection(A) (reference defaults). rho: rho(D^-1 A)
    (None: approximate_spectral_radius, pyamg's estimate)."""
    A = sp.csr_matrix(A, dtype=np.float64, copy=True)
    D = A.diagonal()
    Dinv = np.zeros_like(D)
    mask = D != 0.0
    Dinv[mask] = 1.0 / D[mask]
    Dinv[D == 0] = 1.0
    Dinv_A = A.copy()
    Dinv_A.data = Dinv_A.data * np.repeat(Dinv, np.diff(Dinv_A.indptr))  # csr_scale_rows
    A.eliminate_zeros()
    A.sort_indices()
    n = A.shape[0]
    if rho is None:
        rho = approximate_spectral_radius(Dinv_A)
    Id = sp.eye(n, n, format="csr", dtype=A.dtype)
    Atilde = (Id - (1.0 / rho) * Dinv_A)
    Atilde = Atilde.T.tocsr()
    Atilde.sort_indices()
    S = _incomplete_mat_mult(Atilde, A)           # k = 2: one incomplete product
    S.eliminate_zeros()
    # B = ones shortcut
    DA = S.diagonal()
    rows = np.repeat(np.arange(n), np.diff(S.indptr))
    data = S.data.copy()
    zt = DA[rows] * 1.0                           # scale_rows(ones, DA / 1) then columns by 1
    angle = (zt * data + 0.0 * 0.0) < 0.0
    ratio = zt / data
    weak = np.abs(ratio) < 1e-4
    v = np.abs(1.0 - ratio)
    v[weak] = 0.0
    v[angle] = 0.0
    S.data = v
    S.eliminate_zeros()
    S.data[S.data < np.sqrt(np.finfo(float).eps)] = 1e-4
    # amg_core apply_distance_filter
    rows = np.repeat(np.arange(n), np.diff(S.indptr))
    off = S.indices != rows
    offv = np.where(off, S.data, np.finfo(float).max)
    Sm = S.copy()
    Sm.data = offv
    mn = _row_reduce(Sm, np.minimum, np.finfo(float).max)
    thr = epsilon * mn
    newv = S.data.copy()
    newv[~off] = 1.0
    newv[off & (S.data >= thr[rows])] = 0.0
    S.data = newv
    S.eliminate_zeros()
    # symmetrize, unit diagonal, invert, scale rows by the largest entry
    S = 0.5 * (S + S.T)
    Id = sp.eye(n, n, format="csr")
    Id.data -= S.diagonal()
    S = S + Id
    S.data = 1.0 / S.data
    mx = _row_reduce(abs(S).tocsr(), np.maximum, 0.0)   # amg_core maximum_row_value
    mx[mx != 0] = 1.0 / mx[mx != 0]
    S = sp.csr_matrix(S)
    S.data = S.data * np.repeat(mx, np.diff(S.indptr))  # scale_rows
    return S


def strength_measure(A, name, rho=None):
    """utils/common.py:25-31 strength_measure_funcs[name](A)."""
    if name == "abs":
        return abs(A)
    if name == "invabs":
        return sp.csr_matrix((1.0 / np.abs(A.data), A.indices, A.indptr), A.shape)
    if name == "unit":
        return sp.csr_matrix((np.ones_like(A.data), A.indices, A.indptr), A.shape)
    ev = evolution_strength(A, rho=rho)
    if name == "evolution":
        return ev + sp.csr_matrix((np.ones_like(A.data), A.indices, A.indptr), A.shape) * 0.1
    if name == "olson":
        return ev + sp.csr_matrix((1. / np.abs(A.data), A.indices, A.indptr), A.shape)
    raise KeyError(name)


# --------------------------------------------------------------------------------------------
# pyamg.aggregation.smoothed_aggregation_solver with its defaults (pyamg 4.x/5.x, absent here:
# restated from its published algorithm; parity unpinned), the multilevel solver the reference's
# PyAMG preconditioner builds (ns/preconditioner/PyAMG.py:94) and applies (:119). The amg_core
# loops are in oracle/oracle.c; the scipy steps are pyamg's own scipy calls.

_SWEEPS = {"forward": 0, "backward": 1, "symmetric": 2}


def pyamg_symmetric_strength(A, theta=0.0):
    """pyamg.strength.symmetric_strength_of_connection(A, theta) on a CSR matrix."""
    ip, ij, ax = _csr_arrays(A)
    n = A.shape[0]
    sp_ = np.empty(n + 1, dtype=np.int32)
    sj = np.empty(max(len(ij), 1), dtype=np.int32)
    sx = np.empty(max(len(ij), 1), dtype=np.float64)
    nnz = lib().pyamg_symmetric_strength(n, _p(ip), _p(ij), _p(ax), float(theta), _p(sp_),
                                         _p(sj), _p(sx))
    return sp.csr_matrix((sx[:nnz], sj[:nnz], sp_), shape=A.shape)


def pyamg_standard_aggregation(C):
    """pyamg.aggregation.standard_aggregation(C): (per-row aggregate, -1 none; Cpts; count)."""
    ip, ij, _ = _csr_arrays(C)
    n = C.shape[0]
    x = np.empty(max(n, 1), dtype=np.int32)
    y = np.empty(max(n, 1), dtype=np.int32)
    k = lib().pyamg_standard_aggregation(n, _p(ip), _p(ij), _p(x), _p(y))
    return x[:n], y[:k].copy(), int(k)


def pyamg_aggop(agg, k):
    """AggOp as standard_aggregation returns it (rows with agg == -1 empty)."""
    agg = np.asarray(agg)
    rows = np.nonzero(agg >= 0)[0]
    return sp.csr_matrix((np.ones(len(rows)), (rows, agg[rows])), shape=(len(agg), k))


def pyamg_block_gauss_seidel(A, x, b, iterations=1, sweep="forward"):
    """pyamg.relaxation.relaxation.block_gauss_seidel(A, x, b, iterations, sweep) with 1 x 1
    blocks, in place on x (float64, contiguous)."""
    ip, ij, ax = _csr_arrays(A)
    assert x.dtype == np.float64 and x.flags.c_contiguous
    b = np.ascontiguousarray(b, dtype=np.float64)
    lib().pyamg_block_gauss_seidel(A.shape[0], _p(ip), _p(ij), _p(ax), _p(x), _p(b),
                                   int(iterations), _SWEEPS[sweep])
    return x


def pyamg_fit_candidates(agg, k, B, tol=1e-10):
    """pyamg.aggregation.fit_candidates(AggOp, B[:, None], tol): (T as CSR, B_c)."""
    agg = np.ascontiguousarray(agg, dtype=np.int32)
    B = np.ascontiguousarray(B, dtype=np.float64).reshape(-1)
    n = agg.shape[0]
    rows = np.nonzero(agg >= 0)[0]
    tx = np.empty(max(len(rows), 1))
    Bc = np.empty(max(k, 1))
    lib().pyamg_fit_candidates(n, _p(agg), int(k), _p(B), float(tol), _p(tx), _p(Bc))
    T = sp.csr_matrix((tx[:len(rows)], (rows, agg[rows])), shape=(n, k))
    return T, Bc[:k].copy()


def pyamg_dinv(A):
    """pyamg.util.utils.get_diagonal(A, inv=True): 1 / diag, 0 where diag == 0."""
    D = A.diagonal()
    Dinv = np.zeros_like(D, dtype=np.float64)
    mask = D != 0.0
    Dinv[mask] = 1.0 / D[mask]
    return Dinv


def pyamg_jacobi_prolongation(A, T, rho, omega=4.0 / 3.0):
    """pyamg jacobi_prolongation_smoother(A, T, C, B, omega, degree=1, filter=False,
    weighting='diagonal') with the spectral radius given: D_inv_S = scale_rows(A, D_inv)
    (csr_scale_rows: a_ij * d_i, pattern and order kept), times (omega / rho) (data * c),
    P = T - D_inv_S @ T (scipy csr_matmat, then the csr binop; zeros dropped). Columns sorted."""
    A = sp.csr_matrix(A)
    d = pyamg_dinv(A)
    row = np.repeat(np.arange(A.shape[0]), np.diff(A.indptr))
    S = sp.csr_matrix((A.data * d[row], A.indices.copy(), A.indptr.copy()), shape=A.shape)
    c = omega / rho
    S = sp.csr_matrix((S.data * c, S.indices, S.indptr), shape=A.shape)
    P = sp.csr_matrix(T - S @ T)
    P.sort_indices()
    return P


def pyamg_sa_setup(A, rhos=None, max_levels=10, max_coarse=10, theta=0.0, omega=4.0 / 3.0,
                   improve_iterations=4, B=None):
    """The levels of smoothed_aggregation_solver(A, max_levels=...): a list of dicts (A, C,
    agg, k, B, T, P, R, rho) and the coarsest operator. rhos: per-level rho(D^-1 A) (default:
    scipy eigs of D^-1 A, largest magnitude). A_c = (P^T A) P in scipy."""
    A = canonical(sp.csr_matrix(A, dtype=np.float64))
    Bv = np.ones(A.shape[0]) if B is None else np.asarray(B, dtype=np.float64).reshape(-1).copy()
    levels = []
    while A.shape[0] > max_coarse and len(levels) + 1 < max_levels:
        lvl = len(levels)
        C = pyamg_symmetric_strength(A, theta)
        agg, cpts, k = pyamg_standard_aggregation(C)
        if lvl == 0 and improve_iterations > 0:
            pyamg_block_gauss_seidel(A, Bv, np.zeros(A.shape[0]), improve_iterations,
                                     "symmetric")
        T, Bc = pyamg_fit_candidates(agg, k, Bv)
        if rhos is None:
            Dinv_A = sp.diags(pyamg_dinv(A)) @ A
            rho = float(np.abs(spla.eigs(Dinv_A, k=1, which="LM",
                                         return_eigenvectors=False)[0]))
        else:
            rho = float(rhos[lvl])
        P = pyamg_jacobi_prolongation(A, T, rho, omega)
        R = sp.csr_matrix(P.T)
        R.sort_indices()
        levels.append({"A": A, "C": C, "agg": agg, "cpts": cpts, "k": k, "B": Bv.copy(),
                       "T": T, "P": P, "R": R, "rho": rho})
        A = canonical((P.T @ A) @ P)
        Bv = Bc
    return levels, A


def pyamg_sa_vcycle(levels, Ac_pinv, b, x, lvl=0):
    """pyamg MultilevelSolver.__solve(lvl, x, b, 'V') with block Gauss-Seidel symmetric pre/post
    smoothing and the 'pinv' coarse solve (np.dot(pinv, b)); x updated in place."""
    if not levels:
        x[:] = Ac_pinv @ b
        return x
    L = levels[lvl]
    A = L["A"]
    pyamg_block_gauss_seidel(A, x, b, 1, "symmetric")
    r = b - A @ x
    bc = L["R"] @ r
    xc = np.zeros_like(bc)
    if lvl == len(levels) - 1:
        xc[:] = Ac_pinv @ bc
    else:
        pyamg_sa_vcycle(levels, Ac_pinv, bc, xc, lvl + 1)
    x += L["P"] @ xc
    pyamg_block_gauss_seidel(A, x, b, 1, "symmetric")
    return x


def _mysign(v):
    return 1.0 if v == 0.0 else (1.0 if v > 0.0 else -1.0)


def pyamg_gmres_householder(A, b, M, x0=None, tol=1e-5, maxiter=None):
    """pyamg.krylov.gmres(A, b, x0, tol, restrt=None, maxiter, M) with orthog='householder'
    (pyamg 4.x _gmres_householder, restated; pyamg absent: parity unpinned). M: callable, the
    preconditioner. Returns (x, info, niter, residuals)."""
    A = sp.csr_matrix(A)
    n = A.shape[0]
    b = np.asarray(b, dtype=np.float64)
    x = np.zeros(n) if x0 is None else np.array(x0, dtype=np.float64)
    if maxiter is None:
        maxiter = min(n, 40)
    max_inner = min(maxiter, n)
    r = M(b - A @ x)
    normr = np.linalg.norm(r)
    res = [normr]
    normb = np.linalg.norm(b)
    if normb == 0.0:
        normb = 1.0
    if normr < tol * normb:
        return x, 0, 0, res
    if normr != 0.0:
        tol = tol * normr
    W = np.zeros((max_inner + 1, n))
    w = r.copy()
    w[0] = w[0] + _mysign(w[0]) * normr
    W[0] = w / np.linalg.norm(w)
    g = np.zeros(max_inner + 1)
    g[0] = -_mysign(r[0]) * normr
    H = np.zeros((max_inner, max_inner))
    Q = []
    niter = 0
    inner = 0
    for inner in range(max_inner):
        v = -2.0 * W[inner, inner] * W[inner]
        v[inner] = v[inner] + 1.0
        for j in range(inner - 1, -1, -1):
            v = v + (-2.0 * np.dot(W[j], v)) * W[j]
        v = M(A @ v)
        for j in range(inner + 1):
            v = v + (-2.0 * np.dot(W[j], v)) * W[j]
        if inner != n - 1:
            alpha = np.linalg.norm(v[inner + 1:])
            if alpha != 0.0:
                alpha = _mysign(v[inner + 1]) * alpha
                if inner < max_inner - 1:
                    w = np.zeros(n)
                    w[inner + 1:] = v[inner + 1:]
                    w[inner + 1] = w[inner + 1] + alpha
                    W[inner + 1] = w / np.linalg.norm(w)
                v[inner + 1] = -alpha
                v[inner + 2:] = 0.0
        for j, (c, s) in enumerate(Q):
            a0, a1 = v[j], v[j + 1]
            v[j] = c * a0 + s * a1
            v[j + 1] = -s * a0 + c * a1
        if inner != n - 1 and v[inner + 1] != 0.0:
            f, gg = v[inner], v[inner + 1]
            d = np.sqrt(f * f + gg * gg)
            c = abs(f) / d if f != 0.0 else 0.0
            rr = (d if f > 0 else -d) if f != 0.0 else abs(gg)
            s = gg / rr if f != 0.0 else (1.0 if gg > 0 else -1.0)
            Q.append((c, s))
            g0, g1 = g[inner], g[inner + 1]
            g[inner] = c * g0 + s * g1
            g[inner + 1] = -s * g0 + c * g1
            v[inner] = c * v[inner] + s * v[inner + 1]
            v[inner + 1] = 0.0
        else:
            Q.append((1.0, 0.0))
        H[:inner + 1, inner] = v[:inner + 1]
        niter += 1
        if inner < max_inner - 1:
            normr = abs(g[inner + 1])
            if normr < tol:  # pyamg _gmres_householder: break, then callback / residuals
                break
            res.append(normr)
    y = np.linalg.solve(np.triu(H[:inner + 1, :inner + 1]), g[:inner + 1])
    update = np.zeros(n)
    for j in range(inner, -1, -1):
        update[j] = update[j] + y[j]
        update = update + (-2.0 * np.dot(W[j], update)) * W[j]
    x = x + update
    normr = np.linalg.norm(M(b - A @ x))
    res.append(normr)
    return x, (0 if normr < tol else niter), niter, res
