"""Synthetic test matrices of the benchmark configurations.

  poisson_1d        C1: tridiag(-1, 2, -1), unscaled (demos/1d_poisson.py:35)
  poisson_2d_5pt    C2: [4, -1 x4] on an nx x ny interior grid — the stencil P1 elements give on
                    pyamg's regular_triangle_mesh (ns/model/data.py:435-497)
  poisson_3d_7pt    C4: [6, -1 x6] on n^3 (the 7-point analogue of utils/create_3d_laplace.py)
  jump_2d           C5: 2D 5-point diffusion with Voronoi jump coefficients (utils/create_data.py
                    :69-78, demos/voronoi_jump_disc.py:10-22), harmonic-mean face coefficients
  box_aggregates_*  fixed aggregates (demos/1d_poisson.py:52-55 pattern)

All CSRs are canonical (sorted columns) with int32 indices and fp64 values; they are built
directly from index arithmetic so the 10M-row C4 matrix takes a few seconds.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp


def _csr_from_stencil(n_rows, cols_list, vals_list):
    """Rows = natural order; cols_list/vals_list: per-offset arrays with -1 where absent."""
    cols = np.stack(cols_list, axis=1)  # (n, k), ascending offsets
    vals = np.stack(vals_list, axis=1)
    mask = cols >= 0
    counts = mask.sum(axis=1)
    indptr = np.zeros(n_rows + 1, dtype=np.int64)
    np.cumsum(counts, out=indptr[1:])
    indices = cols[mask].astype(np.int32)
    data = vals[mask].astype(np.float64)
    return sp.csr_matrix((data, indices, indptr.astype(np.int32)), shape=(n_rows, n_rows))


def poisson_1d(n):
    A = sp.eye(n) * 2 - sp.eye(n, k=-1) - sp.eye(n, k=1)
    A = A.tocsr()
    A.sort_indices()
    A.indices = A.indices.astype(np.int32)
    A.indptr = A.indptr.astype(np.int32)
    return A


def poisson_2d_5pt(nx, ny=None):
    ny = nx if ny is None else ny
    n = nx * ny
    idx = np.arange(n, dtype=np.int64)
    x = idx % nx
    y = idx // nx
    offs = [
        (np.where(y > 0, idx - nx, -1), -1.0),
        (np.where(x > 0, idx - 1, -1), -1.0),
        (idx, 4.0),
        (np.where(x < nx - 1, idx + 1, -1), -1.0),
        (np.where(y < ny - 1, idx + nx, -1), -1.0),
    ]
    return _csr_from_stencil(n, [c for c, _ in offs], [np.full(n, v) for _, v in offs])


def poisson_3d_7pt(nx, ny=None, nz=None):
    ny = nx if ny is None else ny
    nz = nx if nz is None else nz
    n = nx * ny * nz
    idx = np.arange(n, dtype=np.int64)
    x = idx % nx
    y = (idx // nx) % ny
    z = idx // (nx * ny)
    pl = nx * ny
    cols, vals = [], []
    for c, v in (
        (np.where(z > 0, idx - pl, -1), -1.0),
        (np.where(y > 0, idx - nx, -1), -1.0),
        (np.where(x > 0, idx - 1, -1), -1.0),
        (idx, 6.0),
        (np.where(x < nx - 1, idx + 1, -1), -1.0),
        (np.where(y < ny - 1, idx + nx, -1), -1.0),
        (np.where(z < nz - 1, idx + pl, -1), -1.0),
    ):
        cols.append(c)
        vals.append(np.full(n, v))
        del c
    return _csr_from_stencil(n, cols, vals)


def random_coeff_3d_7pt(nx, seed=0, decades=1.0):
    """7-point finite-volume diffusion -div(k grad u) on an nx^3 interior grid (Dirichlet), with
    an independent coefficient k = 10^U(-decades, decades) on every cell face (RandomState(seed)),
    boundary faces included: a symmetric M-matrix with the C4 sparsity (nnz 70,263,936 at 216^3)
    whose values are all distinct, so no stencil re-encoding (row-pair patterns, dictionary
    SELL) applies — the generic-operator counterpart of the C4 headline."""
    n = nx ** 3
    rs = np.random.RandomState(seed)
    # face coefficients: kx[i] couples cell i with its +x neighbour (or the boundary)
    kx = 10.0 ** rs.uniform(-decades, decades, n)
    ky = 10.0 ** rs.uniform(-decades, decades, n)
    kz = 10.0 ** rs.uniform(-decades, decades, n)
    # the -x / -y / -z faces of the first cells of each line are boundary faces of their own
    kx0 = 10.0 ** rs.uniform(-decades, decades, n)
    ky0 = 10.0 ** rs.uniform(-decades, decades, n)
    kz0 = 10.0 ** rs.uniform(-decades, decades, n)
    idx = np.arange(n, dtype=np.int64)
    x = idx % nx
    y = (idx // nx) % nx
    z = idx // (nx * nx)
    pl = nx * nx
    kxm = np.where(x > 0, kx[np.maximum(idx - 1, 0)], kx0)
    kym = np.where(y > 0, ky[np.maximum(idx - nx, 0)], ky0)
    kzm = np.where(z > 0, kz[np.maximum(idx - pl, 0)], kz0)
    diag = kxm + kx + kym + ky + kzm + kz
    cols = [np.where(z > 0, idx - pl, -1), np.where(y > 0, idx - nx, -1),
            np.where(x > 0, idx - 1, -1), idx, np.where(x < nx - 1, idx + 1, -1),
            np.where(y < nx - 1, idx + nx, -1), np.where(z < nx - 1, idx + pl, -1)]
    vals = [-kzm, -kym, -kxm, diag, -kx, -ky, -kz]
    return _csr_from_stencil(n, cols, vals)


def voronoi_jumps(rand, ns=None):
    """Jump seeds [x, y, d] like utils/create_data.py:69-78 (d = 10^U(-4,4), ptp > 1e3)."""
    ns = rand.randint(2, 4) if ns is None else ns
    while True:
        pts = rand.rand(ns, 2)
        d = 10.0 ** rand.uniform(-4, 4, ns)
        if np.ptp(d) > 1e3:
            return np.column_stack([pts, d])


def jump_2d(nx, jumps):
    """5-point finite-volume diffusion -div(k grad u) on the unit square interior grid, with k
    piecewise constant on the Voronoi cells of jumps[:, :2] (value jumps[:, 2]); face
    coefficients are harmonic means of the two cell values (documented deviation from the
    reference's P1 quadrature)."""
    n = nx * nx
    h = 1.0 / (nx + 1)
    g = (np.arange(nx) + 1) * h
    X, Y = np.meshgrid(g, g)
    P = np.column_stack([X.ravel(), Y.ravel()])
    dist = ((P[:, None, :] - jumps[None, :, :2]) ** 2).sum(-1)
    kap = jumps[np.argmin(dist, axis=1), 2]
    idx = np.arange(n, dtype=np.int64)
    x = idx % nx
    y = idx // nx

    def hm(a, b):
        return 2.0 * a * b / (a + b)

    kc = kap
    kxm = np.where(x > 0, hm(kc, kap[np.maximum(idx - 1, 0)]), kc)
    kxp = np.where(x < nx - 1, hm(kc, kap[np.minimum(idx + 1, n - 1)]), kc)
    kym = np.where(y > 0, hm(kc, kap[np.maximum(idx - nx, 0)]), kc)
    kyp = np.where(y < nx - 1, hm(kc, kap[np.minimum(idx + nx, n - 1)]), kc)
    diag = kxm + kxp + kym + kyp
    cols = [np.where(y > 0, idx - nx, -1), np.where(x > 0, idx - 1, -1), idx,
            np.where(x < nx - 1, idx + 1, -1), np.where(y < nx - 1, idx + nx, -1)]
    vals = [-kym, -kxm, diag, -kxp, -kyp]
    return _csr_from_stencil(n, cols, vals)


def box_aggregates_1d(n, size=3):
    """Agg[i, i // size] = 1 (demos/1d_poisson.py:52-55; last aggregate may be short)."""
    k = (n + size - 1) // size
    return sp.csr_matrix((np.ones(n), np.arange(n) // size, np.arange(n + 1)), shape=(n, k))


def box_aggregates_2d(nx, ny=None, size=3):
    ny = nx if ny is None else ny
    n = nx * ny
    idx = np.arange(n)
    x, y = idx % nx, idx // nx
    kx = (nx + size - 1) // size
    ky = (ny + size - 1) // size
    col = (y // size) * kx + (x // size)
    return sp.csr_matrix((np.ones(n), col, np.arange(n + 1)), shape=(n, kx * ky))


def strength_invabs(A):
    """utils/common.py:28."""
    return sp.csr_matrix((1.0 / np.abs(A.data), A.indices, A.indptr), A.shape)


def strength_abs(A):
    """utils/common.py:26."""
    return abs(A)


def strength_unit(A):
    """utils/common.py:29."""
    return sp.csr_matrix((np.ones_like(A.data), A.indices, A.indptr), A.shape)
