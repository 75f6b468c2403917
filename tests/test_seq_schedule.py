"""CPU: the decomposition the device uses to run the reference's sequential sweeps in parallel
(csrc/graph.hip, "sequential sweeps (exact)") — restated here in numpy at the device's
granularity (a level's rows in any order, phases separated) — reproduces the reference's own
sweep (the oracle's transcription, itself bitwise the reference's outputs in
test_oracle_golden.py) bit for bit, ties and sweep count included:

* push (ns/lib/graph.py:40-51): mid_j = the previous value folded with the pushes of in-edges
  from rows k < j (level-scheduled), end_j = mid_j folded with the rows k > j, both in
  ascending k and from the mid values;
* pull (pyamg amg_core bellman_ford): rows by level, level(i) = 1 + max level(j) over j < i
  coupled either way.

The level order is shuffled inside every level to show that no intra-level order matters."""
import numpy as np
import pytest
import scipy.sparse as sp

from conftest import golden_csr


def _levels_push(C):
    n = C.shape[0]
    level = np.zeros(n, dtype=np.int64)
    for k in range(n):
        for q in range(C.indptr[k], C.indptr[k + 1]):
            j = C.indices[q]
            if j > k:
                level[j] = max(level[j], level[k] + 1)
    return level


def _order(level, rs):
    order = []
    for l in range(level.max() + 1):
        rows = np.nonzero(level == l)[0]
        order.extend(rs.permutation(rows))
    return order


def push_two_phase(C, seeds, rs):
    n = C.shape[0]
    w32 = C.data.astype(np.float32)
    T = sp.csr_matrix((w32, C.indices, C.indptr), shape=C.shape).T.tocsr()
    T.sort_indices()  # in-edges of j with sources ascending
    tip, tsrc, tw = T.indptr, T.indices, T.data.astype(np.float32)
    order = _order(_levels_push(C), rs)
    d = np.full(n, np.inf, dtype=np.float32)
    z = np.full(n, -1, dtype=np.int64)
    d[seeds] = 0
    z[seeds] = seeds
    dm, zm = d.copy(), z.copy()
    sweeps = 0
    while True:
        sweeps += 1
        for j in order:
            cur, lab = d[j], z[j]
            for e in range(tip[j], tip[j + 1]):
                k = tsrc[e]
                if k >= j:
                    break
                cand = np.float32(dm[k] + tw[e])
                if cand < cur:
                    cur, lab = cand, zm[k]
            dm[j], zm[j] = cur, lab
        changed = False
        for j in rs.permutation(n):
            cur, lab = dm[j], zm[j]
            for e in range(tip[j], tip[j + 1]):
                k = tsrc[e]
                if k <= j:
                    continue
                cand = np.float32(dm[k] + tw[e])
                if cand < cur:
                    cur, lab = cand, zm[k]
            changed |= bool(cur < d[j])
            d[j], z[j] = cur, lab
        if not changed:
            return d, np.where(z < 0, 0, z), sweeps


@pytest.mark.parametrize("k", ("p2d", "lap3d", "rnd"))
@pytest.mark.parametrize("weights", ("invabs", "unit"))
def test_push_two_phase_is_the_reference_sweep(golden, oracle, k, weights):
    A = golden_csr(golden, k)
    vals = 1.0 / np.abs(A.data) if weights == "invabs" else np.ones_like(A.data)
    C = oracle.canonical(sp.csr_matrix((vals, A.indices, A.indptr), A.shape))
    seeds = golden[f"{k}_bf_seeds"]
    d, z, sw = push_two_phase(C, seeds, np.random.RandomState(1))
    dr, zr, swr = oracle.modified_bellman_ford(C, seeds)
    assert np.array_equal(d, dr) and np.array_equal(z, zr) and sw == swr
    if weights == "invabs":
        assert np.array_equal(z, golden[f"{k}_bf_nearest"])


def pull_levels(C, x, z, rs):
    n = C.shape[0]
    ip, ij, w = C.indptr, C.indices, C.data
    level = np.zeros(n, dtype=np.int64)
    req = np.zeros(n, dtype=np.int64)
    for i in range(n):
        L = req[i]
        for q in range(ip[i], ip[i + 1]):
            if ij[q] < i:
                L = max(L, level[ij[q]] + 1)
        level[i] = L
        for q in range(ip[i], ip[i + 1]):
            if ij[q] > i:
                req[ij[q]] = max(req[ij[q]], L + 1)
    order = _order(level, rs)
    sweeps = 0
    while True:
        sweeps += 1
        changed = False
        for i in order:
            xi, zi = x[i], z[i]
            for q in range(ip[i], ip[i + 1]):
                d = w[q] + x[ij[q]]
                if d < xi:
                    xi, zi = d, z[ij[q]]
            changed |= bool(xi != x[i])
            x[i], z[i] = xi, zi
        if not changed:
            return x, z, sweeps


@pytest.mark.parametrize("k", ("p2d", "lap3d"))
def test_pull_levels_is_pyamgs_sweep(golden, oracle, k):
    A = golden_csr(golden, k)
    G = sp.csr_matrix((np.abs(A.data), A.indices, A.indptr), A.shape)
    seeds = golden[f"{k}_bf_seeds"].astype(np.int32)
    dr, zr, swr = oracle.pyamg_bellman_ford(G, seeds, dtype=np.float64)
    x = np.full(G.shape[0], np.finfo(np.float64).max)
    z = np.full(G.shape[0], -1, dtype=np.int32)
    x[seeds], z[seeds] = 0.0, seeds
    x, z, sw = pull_levels(G, x, z, np.random.RandomState(2))
    assert np.array_equal(x, dr) and np.array_equal(z, zr) and sw == swr
