"""Drop-in mirror of ns/lib/graph.py (aggregation) running on the MI355X.

  modified_bellman_ford   ns/lib/graph.py:7-53     seeded Bellman-Ford, fp32 (torch) arithmetic
  bellman_ford            pyamg 4.x graph.bellman_ford (ns/model/agg_interp.py:475, the
                          aggregation step of FullAggNet.forward)
  nearest_center_to_agg   ns/lib/graph.py:56-86    aggregate matrix from assignments
  lloyd_aggregation       ns/lib/graph.py:156-239  seeds + pyamg 4.x lloyd_cluster + AggOp
  lloyd_cluster           pyamg 4.x graph.lloyd_cluster (what graph.py:232 calls)
  num_connected_components, check_aggregates_connected   ns/lib/graph.py:89-153 (host-side
                          graph checks, kept so an alias of ns.lib.graph to this module is whole)

All three reference sweeps are sequential and in place, so on equal-length paths the winning
seed depends on the sweep order. The device runs those orders themselves, level-scheduled
(csrc/graph.hip): distances and labels are bitwise the reference's on every input, ties
included. The order-independent variants (bellman_ford_device, lloyd_cluster_device(...,
exact=False): label = smallest seed among tight predecessors, multi-workgroup sweeps) serve the
multilevel / distributed hierarchy, which has no reference counterpart.
"""
from __future__ import annotations

import ctypes

import numpy as np
import scipy.sparse as sp
import torch

from ._lib import call, ptr, stream_ptr
from .sparse import DeviceCSR, _device


def _coo_to_device_csr(S_T):
    """torch COO (coalesced, row-major) -> DeviceCSR with the fp32 values widened exactly."""
    S_T = S_T.coalesce()
    n, m = S_T.shape
    idx = S_T.indices().cpu().numpy()
    vals = S_T.values().detach().cpu().numpy().astype(np.float64)
    A = sp.csr_matrix((vals, (idx[0], idx[1])), shape=(n, m))
    # coalesced COO is sorted by (row, col); csr_matrix keeps that order
    return DeviceCSR.from_scipy(A, check=False)


def bellman_ford_device(G, seeds_dev):
    """Order-independent device Bellman-Ford on G (push form: edge i -> j, weight G[i, j]) —
    the hierarchy's aggregation. Labels: smallest seed id among tight predecessors.

    Returns (distance fp32 tensor, label int32 tensor (seed node id, -1 unreachable), sweeps).
    """
    n = G.shape[0]
    dev = _device()
    dist = torch.empty(n, dtype=torch.float32, device=dev)
    lab = torch.empty(n, dtype=torch.int32, device=dev)
    sweeps = ctypes.c_int32()
    call("mlamg_bellman_ford_canon", G.handle, ptr(seeds_dev), int(seeds_dev.numel()), ptr(dist),
         ptr(lab), ctypes.byref(sweeps), stream_ptr())
    return dist, lab, int(sweeps.value)


def modified_bellman_ford_device(G, seeds_dev):
    """ns/lib/graph.py:40-51 exactly on a DeviceCSR: the reference's row-major in-place push
    sweeps in fp32, level-scheduled. Returns (distance fp32 tensor, nearest int32 tensor (seed
    node id, -1 unreachable), sweeps = the reference's count)."""
    n = G.shape[0]
    dev = _device()
    dist = torch.empty(n, dtype=torch.float32, device=dev)
    lab = torch.empty(n, dtype=torch.int32, device=dev)
    sweeps = ctypes.c_int32()
    call("mlamg_bellman_ford", G.handle, ptr(seeds_dev), int(seeds_dev.numel()), ptr(dist),
         ptr(lab), ctypes.byref(sweeps), stream_ptr())
    return dist, lab, int(sweeps.value)


def bellman_ford_pyamg_device(G, seeds_dev, fp64=False):
    """pyamg 4.x graph.bellman_ford on a DeviceCSR (pull form: x_i <- min(x_i, G[i, j] + x_j)).

    Returns (distances float32/float64 tensor (unreached: the dtype's max), nearest seed int32
    tensor (seed node id, -1 unreached), sweeps)."""
    n = G.shape[0]
    dev = _device()
    dist = torch.empty(n, dtype=torch.float64 if fp64 else torch.float32, device=dev)
    near = torch.empty(n, dtype=torch.int32, device=dev)
    sweeps = ctypes.c_int32()
    call("mlamg_bellman_ford_pyamg", G.handle, ptr(seeds_dev), int(seeds_dev.numel()),
         1 if fp64 else 0, ptr(dist), ptr(near), ctypes.byref(sweeps), stream_ptr())
    return dist, near, int(sweeps.value)


def bellman_ford(G, seeds, maxiter=None):
    """Drop-in for pyamg.graph.bellman_ford (pyamg 4.x, as ns/model/agg_interp.py:475 calls it).

    G: scipy sparse graph (asgraph: anything but CSR/CSC becomes csr_matrix, duplicates summed;
    a CSC graph's arrays are walked as CSR, like amg_core does), float32 or float64 weights;
    seeds: node ids. Returns numpy (distances in G's dtype, nearest_seed intc). maxiter only
    validated: pyamg 4.x never advances its counter, so it sweeps to the fixed point anyway."""
    if maxiter is not None and maxiter < 0:
        raise ValueError('maxiter must be positive')
    if not (sp.isspmatrix_csr(G) or sp.isspmatrix_csc(G)):
        G = sp.csr_matrix(G)
    if G.dtype == complex:
        raise ValueError('Bellman-Ford algorithm only defined for real weights')
    if G.dtype not in (np.float32, np.float64):
        raise TypeError(f'graph weights must be float32 or float64, got {G.dtype}')
    Gc = sp.csr_matrix((G.data.astype(np.float64), G.indices, G.indptr), shape=G.shape)
    Gd = DeviceCSR.from_scipy(Gc, check=False)
    seeds = np.asarray(seeds, dtype=np.intc).reshape(-1)
    seeds_dev = torch.as_tensor(seeds.astype(np.int32)).to(_device())
    d, z, _ = bellman_ford_pyamg_device(Gd, seeds_dev, fp64=G.dtype == np.float64)
    return d.cpu().numpy(), z.cpu().numpy().astype(np.intc)


def modified_bellman_ford(S_T, centers):
    """ns/lib/graph.py:7-53. S_T: torch sparse COO strength matrix; centers: 1-D int tensor.

    Returns (distance, nearest_center) on centers.device, fp32 / int64 like the reference
    (unreachable nodes: distance inf, nearest_center 0, as the reference's initial values).
    """
    G = _coo_to_device_csr(S_T)
    seeds = torch.as_tensor(centers).to(device=_device(), dtype=torch.int32)
    dist, lab, _ = modified_bellman_ford_device(G, seeds)
    nearest = lab.to(torch.int64)
    nearest = torch.where(nearest < 0, torch.zeros_like(nearest), nearest)
    dev = centers.device if isinstance(centers, torch.Tensor) else torch.device("cpu")
    return dist.to(dev), nearest.to(dev)


def legacy_permutation(seed, n, k):
    """np.random.RandomState(seed).permutation(n)[:k] (int seed in [0, 2^32)), bit for bit, as
    an int32 device tensor: numpy's MT19937 draws on the host, the Fisher-Yates swaps resolved
    for the first k positions on the device (csrc/seeds.hip) — instead of n random-address swaps
    of an 8n-byte array on the host (~1 s at the C4 size). Seeds of graph.py:230-231 and
    utils/evaluate_dataset.py:80-85. numpy's global generator is not touched (the caller's
    RandomState(seed) was a fresh generator too)."""
    seed = int(seed)
    if not 0 <= seed < 2 ** 32:
        raise ValueError("Seed must be between 0 and 2**32 - 1")
    if not 0 <= k <= n:
        raise ValueError("need 0 <= k <= n")
    out = torch.empty(max(int(k), 1), dtype=torch.int32, device=_device())
    call("mlamg_legacy_permutation", ctypes.c_uint32(seed), int(n), int(k), ptr(out),
         stream_ptr())
    return out[:k]


def aggregate_op_device(col_dev, k):
    """Agg (n x k, ones) from per-node aggregate columns (-1 = none) on the device."""
    h = ctypes.c_void_p()
    call("mlamg_aggregate_op", ptr(col_dev), int(col_dev.numel()), int(k), ctypes.byref(h),
         stream_ptr())
    return DeviceCSR(h)


def labels_to_columns(lab_dev, seeds_dev):
    col = torch.empty_like(lab_dev)
    call("mlamg_labels_to_columns", ptr(lab_dev), int(lab_dev.numel()), ptr(seeds_dev),
         int(seeds_dev.numel()), ptr(col), stream_ptr())
    return col


def nearest_center_to_agg(top_k, nearest_center):
    """ns/lib/graph.py:56-86: torch sparse COO (n x m) of fp32 ones, coalesced.

    Raises KeyError for an assignment that is not one of top_k, like the reference's dict lookup.
    """
    dev = _device()
    seeds = torch.as_tensor(top_k).to(device=dev, dtype=torch.int32)
    lab = torch.as_tensor(nearest_center).to(device=dev, dtype=torch.int32)
    col = labels_to_columns(lab, seeds)
    if bool((col < 0).any()):
        bad = int(lab[col < 0][0].item())
        raise KeyError(bad)
    Agg = aggregate_op_device(col, seeds.numel())
    A = Agg.to_scipy().tocoo()
    out_dev = top_k.device if isinstance(top_k, torch.Tensor) else torch.device("cpu")
    T = torch.sparse_coo_tensor(
        torch.as_tensor(np.vstack([A.row, A.col]).astype(np.int64)),
        torch.ones(A.nnz, dtype=torch.float32), (lab.numel(), seeds.numel()), device=out_dev)
    return T.coalesce()


def lloyd_cluster_device(G, seeds_dev, maxiter=10, exact=True):
    """pyamg 4.x lloyd_cluster on the device (seeds_dev updated in place). exact=True runs the
    outward pass in amg_core's sweep order as restated from pyamg 4.x (bitwise the oracle's
    restatement, ties included; pyamg itself is absent: parity unpinned); exact=False the
    order-independent rule (the hierarchy's option). Returns (distances, clusters, seeds,
    iters)."""
    n = G.shape[0]
    dev = _device()
    d = torch.empty(n, dtype=torch.float64, device=dev)
    c = torch.empty(n, dtype=torch.int32, device=dev)
    its = ctypes.c_int32()
    call("mlamg_lloyd_cluster" if exact else "mlamg_lloyd_cluster_canon", G.handle, ptr(seeds_dev), int(seeds_dev.numel()), int(maxiter),
         ptr(d), ptr(c), ctypes.byref(its), stream_ptr())
    return d, c, seeds_dev, int(its.value)


def distance_data(C, distance):
    """Edge weights of lloyd_aggregation (ns/lib/graph.py:201-212)."""
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
        raise ValueError(f'Unrecognized value distance={distance}')
    return data


def lloyd_aggregation(C, ratio=0.03, distance='unit', maxiter=10, rand=None):
    """ns/lib/graph.py:156-239 with pyamg.graph.lloyd_cluster run on the device.

    Returns (AggOp CSR int8 N x num_seeds, roots, seeds) like the reference.
    """
    if ratio <= 0 or ratio > 1:
        raise ValueError('ratio must be > 0.0 and <= 1.0')
    if not (sp.isspmatrix_csr(C) or sp.isspmatrix_csc(C)):
        raise TypeError('expected csr_matrix or csc_matrix')
    data = distance_data(C, distance)
    if rand is None:
        rand = np.random
    elif isinstance(rand, int):
        rand = np.random.RandomState(rand)
    elif not isinstance(rand, np.random.RandomState):
        raise TypeError('rand should be an integer seed value or a random state')
    if C.dtype == complex:
        data = np.real(data)
    assert data.min() >= 0
    G = C.__class__((data, C.indices, C.indptr), shape=C.shape)
    if sp.isspmatrix_csc(G):
        # pyamg's amg_core reads G.indptr/G.indices as CSR arrays whatever the format, so a CSC
        # graph is walked as its transpose; reproduce that
        G = sp.csr_matrix((G.data, G.indices, G.indptr), shape=G.shape)
    N = C.shape[0]
    num_seeds = int(np.ceil(ratio * N))
    seeds = rand.permutation(N)[:num_seeds]
    Gd = DeviceCSR.from_scipy(G)
    seeds_dev = torch.as_tensor(seeds.astype(np.int32)).to(_device())
    _, clusters, roots_dev, _ = lloyd_cluster_device(Gd, seeds_dev, maxiter)
    Agg = aggregate_op_device(clusters, num_seeds).to_scipy()
    AggOp = sp.csr_matrix((Agg.data.astype(np.int8), Agg.indices, Agg.indptr),
                          shape=(G.shape[0], num_seeds))
    roots = roots_dev.cpu().numpy().astype(np.intc)
    return AggOp, roots, seeds


def _asgraph(G):
    """pyamg.graph.asgraph: CSR/CSC kept (amg_core walks either's arrays as CSR), anything else
    becomes csr_matrix; square required."""
    if not (sp.isspmatrix_csr(G) or sp.isspmatrix_csc(G)):
        G = sp.csr_matrix(G)
    if G.shape[0] != G.shape[1]:
        raise ValueError('expected square matrix')
    return G


def lloyd_cluster(G, seeds, maxiter=10):
    """pyamg 4.x pyamg.graph.lloyd_cluster(G, seeds, maxiter) on the device (the call at
    ns/lib/graph.py:232 and inside pyamg.aggregation.lloyd_aggregation, utils/common.py:91).

    seeds: an int (that many seeds drawn as np.random.permutation(N)[:seeds] from numpy's
    GLOBAL generator, like pyamg) or an array of seed nodes. Returns (distances float64,
    clusters intc, seeds intc) like pyamg; clusters and seeds bitwise the oracle's restatement of
    amg_core's sweep order, ties included (pyamg absent: parity with amg_core unpinned).
    Weights are used in float64 (the reference's graphs are float64)."""
    G = _asgraph(G)
    N = G.shape[0]
    if G.dtype.kind == 'c':
        G = abs(G)
    if np.isscalar(seeds):
        seeds = np.random.permutation(N)[:seeds].astype('intc')
    else:
        seeds = np.array(seeds, dtype='intc')
    if len(seeds) < 1:
        raise ValueError('at least one seed is required')
    if seeds.min() < 0:
        raise ValueError('invalid seed index (%d)' % seeds.min())
    if seeds.max() >= N:
        raise ValueError('invalid seed index (%d)' % seeds.max())
    if maxiter < 1:  # pyamg's loop would not run and return uninitialised arrays
        raise ValueError('maxiter must be >= 1')
    Gc = sp.csr_matrix((np.asarray(G.data, dtype=np.float64), G.indices, G.indptr),
                       shape=G.shape)
    Gd = DeviceCSR.from_scipy(Gc, check=False)
    seeds_dev = torch.as_tensor(seeds.astype(np.int32)).to(_device())
    d, c, s, _ = lloyd_cluster_device(Gd, seeds_dev, maxiter)
    return d.cpu().numpy(), c.cpu().numpy().astype('intc'), s.cpu().numpy().astype('intc')


def pyamg_lloyd_aggregation(C, ratio=0.03, distance='unit', maxiter=10):
    """pyamg 4.x pyamg.aggregation.lloyd_aggregation (utils/common.py:91,
    utils/evaluate_dataset.py:77 call it directly): no `rand`; num_seeds = int(min(max(ratio N,
    1), N)) drawn inside lloyd_cluster from the global generator; returns (AggOp int8 CSR,
    seeds)."""
    if ratio <= 0 or ratio > 1:
        raise ValueError('ratio must be > 0.0 and <= 1.0')
    if not (sp.isspmatrix_csr(C) or sp.isspmatrix_csc(C)):
        raise TypeError('expected csr_matrix or csc_matrix')
    data = distance_data(C, distance)
    if C.dtype == complex:
        data = np.real(data)
    assert data.min() >= 0
    G = C.__class__((data, C.indices, C.indptr), shape=C.shape)
    num_seeds = int(min(max(ratio * G.shape[0], 1), G.shape[0]))
    _, clusters, seeds = lloyd_cluster(G, num_seeds, maxiter=maxiter)
    row = (clusters >= 0).nonzero()[0]
    col = clusters[row]
    AggOp = sp.coo_matrix((np.ones(len(row), dtype='int8'), (row, col)),
                          shape=(G.shape[0], num_seeds)).tocsr()
    return AggOp, seeds


def num_connected_components(adj):
    """ns/lib/graph.py:89-122: number of depth-first searches needed to visit every node, each
    started at the first unvisited node and following, from node i, the nonzeros of column i
    (adj[:, i]) — the connected components of a symmetric adjacency. Host-side graph utility
    (not on the V-cycle path); iterative, O(nnz)."""
    A = sp.csc_matrix(adj)
    A.eliminate_zeros()
    n = A.shape[0]
    ip, ij = A.indptr, A.indices
    visited = np.zeros(n, dtype=bool)
    count = 0
    start = 0
    while True:
        while start < n and visited[start]:
            start += 1
        if start >= n:
            return count
        count += 1
        stack = [start]
        while stack:
            i = stack.pop()
            visited[i] = True
            nb = ij[ip[i]:ip[i + 1]]
            stack.extend(nb[~visited[nb]].tolist())


def check_aggregates_connected(A, Agg):
    """ns/lib/graph.py:125-153: True when every aggregate (column of the tentative Agg) induces
    a connected subgraph of A — the block diagonal of the aggregates' principal submatrices has
    exactly k connected components."""
    A = sp.csr_matrix(A)
    Agg = sp.csc_matrix(Agg)
    n, k = Agg.shape
    blocks = []
    for i in range(k):
        nodes = Agg[:, i].nonzero()[0]
        blocks.append(A[nodes][:, nodes])
    return num_connected_components(sp.block_diag(blocks).tocsc()) == k
