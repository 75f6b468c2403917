"""GNN inference for learned aggregates and interpolation on the device.

Mirrors ns/model/agg_interp.py: `FullAggNet.forward(A, alpha)` (:432-486) -> AggNet node scores
(TAGConv / InstanceNorm / MLP layers, top-k seeds), CNet (MPNN: NNConv + edge models) edge
weights for Bellman-Ford, the aggregates, PNet (MPNN) edge values P_hat and P = P_hat Agg. The
modules hold their parameters like the reference's (same attribute names and shapes, so a
reference state_dict — e.g. from ns.ga.torch.model_weights_as_dict — loads with
load_state_dict); the forward passes run on csrc/gnn.hip kernels (fp32, like the reference),
not on torch ops. torch_geometric is absent: its layers (TAGConv K=3 with gcn_norm, NNConv aggr
'add' with root weight, InstanceNorm) are restated from its 2.x semantics; the reference's
trained weights are not shipped, so parity is against oracle/gnn_ref.py (a torch restatement
of the same layers) at seeded weights — parity unpinned with respect to torch_geometric itself.
"""
from __future__ import annotations

import ctypes

import numpy as np
import scipy.sparse as sp
import torch
import torch.nn as nn

from . import _lib
from ._lib import call, ptr, stream_ptr


def _p(t):
    return ptr(t) if t is not None else None


# ------------------------------------------------------------------------------------ graphs
class Graph:
    """graph_from_matrix_basic(A) / graph_from_matrix(A, agg) (ns/model/data.py:22-46) on the
    device: edges = A's stored entries in row-major order (networkx DiGraph order), edge_attr =
    |a_ij| (fp32) [, cluster_adj = 0 if both ends are in the same aggregate], x = 1/n."""

    def __init__(self, A, agg=None, device=None):
        A = sp.csr_matrix(A)
        dev = device or torch.device("cuda", torch.cuda.current_device())
        n = A.shape[0]
        src = np.repeat(np.arange(n, dtype=np.int32), np.diff(A.indptr))
        tgt = A.indices.astype(np.int32)
        feats = [np.abs(A.data.astype(np.float32))]
        if agg is not None:
            clusters = np.asarray(sp.csr_matrix(agg).argmax(axis=1)).ravel()
            feats.append((clusters[src] != clusters[tgt]).astype(np.float32))
        ea = np.stack(feats, axis=1)
        order = np.argsort(tgt, kind="stable")          # each target's edges, ascending source
        tptr = np.zeros(n + 1, dtype=np.int32)
        np.cumsum(np.bincount(tgt, minlength=n), out=tptr[1:])
        self.n, self.E, self.fe = n, int(len(src)), ea.shape[1]
        self.crow = torch.as_tensor(A.indptr.astype(np.int32), device=dev)
        self.src = torch.as_tensor(src, device=dev)
        self.tgt = torch.as_tensor(tgt, device=dev)
        self.tptr = torch.as_tensor(tptr, device=dev)
        self.teid = torch.as_tensor(order.astype(np.int32), device=dev)
        self.edge_attr = torch.as_tensor(np.ascontiguousarray(ea), device=dev)
        self.x = torch.full((n, 1), 1.0 / n, dtype=torch.float32, device=dev)
        self.edge_index = torch.stack([self.src.long(), self.tgt.long()])
        self._gcn = None

    def with_clusters(self, col):
        """graph_from_matrix(A, Agg) from this graph and the device aggregate column of every
        node (-1: none; agg_op.argmax(axis=1) of an empty row is 0): edge feature 2 =
        cluster_adj = 0 if both ends are in the same aggregate, else 1. Shares the structure."""
        g = object.__new__(Graph)
        g.__dict__.update(self.__dict__)
        c = torch.where(col < 0, torch.zeros_like(col), col)
        adj = (c[self.src.long()] != c[self.tgt.long()]).to(torch.float32)
        g.edge_attr = torch.stack([self.edge_attr[:, 0], adj], dim=1).contiguous()
        g.fe = 2
        g._gcn = None
        return g

    def csr(self, values):
        """A DeviceCSR on this graph's pattern with the given per-edge values (fp64 copy)."""
        from .sparse import DeviceCSR
        return DeviceCSR.from_torch(self.crow, self.tgt, values.reshape(-1).double().contiguous(),
                                    (self.n, self.n))

    def gcn_weights(self):
        """gcn_norm(edge_index, edge_attr[:, 0]) without self loops (TAGConv normalize=True)."""
        if self._gcn is None:
            w = self.edge_attr[:, 0].contiguous()
            dis = torch.empty(self.n, dtype=torch.float32, device=w.device)
            wn = torch.empty(self.E, dtype=torch.float32, device=w.device)
            call("mlamg_gnn_gcn_norm", ptr(self.tptr), ptr(self.teid), ptr(self.src),
                 ptr(self.tgt), ptr(w), int(self.n), int(self.E), ptr(dis), ptr(wn), stream_ptr())
            self._gcn = wn
        return self._gcn


# ------------------------------------------------------------------------------------ kernels
def linear(x, W, b=None, act=0, out=None, beta=0.0, residual=None):
    x = x.contiguous()
    M, K = x.shape
    N = W.shape[0]
    y = out if out is not None else torch.empty((M, N), dtype=torch.float32, device=x.device)
    rc = 0 if residual is None else residual.shape[1]
    call("mlamg_gnn_linear", ptr(x), int(M), int(K), ptr(W.detach().contiguous()),
         _p(None if b is None else b.detach().contiguous()), int(N), int(act), float(beta),
         _p(None if residual is None else residual.contiguous()), int(rc), ptr(y), stream_ptr())
    return y


def instance_norm(x, eps=1e-5):
    x = x.contiguous()
    y = torch.empty_like(x)
    call("mlamg_gnn_instance_norm", ptr(x), int(x.shape[0]), int(x.shape[1]), float(eps), ptr(y),
         stream_ptr())
    return y


def propagate(g, w, x):
    x = x.contiguous()
    y = torch.empty_like(x)
    call("mlamg_gnn_propagate", ptr(g.tptr), ptr(g.teid), ptr(g.src), ptr(w), ptr(x), int(g.n),
         int(x.shape[1]), ptr(y), stream_ptr())
    return y


def topk_vec(x, k):
    """agg_interp.py:14-22; ties broken by the smaller node index (torch.argsort leaves them
    unspecified)."""
    s = x.reshape(-1).contiguous()
    vec = torch.empty_like(s)
    idx = torch.empty(int(k), dtype=torch.int32, device=s.device)
    call("mlamg_gnn_topk", ptr(s), int(s.numel()), int(k), ptr(vec), _p(idx if k else None),
         stream_ptr())
    return vec, idx


# ------------------------------------------------------------------------------------ modules
class TensorLambda(nn.Module):
    """Parameter-free placeholder at index 0 of NNConv's edge network (agg_interp.py:24-34)."""

    def __init__(self, func=None):
        super().__init__()
        self.f = func

    def forward(self, x):
        return self.f(x) if self.f else x


class TAGConv(nn.Module):
    """torch_geometric TAGConv(in, out, K=3): sum_k lins[k](A_hat^k x) + bias."""

    def __init__(self, in_channels, out_channels, K=3):
        super().__init__()
        self.K = K
        self.lins = nn.ModuleList([nn.Linear(in_channels, out_channels, bias=False)
                                   for _ in range(K + 1)])
        self.bias = nn.Parameter(torch.zeros(out_channels))

    def run(self, g, x, act=0):
        wn = g.gcn_weights()
        out = linear(x, self.lins[0].weight)
        for k in range(1, self.K + 1):
            x = propagate(g, wn, x)
            last = k == self.K
            out = linear(x, self.lins[k].weight, b=self.bias if last else None,
                         act=act if last else 0, out=out, beta=1.0)
        return out


class NNConv(nn.Module):
    """torch_geometric NNConv(in, out, nn, aggr='add'): sum over incoming edges of
    x_src @ nn(e).view(in, out), + lin(x) (root weight), + bias."""

    def __init__(self, in_channels, out_channels, edge_features):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.nn = nn.Sequential(TensorLambda(), nn.Linear(edge_features, 4), nn.ReLU(),
                                nn.Linear(4, 16), nn.ReLU(),
                                nn.Linear(16, in_channels * out_channels), nn.ReLU())
        self.lin = nn.Linear(in_channels, out_channels, bias=False)
        self.bias = nn.Parameter(torch.zeros(out_channels))

    def run(self, g, x, ea, act=0, residual=None):
        x = x.contiguous()
        ea = ea.contiguous()
        n = x.shape[0]
        root = linear(x, self.lin.weight)
        msg = torch.empty((max(g.E, 1), self.out_channels), dtype=torch.float32, device=x.device)
        y = torch.empty((n, self.out_channels), dtype=torch.float32, device=x.device)
        L1, L2, L3 = self.nn[1], self.nn[3], self.nn[5]
        rc = 0 if residual is None else residual.shape[1]
        call("mlamg_gnn_nnconv", ptr(g.tptr), ptr(g.teid), ptr(g.src), ptr(ea), int(g.E),
             int(ea.shape[1]), ptr(L1.weight.detach()), ptr(L1.bias.detach()),
             ptr(L2.weight.detach()), ptr(L2.bias.detach()), ptr(L3.weight.detach()),
             ptr(L3.bias.detach()), ptr(x), int(n), int(self.in_channels),
             int(self.out_channels), ptr(root), ptr(self.bias.detach()), int(act),
             _p(None if residual is None else residual.contiguous()), int(rc), ptr(msg), ptr(y),
             stream_ptr())
        return y


class SmallEdgeModel(nn.Module):
    """agg_interp.py:37-55: Linear(in, hid) - ReLU - LayerNorm - Linear(hid, out)."""

    def __init__(self, in_dim, hid_dim, out_dim):
        super().__init__()
        self.edge_mlp = nn.Sequential(nn.Linear(in_dim, hid_dim), nn.ReLU(),
                                      nn.LayerNorm([hid_dim]), nn.Linear(hid_dim, out_dim))

    def run(self, g, x, ea, act=0, residual=None):
        l1, ln, l2 = self.edge_mlp[0], self.edge_mlp[2], self.edge_mlp[3]
        x = x.contiguous()
        ea = ea.contiguous()
        C = l2.weight.shape[0]
        out = torch.empty((max(g.E, 1), C), dtype=torch.float32, device=x.device)
        rc = 0 if residual is None else residual.shape[1]
        call("mlamg_gnn_edge_mlp", ptr(g.src), ptr(g.tgt), ptr(x), int(x.shape[1]), ptr(ea),
             int(ea.shape[1]), int(g.E), ptr(l1.weight.detach()), ptr(l1.bias.detach()),
             int(l1.weight.shape[0]), ptr(ln.weight.detach()), ptr(ln.bias.detach()),
             ptr(l2.weight.detach()), ptr(l2.bias.detach()), int(C), int(act),
             _p(None if residual is None else residual.contiguous()), int(rc), ptr(out),
             stream_ptr())
        return out[:g.E]


class MPNN(nn.Module):
    """agg_interp.py:80-141 (node/edge activations ReLU)."""

    def __init__(self, dim, num_internal_conv=4, input_edge_features=1):
        super().__init__()
        self.node_conv_in = NNConv(1, dim, input_edge_features)
        self.normalize_in = nn.Identity()  # InstanceNorm(dim): no parameters
        self.edge_conv_in = SmallEdgeModel(dim * 2 + input_edge_features, dim, 2)
        self.node_convs = nn.ModuleList([NNConv(dim, dim, 2) for _ in range(num_internal_conv)])
        self.edge_convs = nn.ModuleList([SmallEdgeModel(dim * 2 + 2, dim, 2)
                                         for _ in range(num_internal_conv)])
        self.normalizations = nn.ModuleList([nn.Identity() for _ in range(num_internal_conv)])
        self.num_internal_conv = num_internal_conv
        self.node_conv_out = NNConv(dim, 1, 2)
        self.normalize_out = nn.Identity()
        self.edge_conv_out = SmallEdgeModel(4, dim, 1)

    @torch.no_grad()
    def run(self, g):
        x = g.x
        ea = g.edge_attr
        x = self.node_conv_in.run(g, instance_norm(x), ea, act=1, residual=x)
        ea = self.edge_conv_in.run(g, x, ea, act=1, residual=ea)
        for i in range(self.num_internal_conv):
            x = self.node_convs[i].run(g, instance_norm(x), ea, act=1, residual=x)
            ea = self.edge_convs[i].run(g, x, ea, act=1, residual=ea)
        x = self.node_conv_out.run(g, instance_norm(x), ea, act=1)
        ea = self.edge_conv_out.run(g, x, ea, act=1)
        return x, ea


def _fc(dim, last_out):
    layers = []
    for i in range(5 if last_out is None else 4):
        layers += [nn.Linear(dim, dim), nn.ReLU()]
    if last_out is not None:
        layers += [nn.Linear(dim, last_out), nn.ReLU()]
    return nn.Sequential(*layers)


class AggBinarizationLayer(nn.Module):
    """agg_interp.py:144-220."""

    def __init__(self, dim, num_conv=6):
        super().__init__()
        ncs = [TAGConv(1, dim)] + [TAGConv(dim, dim) for _ in range(num_conv - 1)]
        fcs = [_fc(dim, None) for _ in range(num_conv - 1)] + [_fc(dim, 1)]
        self.ncs = nn.ModuleList(ncs)
        self.fcs = nn.ModuleList(fcs)
        self.norms = nn.ModuleList([nn.Identity() for _ in range(num_conv)])  # InstanceNorm
        self.num_conv = num_conv
        self.dim = dim

    def run_raw(self, g, x):
        if x.dim() == 1:
            x = x.unsqueeze(1)
        for i in range(self.num_conv):
            x = instance_norm(x)
            x = self.ncs[i].run(g, x, act=1)        # relu(TAGConv(x))
            for lin in self.fcs[i]:
                if isinstance(lin, nn.Linear):
                    x = linear(x, lin.weight, lin.bias, act=1)
        return x

    @torch.no_grad()
    def run(self, g, x, k):
        return topk_vec(self.run_raw(g, x), k)[0]


class AggNet(nn.Module):
    """agg_interp.py:223-241."""

    def __init__(self, dim, iterations=2, num_conv=6):
        super().__init__()
        self.layers = nn.ModuleList([AggBinarizationLayer(dim, num_conv=num_conv)
                                     for _ in range(iterations)])
        self.num_iterations = iterations

    @torch.no_grad()
    def run(self, g, k):
        x = g.x
        for layer in self.layers:
            x = layer.run(g, x, k)
        return x


class FullAggNet(nn.Module):
    """agg_interp.py:379-486 (inference)."""

    def __init__(self, dim=64, num_conv=2, iterations=4):
        super().__init__()
        self.PNet = MPNN(dim, num_internal_conv=4, input_edge_features=2)
        self.AggNet = AggNet(dim, num_conv=num_conv, iterations=iterations)
        self.CNet = MPNN(dim, num_internal_conv=5)

    @property
    def device(self):
        return next(self.parameters()).device

    @torch.no_grad()
    def forward(self, A, alpha, aggregation="pyamg", x=None):
        """Returns (agg, P, bf_weights, cluster_centers, node_weights) like :442-486: agg and P
        as torch sparse COO (n x k, fp32), bf_weights as torch sparse COO (the CNet edge
        values C, edge (i, j) = A's entry (i, j)), cluster_centers the seed nodes (ascending),
        node_weights the 0/1 scores.

        aggregation: "pyamg" (default) is the reference's step, pyamg.graph.bellman_ford(C,
        top_k) (:475): pull sweeps x_i <- min(x_i, C_ij + x_j) in float32, emulated exactly
        on the device (graph.bellman_ford_pyamg_device), so every node's nearest seed is pyamg's,
        ties included; a node no seed reaches raises KeyError like nearest_center_to_agg's dict
        lookup (ns/lib/graph.py:83). "parallel" runs the same distances with the multi-workgroup
        order-independent Bellman-Ford (graph.hip k_bf_sweep, on C^T so the direction is
        pyamg's): nearest seeds equal pyamg's whenever shortest paths are unique, ties go to the
        smallest seed id, unreached nodes get no aggregate. "pyamg64": pyamg's sweeps in float64
        on the widened weights (what a pyamg build binding only double computes; the pyamg
        version is unpinned). x: node features replacing the
        reference graph's constant 1/n (graph_from_matrix_basic, ns/model/data.py:22-31) —
        not in the reference's signature; a test hook for well-conditioned inputs."""
        from .graph import (aggregate_op_device, bellman_ford_device, bellman_ford_pyamg_device,
                            labels_to_columns)
        from .sparse import DeviceCSR
        if aggregation not in ("pyamg", "pyamg64", "parallel"):
            raise ValueError("aggregation must be 'pyamg', 'pyamg64' or 'parallel', got "
                             f"{aggregation!r}")
        A = sp.csr_matrix(A)
        m = A.shape[0]
        k = int(np.ceil(alpha * m))
        g = Graph(A, device=self.device)
        if x is not None:
            g.x = torch.as_tensor(x, dtype=torch.float32).reshape(m, 1).to(self.device)
        node_scores = self.AggNet.run(g, k).reshape(-1)
        top_k = torch.nonzero(node_scores == 1).reshape(-1)
        # Bellman-Ford over the CNet edge weights from the seeds (:466-475), on the device
        _, bf_edges = self.CNet.run(g)
        C = g.csr(bf_edges)
        seeds = top_k.to(torch.int32)
        if aggregation != "parallel" and not A.has_canonical_format:
            # pyamg's asgraph turns the COO C (:471) into csr_matrix: columns sorted, duplicate
            # edges summed in C's float32; its sweep visits each row in that order
            Cs = C.to_scipy()
            Cc = sp.coo_matrix((Cs.data.astype(np.float32), (np.repeat(np.arange(m),
                                np.diff(Cs.indptr)), Cs.indices)), shape=(m, m)).tocsr()
            Cc.sum_duplicates()
            C = DeviceCSR.from_scipy(sp.csr_matrix((Cc.data.astype(np.float64), Cc.indices,
                                                    Cc.indptr), shape=(m, m)), check=False)
        if aggregation != "parallel":
            _, lab, _ = bellman_ford_pyamg_device(C, seeds, fp64=aggregation == "pyamg64")
            if bool((lab < 0).any()):
                raise KeyError(-1)
        else:
            _, lab, _ = bellman_ford_device(C.T, seeds)
        col = labels_to_columns(lab, seeds)
        Agg = aggregate_op_device(col, k)
        # P_hat from PNet on graph_from_matrix(A, Agg), P = P_hat Agg (:476-484)
        _, p_edges = self.PNet.run(g.with_clusters(col))
        P = g.csr(p_edges) @ Agg

        def to_t(M, dtype=torch.float32):
            crow, cj, v = M.to_torch()
            rows = torch.repeat_interleave(torch.arange(M.shape[0], device=crow.device),
                                           (crow[1:] - crow[:-1]).long())
            return torch.sparse_coo_tensor(torch.stack([rows, cj.long()]), v.to(dtype),
                                           M.shape).coalesce()

        return to_t(Agg), to_t(P), to_t(C), top_k, node_scores
