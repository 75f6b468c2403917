"""TEST INFRASTRUCTURE ONLY — torch (CPU, fp32) restatement of the GNN layers of
ns/model/agg_interp.py (FullAggNet and its parts, :80-486) with torch_geometric 2.x semantics
(torch_geometric is absent): TAGConv (K=3, gcn_norm without self loops, aggr 'add'), NNConv
(edge network x_j @ nn(e).view(in, out), aggr 'add', root weight, bias), InstanceNorm
(affine False, per channel over the nodes, biased variance, eps 1e-5). It runs on the parameters
of an mlamg.gnn module (same layout as the reference's) with plain torch ops, so the device
kernels can be compared with it at the same (seeded) weights.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
import torch
import torch.nn.functional as F


class RefGraph:
    """graph_from_matrix_basic / graph_from_matrix (ns/model/data.py:22-46)."""

    def __init__(self, A, agg=None):
        A = sp.csr_matrix(A)
        n = A.shape[0]
        src = np.repeat(np.arange(n), np.diff(A.indptr))
        tgt = A.indices.astype(np.int64)
        feats = [np.abs(A.data.astype(np.float32))]
        if agg is not None:
            clusters = np.asarray(sp.csr_matrix(agg).argmax(axis=1)).ravel()
            feats.append((clusters[src] != clusters[tgt]).astype(np.float32))
        self.n = n
        self.edge_index = torch.as_tensor(np.vstack([src, tgt]).astype(np.int64))
        self.edge_attr = torch.as_tensor(np.stack(feats, axis=1))
        self.x = torch.full((n,), 1.0 / n, dtype=torch.float32)


def _scatter_add(vals, index, n):
    out = torch.zeros((n,) + tuple(vals.shape[1:]), dtype=vals.dtype)
    return out.index_add_(0, index, vals)


def instance_norm(x):
    return F.instance_norm(x.t().unsqueeze(0), eps=1e-5).squeeze(0).t()


def gcn_norm(edge_index, w, n):
    row, col = edge_index
    deg = _scatter_add(w, col, n)
    dis = deg.pow(-0.5)
    dis[torch.isinf(dis)] = 0.0
    return dis[row] * w * dis[col]


def tagconv(mod, x, edge_index, edge_weight, n):
    w = gcn_norm(edge_index, edge_weight.reshape(-1), n)
    out = F.linear(x, mod.lins[0].weight)
    for lin in mod.lins[1:]:
        x = _scatter_add(w.view(-1, 1) * x[edge_index[0]], edge_index[1], n)
        out = out + F.linear(x, lin.weight)
    return out + mod.bias


def nnconv(mod, x, edge_index, edge_attr, n):
    h = edge_attr.reshape(-1, mod.nn[1].in_features)
    for layer in list(mod.nn)[1:]:
        h = layer(h)
    weight = h.view(-1, mod.in_channels, mod.out_channels)
    msg = torch.matmul(x[edge_index[0]].unsqueeze(1), weight).squeeze(1)
    out = _scatter_add(msg, edge_index[1], n)
    return out + F.linear(x, mod.lin.weight) + mod.bias


def edge_model(mod, src, dest, edge_attr):
    return mod.edge_mlp(torch.cat([src, dest, edge_attr], 1))


@torch.no_grad()
def mpnn(mod, g):
    """MPNN.forward (agg_interp.py:124-141)."""
    x, ei, ea = g.x.reshape(-1, 1), g.edge_index, g.edge_attr
    row, col = ei
    n = g.n
    x = F.relu(nnconv(mod.node_conv_in, instance_norm(x), ei, abs(ea), n)) + x
    ea = F.relu(edge_model(mod.edge_conv_in, x[row], x[col], ea.float())) + ea
    for i in range(mod.num_internal_conv):
        x = F.relu(nnconv(mod.node_convs[i], instance_norm(x), ei, ea, n)) + x
        ea = F.relu(edge_model(mod.edge_convs[i], x[row], x[col], ea.float())) + ea
    x = F.relu(nnconv(mod.node_conv_out, instance_norm(x), ei, ea, n))
    ea = F.relu(edge_model(mod.edge_conv_out, x[row], x[col], ea.float()))
    return x, ea


def topk_vec(x, k):
    """agg_interp.py:14-22 with ties to the smaller index (stable descending sort)."""
    x = x.reshape(-1)
    order = torch.sort(x, descending=True, stable=True).indices[:k]
    v = torch.zeros_like(x)
    v[order] = 1.0
    return v


@torch.no_grad()
def agg_layer_raw(mod, g, x):
    """AggBinarizationLayer.forward_raw (agg_interp.py:209-220)."""
    if x.dim() == 1:
        x = x.unsqueeze(1)
    for i in range(mod.num_conv):
        x = instance_norm(x)
        x = tagconv(mod.ncs[i], x, g.edge_index, g.edge_attr, g.n)
        x = F.relu(x)
        x = mod.fcs[i](x)
    return x


@torch.no_grad()
def aggnet(mod, g, k):
    x = g.x
    for layer in mod.layers:
        x = topk_vec(agg_layer_raw(layer, g, x), k)
    return x


@torch.no_grad()
def full_forward(net, A, alpha, x=None, bf_dtype=np.float32):
    """FullAggNet.forward (agg_interp.py:458-486) restated on a module's parameters: AggNet
    scores and top-k seeds, CNet edge weights C (sp.coo_matrix over the graph's edges, :469-471),
    pyamg 4.x bellman_ford(C, top_k) (restated.pyamg_bellman_ford, the oracle's C restatement),
    nearest_center_to_agg (dict lookup: KeyError on an unreached node), PNet on
    graph_from_matrix(A, Agg) and P = P_hat Agg. x replaces the constant 1/n node input;
    bf_dtype the Bellman-Ford arithmetic (float32: the weights' dtype; float64 widened).
    Returns (Agg scipy CSR n x k, P scipy CSR, C scipy CSR, top_k tensor, scores tensor)."""
    from . import restated
    A = sp.csr_matrix(A)
    m = A.shape[0]
    k = int(np.ceil(alpha * m))
    g = RefGraph(A)
    if x is not None:
        g.x = torch.as_tensor(np.asarray(x), dtype=torch.float32).reshape(-1)
    scores = aggnet(net.AggNet, g, k).reshape(-1)
    top_k = torch.where(scores == 1)[0]
    _, bfe = mpnn(net.CNet, g)
    ei = g.edge_index.numpy()
    C = sp.coo_matrix((bfe.reshape(-1).numpy(), (ei[0], ei[1])), shape=(m, m))
    _, nearest, _ = restated.pyamg_bellman_ford(C, top_k.numpy(), dtype=bf_dtype)
    pos = {int(s): t for t, s in enumerate(top_k.tolist())}
    col = np.array([pos[int(c)] for c in nearest], dtype=np.int64)
    Agg = sp.csr_matrix((np.ones(m), (np.arange(m), col)), shape=(m, len(pos)))
    gp = RefGraph(A, agg=Agg)
    if x is not None:
        gp.x = g.x
    _, pe = mpnn(net.PNet, gp)
    P_hat = sp.csr_matrix((pe.reshape(-1).numpy().astype(np.float64), A.indices, A.indptr),
                          shape=A.shape)
    return Agg, (P_hat @ Agg).tocsr(), C.tocsr(), top_k, scores
