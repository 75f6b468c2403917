"""GPU: GNN inference of ns/model/agg_interp.py FullAggNet on the device
(csrc/gnn.hip, mlamg.gnn) against oracle/gnn_ref.py, a torch fp32 restatement of the same layers
(torch_geometric 2.x semantics; torch_geometric and the reference's trained weights are absent:
parity unpinned with respect to them) at the same seeded weights. fp32 with different summation
orders: rtol 1e-4 relative to each tensor's scale. Top-k seed selection is exact given the same
scores (ties to the smaller node index)."""
import numpy as np
import pytest
import scipy.sparse as sp

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch


def _close(a, b, rtol=1e-4):
    a = a.detach().cpu().numpy().astype(np.float64)
    b = b.detach().cpu().numpy().astype(np.float64)
    scale = max(np.abs(b).max(), 1e-30)
    return np.abs(a - b).max() <= rtol * scale, np.abs(a - b).max() / scale


def _A(m=12):
    from mlamg import problems
    return problems.poisson_2d_5pt(m)


@pytest.mark.parametrize("edge_features", (1, 2))
def test_mpnn_layers_match_oracle(torch_cuda, edge_features):
    """Every MPNN layer (NNConv with its edge network, InstanceNorm, the edge model with
    LayerNorm, the ReLU + residual post-ops) on the device, fed the oracle's own input at that
    depth, against the oracle's layer: rtol 1e-5. (The whole stack is compared layer by layer:
    InstanceNorm of a nearly constant channel — the constant input x = 1/n of the reference's
    graphs — turns fp32 rounding into O(1) differences that the random-weight network then
    amplifies, so end-to-end equality of two fp32 implementations is not a meaningful test.)"""
    torch = torch_cuda
    import torch.nn.functional as F
    from mlamg import gnn, problems
    from oracle import gnn_ref
    A = problems.jump_2d(24, problems.voronoi_jumps(np.random.RandomState(0)))
    n = A.shape[0]
    agg = sp.csr_matrix((np.ones(n), (np.arange(n), np.arange(n) // 4))) \
        if edge_features == 2 else None
    torch.manual_seed(0)
    net = gnn.MPNN(64, num_internal_conv=3, input_edge_features=edge_features)
    netd = gnn.MPNN(64, num_internal_conv=3, input_edge_features=edge_features)
    netd.load_state_dict(net.state_dict())
    netd = netd.cuda()
    g, rg = gnn.Graph(A, agg=agg), gnn_ref.RefGraph(A, agg=agg)
    row, col = rg.edge_index
    c = lambda t: t.cuda()  # noqa: E731
    x = torch.randn(n, 1)  # a non-constant input: InstanceNorm well conditioned
    ea = rg.edge_attr
    xn = gnn_ref.instance_norm(x)
    assert _close(gnn.instance_norm(c(x)), xn, 1e-6)[0]
    x1 = F.relu(gnn_ref.nnconv(net.node_conv_in, xn, rg.edge_index, ea, n)) + x
    ok, err = _close(netd.node_conv_in.run(g, c(xn), c(ea), act=1, residual=c(x)), x1, 1e-5)
    assert ok, err
    ea1 = F.relu(gnn_ref.edge_model(net.edge_conv_in, x1[row], x1[col], ea)) + ea
    ok, err = _close(netd.edge_conv_in.run(g, c(x1), c(ea), act=1, residual=c(ea)), ea1, 1e-5)
    assert ok, err
    x, ea = x1 + 0.1 * torch.randn(n, 64), ea1
    for i in range(net.num_internal_conv):
        xn = gnn_ref.instance_norm(x)
        ok, err = _close(gnn.instance_norm(c(x)), xn, 1e-5)
        assert ok, (i, err)
        y = F.relu(gnn_ref.nnconv(net.node_convs[i], xn, rg.edge_index, ea, n)) + x
        ok, err = _close(netd.node_convs[i].run(g, c(xn), c(ea), act=1, residual=c(x)), y, 1e-5)
        assert ok, (i, err)
        x = y
        e2 = F.relu(gnn_ref.edge_model(net.edge_convs[i], x[row], x[col], ea)) + ea
        ok, err = _close(netd.edge_convs[i].run(g, c(x), c(ea), act=1, residual=c(ea)), e2, 1e-5)
        assert ok, (i, err)
        ea = e2
    xn = gnn_ref.instance_norm(x)
    xo = F.relu(gnn_ref.nnconv(net.node_conv_out, xn, rg.edge_index, ea, n))
    ok, err = _close(netd.node_conv_out.run(g, c(xn), c(ea), act=1), xo, 1e-5)
    assert ok, err
    eo = F.relu(gnn_ref.edge_model(net.edge_conv_out, xo[row], xo[col], ea))
    ok, err = _close(netd.edge_conv_out.run(g, c(xo), c(ea), act=1), eo, 1e-5)
    assert ok, err


def test_aggnet_scores_and_topk(torch_cuda):
    torch = torch_cuda
    from mlamg import gnn
    from oracle import gnn_ref
    torch.manual_seed(1)
    layer = gnn.AggBinarizationLayer(64, num_conv=2)
    A = _A(16)
    g = gnn.Graph(A)
    k = int(np.ceil(0.1 * A.shape[0]))
    ld = gnn.AggBinarizationLayer(64, num_conv=2)
    ld.load_state_dict(layer.state_dict())
    sd = ld.cuda().run_raw(g, g.x)
    sr = gnn_ref.agg_layer_raw(layer, gnn_ref.RefGraph(A), gnn_ref.RefGraph(A).x)
    ok, err = _close(sd, sr, 1e-5)
    assert ok, err
    # top-k of the same scores: exact, ties to the smaller index
    vec_d, idx_d = gnn.topk_vec(sd, k)
    vec_r = gnn_ref.topk_vec(sd.cpu(), k)
    assert torch.equal(vec_d.cpu(), vec_r)
    assert int(vec_d.sum().item()) == k
    # explicit ties
    s = torch.tensor([1.0, 3.0, 3.0, 0.0, 3.0, -1.0], device="cuda")
    v, idx = gnn.topk_vec(s, 3)
    assert idx.cpu().tolist() == [1, 2, 4] and v.cpu().tolist() == [0, 1, 1, 0, 1, 0]


def test_fullaggnet_forward(torch_cuda, oracle):
    """FullAggNet.forward on the device: k seeds, every reachable node in one aggregate, and P =
    PNet(graph_from_matrix(A, Agg)) Agg against the oracle's PNet on the device's aggregates."""
    torch = torch_cuda
    from mlamg import gnn
    from oracle import gnn_ref
    torch.manual_seed(2)
    net = gnn.FullAggNet(dim=64, num_conv=2, iterations=2).cuda()
    A = _A(14)
    n = A.shape[0]
    agg, P, C, top_k, scores = net.forward(A, 0.1)
    k = int(np.ceil(0.1 * n))
    assert agg.shape == (n, k) and P.shape == (n, k) and len(top_k) == k
    assert torch.equal(torch.nonzero(scores == 1).reshape(-1), top_k)
    Agg = sp.csr_matrix((agg.values().cpu().numpy(), agg.indices().cpu().numpy()), shape=(n, k))
    assert np.all(np.diff(Agg.indptr) <= 1)
    # the aggregates are the device Bellman-Ford's over the CNet weights from the seeds
    Cs = sp.csr_matrix((C.values().cpu().numpy(), C.indices().cpu().numpy()), shape=(n, n))
    _, lab = oracle.canon_bellman_ford(Cs.astype(np.float64), top_k.cpu().numpy())
    pos = {int(s): t for t, s in enumerate(top_k.cpu().numpy())}
    col = np.array([pos.get(int(l), -1) if l >= 0 else -1 for l in lab])
    rows = np.nonzero(col >= 0)[0]
    Agg_ref = sp.csr_matrix((np.ones(len(rows)), (rows, col[rows])), shape=(n, k))
    assert (abs(Agg - Agg_ref) > 0).nnz == 0
    # P = P_hat Agg with P_hat the device PNet's edge values on graph_from_matrix(A, Agg)
    _, pe = net.PNet.run(gnn.Graph(A, agg=Agg))
    P_hat = sp.csr_matrix((pe.reshape(-1).double().cpu().numpy(), A.indices, A.indptr),
                          shape=A.shape)
    P_ref = (P_hat @ Agg).toarray().astype(np.float32)
    Pd = sp.csr_matrix((P.values().cpu().numpy(), P.indices().cpu().numpy()),
                       shape=(n, k)).toarray()
    assert np.abs(Pd - P_ref).max() <= 1e-6 * max(np.abs(P_ref).max(), 1e-30)
