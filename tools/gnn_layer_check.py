"""Layer-isolated comparison of the device MPNN (mlamg.gnn) with oracle/gnn_ref.py: every layer
fed the oracle's input at that depth (GPU box: python tools/gnn_layer_check.py)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ml-amg_amd")]
import numpy as np
import torch
import torch.nn.functional as F
from mlamg import gnn, problems
from oracle import gnn_ref

def rel(a, b):
    a = a.detach().cpu().double(); b = b.detach().cpu().double()
    return float((a - b).abs().max() / max(b.abs().max(), 1e-30))

A = problems.jump_2d(24, problems.voronoi_jumps(np.random.RandomState(0)))
torch.manual_seed(0)
net = gnn.MPNN(64, num_internal_conv=5, input_edge_features=1)
netd = gnn.MPNN(64, num_internal_conv=5, input_edge_features=1)
netd.load_state_dict(net.state_dict()); netd = netd.cuda()
g = gnn.Graph(A); rg = gnn_ref.RefGraph(A)
row, col = rg.edge_index
c = lambda t: t.cuda()
x = rg.x.reshape(-1, 1); ea = rg.edge_attr
xn = gnn_ref.instance_norm(x)
x1 = F.relu(gnn_ref.nnconv(net.node_conv_in, xn, rg.edge_index, ea, rg.n)) + x
x1d = netd.node_conv_in.run(g, c(xn), c(ea), act=1, residual=c(x))
print("conv_in", rel(x1d, x1))
ea1 = F.relu(gnn_ref.edge_model(net.edge_conv_in, x1[row], x1[col], ea)) + ea
ea1d = netd.edge_conv_in.run(g, c(x1), c(ea), act=1, residual=c(ea))
print("edge_in", rel(ea1d, ea1))
x, ea = x1, ea1
for i in range(5):
    xn = gnn_ref.instance_norm(x)
    print(" inorm", i, rel(gnn.instance_norm(c(x)), xn), "min channel std", float(x.std(0).min()))
    y = gnn_ref.nnconv(net.node_convs[i], xn, rg.edge_index, ea, rg.n)
    yd = netd.node_convs[i].run(g, c(xn), c(ea), act=0)
    print(" conv", i, rel(yd, y), float(y.abs().max()))
    x = F.relu(y) + x
    ea_new = F.relu(gnn_ref.edge_model(net.edge_convs[i], x[row], x[col], ea)) + ea
    ead = netd.edge_convs[i].run(g, c(x), c(ea), act=1, residual=c(ea))
    print(" edge", i, rel(ead, ea_new))
    ea = ea_new
