"""CPU: mlamg.gnn modules hold their parameters like the reference's (ns/model/agg_interp.py
FullAggNet, torch_geometric 2.x TAGConv / NNConv attribute names), so a reference state_dict
loads into them. No GPU call (module construction only)."""
import pytest


def test_fullaggnet_state_dict_layout():
    torch = pytest.importorskip("torch")
    from mlamg import gnn
    net = gnn.FullAggNet(dim=64, num_conv=2, iterations=4)
    sd = net.state_dict()
    shapes = {k: tuple(v.shape) for k, v in sd.items()}
    # MPNN (agg_interp.py:80-121)
    assert shapes["PNet.node_conv_in.nn.1.weight"] == (4, 2)        # Linear(input_edge_features, 4)
    assert shapes["PNet.node_conv_in.nn.5.weight"] == (64, 16)      # Linear(16, 1 * dim)
    assert shapes["PNet.node_conv_in.lin.weight"] == (64, 1)        # root weight
    assert shapes["PNet.node_conv_in.bias"] == (64,)
    assert shapes["PNet.edge_conv_in.edge_mlp.0.weight"] == (64, 130)  # dim*2 + 2
    assert shapes["PNet.edge_conv_in.edge_mlp.2.weight"] == (64,)      # LayerNorm
    assert shapes["PNet.node_convs.3.nn.5.weight"] == (4096, 16)       # Linear(16, dim*dim)
    assert "PNet.node_convs.4.nn.5.weight" not in shapes               # 4 internal convs
    assert shapes["CNet.node_convs.4.nn.5.weight"] == (4096, 16)       # CNet: 5
    assert shapes["CNet.edge_conv_in.edge_mlp.0.weight"] == (64, 129)  # dim*2 + 1
    assert shapes["CNet.node_conv_out.nn.5.weight"] == (64, 16)        # Linear(16, dim * 1)
    assert shapes["CNet.edge_conv_out.edge_mlp.3.weight"] == (1, 64)
    # AggNet (agg_interp.py:144-241): 4 layers of 2 TAGConvs (K = 3: 4 lins) and 5-layer MLPs
    assert shapes["AggNet.layers.3.ncs.0.lins.3.weight"] == (64, 1)
    assert shapes["AggNet.layers.3.ncs.1.lins.0.weight"] == (64, 64)
    assert shapes["AggNet.layers.0.ncs.1.bias"] == (64,)
    assert shapes["AggNet.layers.0.fcs.0.8.weight"] == (64, 64)
    assert shapes["AggNet.layers.0.fcs.1.8.weight"] == (1, 64)
    assert "AggNet.layers.4.ncs.0.bias" not in shapes
    # a state dict round trip
    net2 = gnn.FullAggNet(dim=64, num_conv=2, iterations=4)
    net2.load_state_dict(sd)
