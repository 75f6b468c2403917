"""pyamg.graph (4.x) subset: asgraph, lloyd_cluster, bellman_ford, on the device (mlamg.graph)."""
from ..graph import _asgraph as asgraph  # noqa: F401
from ..graph import bellman_ford, lloyd_cluster  # noqa: F401
