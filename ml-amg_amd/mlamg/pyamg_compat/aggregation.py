"""pyamg.aggregation (4.x) subset: lloyd_aggregation, on the device (mlamg.graph)."""
from ..graph import pyamg_lloyd_aggregation as lloyd_aggregation  # noqa: F401
