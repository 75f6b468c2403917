"""pyamg.strength (4.x) subset: evolution_strength_of_connection at the reference's arguments,
on the device (mlamg.strength; parity unpinned against pyamg itself)."""
from ..strength import evolution_strength_of_connection  # noqa: F401
