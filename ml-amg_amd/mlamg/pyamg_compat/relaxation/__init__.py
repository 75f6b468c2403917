"""pyamg.relaxation (4.x) subset."""
from . import relaxation  # noqa: F401
