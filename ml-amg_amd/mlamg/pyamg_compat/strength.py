"""pyamg.strength (4.x) subset: evolution_strength_of_connection at the reference's arguments,
on the device (mlamg.strength; parity unpinned against pyamg itself), and
symmetric_strength_of_connection (the smoothed_aggregation_solver default, csrc/sa.hip)."""
import scipy.sparse as sp

from ..strength import evolution_strength_of_connection  # noqa: F401


def symmetric_strength_of_connection(A, theta=0):
    """Diagonal and a_ij with a_ij^2 >= theta^2 |a_ii a_jj| kept, |.| / row max (CSR in/out)."""
    import ctypes
    from .._lib import call, stream_ptr
    from ..sparse import DeviceCSR
    if theta < 0:
        raise ValueError("expected a positive theta")
    if not sp.isspmatrix_csr(A):
        raise TypeError("expected csr_matrix or bsr_matrix")
    Ad = DeviceCSR.from_scipy(A)
    h = ctypes.c_void_p()
    call("mlamg_symmetric_strength", Ad.handle, float(theta), ctypes.byref(h), stream_ptr())
    return DeviceCSR(h).to_scipy()
