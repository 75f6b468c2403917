"""pyamg.relaxation.relaxation (4.x) subset on the device (csrc/gs.hip, bitwise the sequential
sweeps): gauss_seidel as ns/lib/multigrid.py:175,184 call it, and block_gauss_seidel with 1 x 1
blocks (the smoother of pyamg's smoothed_aggregation_solver). In place on x."""
import numpy as np
import scipy.sparse as sp


def _sweep(A, x, b, iterations, sweep, block):
    import torch
    from ...multigrid import GaussSeidel
    from ...sparse import DeviceCSR
    if sweep not in ("forward", "backward", "symmetric"):
        raise ValueError("valid sweep directions are 'forward', 'backward', and 'symmetric'")
    if not sp.isspmatrix_csr(A):
        raise TypeError("expected csr_matrix")
    if iterations < 1:
        return
    G = GaussSeidel(DeviceCSR.from_scipy(A), sweep, block=block)
    dev = torch.device("cuda", torch.cuda.current_device())
    xd = torch.as_tensor(np.ascontiguousarray(np.ravel(x), dtype=np.float64)).to(dev)
    bd = torch.as_tensor(np.ascontiguousarray(np.ravel(b), dtype=np.float64)).to(dev)
    G.sweep(xd, bd, int(iterations))
    x[...] = np.reshape(xd.cpu().numpy(), np.shape(x))


def gauss_seidel(A, x, b, iterations=1, sweep='forward'):
    """pyamg gauss_seidel (CSR): x_i = (b_i - sum_{j != i} a_ij x_j) / a_ii in sweep order."""
    _sweep(A, x, b, iterations, sweep, False)


def block_gauss_seidel(A, x, b, iterations=1, sweep='forward', blocksize=1, Dinv=None):
    """pyamg block_gauss_seidel for CSR A with 1 x 1 blocks (Dinv = 1 / a_ii, 0 for a zero
    diagonal); other block sizes or a given Dinv raise NotImplementedError."""
    if blocksize not in (None, 1) or Dinv is not None:
        raise NotImplementedError("1 x 1 blocks with pyamg's own Dinv only")
    _sweep(A, x, b, iterations, sweep, True)
