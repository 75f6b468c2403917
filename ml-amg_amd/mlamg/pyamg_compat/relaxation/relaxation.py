"""pyamg.relaxation.relaxation (4.x) subset: gauss_seidel, as ns/lib/multigrid.py:175,184 call
it (in place on x, forward lexicographic sweeps), on the device (csrc/gs.hip, bitwise the
sequential sweep)."""
import numpy as np
import scipy.sparse as sp


def gauss_seidel(A, x, b, iterations=1, sweep='forward'):
    """x is overwritten in place, like pyamg's amg_core kernel. Only CSR A and the forward sweep
    (what the reference uses) are provided; other sweeps raise NotImplementedError."""
    from ...multigrid import gauss_seidel as _gs
    if sweep != 'forward':
        raise NotImplementedError("only sweep='forward' (the reference's) is provided")
    if not sp.isspmatrix_csr(A):
        raise TypeError('expected csr_matrix')
    if iterations < 1:
        return
    out = _gs(A, np.ravel(b), np.ravel(x), nu=int(iterations))
    x[...] = np.reshape(out, np.shape(x))
