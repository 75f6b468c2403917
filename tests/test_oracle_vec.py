"""CPU: the oracle's restatement of the device CSR-vector summation order (oracle.c vec_matvec),
checked against a literal Python transcription of the order documented in spmv.hip."""
import numpy as np
import pytest
import scipy.sparse as sp


def _literal(A, x, vw):
    g = min(vw, 64)
    y = np.empty(A.shape[0])
    for i in range(A.shape[0]):
        a, b = A.indptr[i], A.indptr[i + 1]
        part = [0.0] * vw
        for l in range(vw):
            s = 0.0
            for k in range(a + l, b, vw):
                s += A.data[k] * x[A.indices[k]]
            part[l] = s
        off = g // 2
        while off:
            part = [part[l] + part[(l & ~(g - 1)) | ((l & (g - 1)) ^ off)] for l in range(vw)]
            off //= 2
        r = part[0]
        for w in range(1, vw // g):
            r += part[w * g]
        y[i] = r
    return y


@pytest.mark.parametrize("vw", (4, 64, 128, 512))
def test_vec_matvec_order(oracle, vw):
    rs = np.random.RandomState(vw)
    A = sp.random(40, 3000, density=0.3, random_state=rs, format="csr")
    A.data -= 0.5
    x = rs.randn(3000)
    y = oracle.vec_matvec(A, x, vw)
    assert np.array_equal(y, _literal(A, x, vw))
    assert np.allclose(y, A @ x, rtol=1e-12, atol=1e-12)
    with pytest.raises(ValueError):
        oracle.vec_matvec(A, x, 1024)
