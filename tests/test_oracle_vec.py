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


def test_omp_baseline_cycle_matches_oracle_cycle():
    """bench.py's parallel CPU baseline (oracle/omp_cycle.c via restated.vcycle_omp) runs the same
    cycle as the scipy restatement: histories agree to rounding (dense inverse vs SuperLU coarse
    solve, parallel norm)."""
    import numpy as np
    import scipy.sparse as sp
    from mlamg import problems
    from oracle import restated as orc
    A = problems.poisson_3d_7pt(20)
    levels, Ac = orc.build_hierarchy(A, alpha=0.1, max_coarse=60)
    for L in levels:
        L["Dw"] = orc.mlamg_dinv(L["A"])
        L["d"] = L["Dw"].diagonal()
    n = A.shape[0]
    x0 = np.random.RandomState(0).randn(n)
    b = np.random.RandomState(1).randn(n)
    _, h_ref = orc.vcycle_solve(levels, Ac, b, x0, 5)
    Ainv = np.linalg.inv(Ac.toarray())
    _, h = orc.vcycle_omp(levels, Ainv, b, x0, 5, threads=4)
    np.testing.assert_allclose(h, h_ref, rtol=1e-10)
