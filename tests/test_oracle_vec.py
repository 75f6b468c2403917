"""CPU: the oracle's restatement of the device CSR-vector summation order (oracle.c vec_matvec),
checked against a literal Python transcription of the canonical order documented in spmv.hip,
and the kernel's per-width schedule shown to compute that same order for every width."""
import numpy as np
import pytest
import scipy.sparse as sp


def _butterfly(a):
    off = 32
    while off:
        a = [a[l] + a[l ^ off] for l in range(64)]
        off //= 2
    return a[0]


def _literal(A, x):
    """The canonical order as documented in spmv.hip (512 virtual lanes)."""
    y = np.empty(A.shape[0])
    for i in range(A.shape[0]):
        a, b = A.indptr[i], A.indptr[i + 1]
        part = []
        for v in range(512):
            s = 0.0
            for k in range(a + v, b, 512):
                s += A.data[k] * x[A.indices[k]]
            part.append(s)
        r = None
        for w in range(8):
            ws = _butterfly(part[64 * w:64 * w + 64])
            r = ws if r is None else r + ws
        y[i] = r
    return y


def _physical(A, x, Q):
    """What k_csr_vcan<Q> computes, step for step: physical wave p of the row holds the virtual
    waves p + Q j in accumulators, Q stripes of 512 entries per step."""
    J = 8 // Q
    y = np.empty(A.shape[0])
    for i in range(A.shape[0]):
        a, b = A.indptr[i], A.indptr[i + 1]
        ws = [None] * 8
        for p in range(Q):
            acc = [[0.0] * 64 for _ in range(J)]
            for base in range(a, b, 512 * Q):
                for t in range(Q):
                    for j in range(J):
                        for lane in range(64):
                            e = base + 512 * t + 64 * (p + Q * j) + lane
                            if e < b:
                                acc[j][lane] += A.data[e] * x[A.indices[e]]
            for j in range(J):
                ws[p + Q * j] = _butterfly(acc[j])
        r = ws[0]
        for w in range(1, 8):
            r += ws[w]
        y[i] = r
    return y


def test_vec_matvec_canonical_order(oracle):
    rs = np.random.RandomState(4)
    A = sp.random(12, 3000, density=0.4, random_state=rs, format="csr")
    A.data -= 0.5
    x = rs.randn(3000)
    y = oracle.vec_matvec(A, x)
    assert np.array_equal(y, _literal(A, x))
    assert np.allclose(y, A @ x, rtol=1e-12, atol=1e-12)
    for vw in (64, 128, 256, 512):
        assert np.array_equal(oracle.vec_matvec(A, x, vw), y)
    with pytest.raises(ValueError):
        oracle.vec_matvec(A, x, 32)


@pytest.mark.parametrize("Q", (1, 2, 4, 8))
def test_every_width_computes_the_canonical_order(oracle, Q):
    """The kernel's per-width schedule (Q waves per row, 8/Q accumulators per lane, Q stripes
    per step) reproduces the canonical order bit for bit — the width is a timing choice only."""
    rs = np.random.RandomState(10 + Q)
    lens = rs.randint(0, 2600, 6)
    lens[0] = 0
    lens[1] = 1
    indptr = np.concatenate([[0], np.cumsum(lens)])
    indices = np.concatenate([rs.randint(0, 4000, l) for l in lens]).astype(np.int32)
    A = sp.csr_matrix((rs.randn(indptr[-1]), indices, indptr), shape=(6, 4000))
    x = rs.randn(4000)
    assert np.array_equal(_physical(A, x, Q), oracle.vec_matvec(A, x))


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
