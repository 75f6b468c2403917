"""GPU: many independent reference-style amg_2_v solves at once (mlamg.multigrid.amg_2_v_batch —
the reference's per-grid task farm, ns/parallel/pool.py, as host threads with one HIP stream each
on one GPU). Every result must equal the sequential call bit for bit: concurrent solves share no
buffer (per-thread scratch, per-handle work buffers)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _problems(ml, oracle, count):
    out = []
    for i in range(count):
        m = 24 + 4 * (i % 7)
        A = ml.problems.poisson_2d_5pt(m)
        Agg = ml.problems.box_aggregates_2d(m, m, 3 if i % 2 else 2)
        P, _ = oracle.smoothed_aggregation_jacobi(A, Agg, omega=2.0 / 3.0)
        x0 = np.random.RandomState(i).randn(A.shape[0])
        b = np.random.RandomState(100 + i).randn(A.shape[0]) if i % 3 == 0 else np.zeros(A.shape[0])
        out.append((A, P, b, x0))
    return out


@pytest.mark.parametrize("smoother", ("gauss_seidel", "jacobi"))
def test_batch_equals_sequential(oracle, smoother):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mlamg.multigrid
    import mlamg.problems
    import mlamg as ml
    probs = _problems(ml, oracle, 14)
    seq = [ml.multigrid.amg_2_v(A, P, b, x.copy(), res_tol=1e-10, smoother=smoother)
           for A, P, b, x in probs]
    bat = ml.multigrid.amg_2_v_batch([(A, P, b, x.copy()) for A, P, b, x in probs], workers=6,
                                     res_tol=1e-10, smoother=smoother)
    assert len(bat) == len(seq)
    for i, ((xs, cs, es, its), (xb, cb, eb, itb)) in enumerate(zip(seq, bat)):
        assert its == itb and np.array_equal(es, eb), i
        assert np.array_equal(xs, xb), i
        assert cs == cb or (np.isnan(cs) and np.isnan(cb)), i
