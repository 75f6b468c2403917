"""GPU, one rank: the RCCL distributed executor (csrc/comm.hip) with 1..all levels partitioned
reproduces the single-GPU V-cycle bit for bit (the multi-rank maps are covered by the gloo
emulation in test_distributed_gloo.py)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def setup():
    from mlamg import problems
    from mlamg.hierarchy import Hierarchy
    from mlamg.distributed import Comm
    A = problems.poisson_3d_7pt(24)
    H = Hierarchy.build(A, alpha=0.1, max_coarse=60)
    assert H.n_levels >= 3
    return A, H, Comm(1, 0)


@pytest.mark.parametrize("min_rows", [10**9, 1000, 0])
def test_distributed_single_rank_bitwise(setup, min_rows):
    from mlamg.distributed import DistributedHierarchy
    A, H, comm = setup
    n = A.shape[0]
    D = DistributedHierarchy(H, comm, min_rows=min_rows, A_host=A)
    if min_rows == 0:
        assert D.K == len(H.levels)
    if min_rows == 10**9:
        assert D.K == 1
    x0 = np.random.RandomState(0).randn(n)
    b = torch.as_tensor(np.random.RandomState(1).randn(n)).cuda()
    x = torch.as_tensor(x0).cuda()
    h_ref = H.cycle(b, x, 6, use_graph=False)
    for coarse_graph, cycle_graph in ((False, False), (True, False), (True, True), (False, True)):
        D.set_coarse_graph(coarse_graph)
        D.set_cycle_graph(cycle_graph)
        for rep in range(2):  # the second call replays the captured cycle
            xe = D.new_x(torch.as_tensor(x0))
            h = D.cycle(b, xe, 6)
            assert torch.equal(xe[:n], x), f"K={D.K} graphs={coarse_graph},{cycle_graph}"
            np.testing.assert_allclose(h, h_ref, rtol=1e-12, atol=0)


def test_distributed_tolerance_stop(setup):
    from mlamg.distributed import DistributedHierarchy
    A, H, comm = setup
    n = A.shape[0]
    D = DistributedHierarchy(H, comm, min_rows=0, A_host=A)
    b = torch.as_tensor(np.random.RandomState(2).randn(n)).cuda()
    x = torch.zeros(n, dtype=torch.float64, device="cuda")
    h_ref = H.cycle(b, x, 50, tol=1e-6 * float(torch.linalg.norm(b)), use_graph=False)
    for cycle_graph in (False, True):
        D.set_cycle_graph(cycle_graph)
        xe = D.new_x(torch.zeros(n, dtype=torch.float64))
        h = D.cycle(b, xe, 50, tol=1e-6 * float(torch.linalg.norm(b)))
        assert len(h) == len(h_ref) < 50
        assert torch.equal(xe[:n], x)


def test_finalize_replicated_matches_full_build():
    """bench.py's N > 1 setup: every rank builds with finalize=False, rank 0 autotunes and
    broadcasts the formats, every rank then builds its coarse solver (finalize_replicated) —
    the cycle is bitwise that of a hierarchy built in one call (world 1 here; the broadcast is
    the same object list sync_formats used)."""
    from mlamg import problems
    from mlamg.distributed import finalize_replicated
    from mlamg.hierarchy import Hierarchy
    A = problems.poisson_3d_7pt(24)
    n = A.shape[0]
    H1 = Hierarchy.build(A, alpha=0.1, max_coarse=60, aggregation="reference",
                         coarse_order="sorted")
    H2 = Hierarchy.build(A, alpha=0.1, max_coarse=60, aggregation="reference",
                         coarse_order="sorted", finalize=False)
    assert H2.handle is None
    finalize_replicated(H2, 1, 0)
    x0 = np.random.RandomState(0).randn(n)
    b = torch.as_tensor(np.random.RandomState(1).randn(n)).cuda()
    x1, x2 = torch.as_tensor(x0).cuda(), torch.as_tensor(x0).cuda()
    h1 = H1.cycle(b, x1, 5)
    h2 = H2.cycle(b, x2, 5)
    assert np.array_equal(h1, h2) and torch.equal(x1, x2)
