"""GPU: the partition maps built with torch ops on the device operators
(partition.build_levels_torch, the distributed executor's default) equal the numpy reference
build (partition.build_levels) on a hierarchy built on the device: the device transpose R is
scipy's P.T.tocsr() order, every local operator's arrays and every halo match, worlds 2-8."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hier():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mlamg import problems
    from mlamg.hierarchy import Hierarchy
    A = problems.poisson_3d_7pt(36)
    return Hierarchy.build(A, alpha=0.1, max_coarse=500, aggregation="reference",
                           coarse_order="sorted")


def test_device_partition_equals_numpy(hier):
    from mlamg import partition
    from test_partition_torch import _same_csr, _same_halo
    H = hier
    K = len(H.levels)
    As = [H.levels[l].A.to_scipy() for l in range(K)]
    Ps = [H.levels[l].P.to_scipy() for l in range(K)]
    seeds = [H.levels[l].seeds for l in range(K)]

    def tc(M):
        return partition.TCSR(*M.to_torch(), M.shape)
    At = [tc(H.levels[l].A) for l in range(K)]
    Pt = [tc(H.levels[l].P) for l in range(K)]
    Rt = [tc(H.levels[l].R) for l in range(K)]
    for l in range(K):  # the device transpose keeps every row's columns ascending
        R = Ps[l].T.tocsr()
        R.sort_indices()
        _same_csr(Rt[l], R)
    for world in (2, 3, 8):
        for rank in range(world):
            ref = partition.build_levels(As, Ps, seeds, world, rank)
            got = partition.build_levels_torch(At, Pt, Rt, seeds, world, rank)
            for g, h in zip(ref, got):
                assert g["c_ranges"] == h["c_ranges"]
                assert h["A_loc"].col.is_cuda
                for key in ("A_loc", "R_own", "P_loc"):
                    _same_csr(h[key], g[key])
                for key in ("halo_x", "halo_r", "halo_p"):
                    _same_halo(h[key], g[key])
