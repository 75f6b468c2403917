"""CPU: the vectorised partition build (mlamg.partition.build_levels_torch, what the distributed
executor runs on the operators' device arrays) gives exactly the maps of the numpy reference build
(partition.build_levels): row and coarse ranges, every local operator's arrays (stored order,
renumbered columns), every halo's ghosts, owners and send lists, at worlds 1-6 on every rank."""
import numpy as np
import pytest


def _levels(kind):
    from mlamg import problems
    from oracle import restated as orc
    A = {"3d": lambda: problems.poisson_3d_7pt(12),
         "jump": lambda: problems.jump_2d(40, np.array([[0.3, 0.4, 1e-2], [0.7, 0.6, 1e2]])),
         "aniso": lambda: problems.random_coeff_3d_7pt(10, seed=2)}[kind]()
    levels, _ = orc.build_hierarchy(A, alpha=0.1, seed=0, sort_seeds=True, max_coarse=30,
                                    omegas=[0.61, 0.63, 0.65, 0.67, 0.69, 0.7])
    return levels


def _same_csr(T, S):
    S = S.tocsr()
    U = T.to_scipy()
    assert U.shape == S.shape
    assert np.array_equal(U.indptr.astype(np.int64), S.indptr.astype(np.int64))
    assert np.array_equal(U.indices.astype(np.int64), S.indices.astype(np.int64))
    assert np.array_equal(U.data, S.data)


def _same_halo(h, g):
    if g is None:
        assert h is None
        return
    assert h.n_own == g.n_own and h.neighbors == g.neighbors
    assert np.array_equal(np.asarray(h.ghosts, np.int64), np.asarray(g.ghosts, np.int64))
    assert np.array_equal(h.ghost_owner, g.ghost_owner)
    assert h.recv_counts == g.recv_counts and h.send_counts == g.send_counts
    assert np.array_equal(h.send_idx, g.send_idx)


@pytest.mark.parametrize("kind", ("3d", "jump", "aniso"))
def test_torch_partition_equals_numpy(oracle, kind):
    from mlamg import partition
    levels = _levels(kind)
    for K in (1, 2, len(levels)):
        As = [levels[l]["A"] for l in range(K)]
        Ps = [levels[l]["P"] for l in range(K)]
        seeds = [levels[l]["seeds"] for l in range(K)]
        T = partition.TCSR.from_scipy
        At = [T(M) for M in As]
        Pt = [T(M) for M in Ps]
        Rt = []
        for M in Ps:
            R = M.T.tocsr()
            R.sort_indices()
            Rt.append(T(R))
        for world in (1, 2, 3, 6):
            for rank in range(world):
                ref = partition.build_levels(As, Ps, seeds, world, rank)
                got = partition.build_levels_torch(At, Pt, Rt, seeds, world, rank)
                assert len(ref) == len(got)
                for g, h in zip(ref, got):
                    for key in ("lo", "hi", "n", "nc", "c_lo", "c_hi", "c_ranges", "ranges"):
                        assert g[key] == h[key], (kind, K, world, rank, key)
                    for key in ("A_loc", "R_own", "P_loc"):
                        _same_csr(h[key], g[key])
                    for key in ("halo_x", "halo_r", "halo_p"):
                        _same_halo(h[key], g[key])


def test_torch_interior_split_equals_numpy():
    from mlamg import partition, problems
    A = problems.poisson_3d_7pt(14).tocsr()
    n = A.shape[0]
    for world in (2, 3, 4):
        for lo, hi in partition.row_ranges(n, world):
            xg = partition._ghost_sets(A[lo:hi].indices, lo, hi)
            A_loc = partition._remap(A[lo:hi], lo, hi, xg)
            for frac in (0.3, 0.5, 0.9):
                assert (partition.interior_split_torch(partition.TCSR.from_scipy(A_loc),
                                                       hi - lo, frac)
                        == partition.interior_split(A_loc, hi - lo, frac))
