"""GPU, one process: every rank's LOCAL operators of the multi-GPU partition (A_loc with ghost
columns, P_loc over owned + x-ghost rows, R_own with r-ghost columns — mlamg.partition.build_levels,
the maps csrc/comm.hip runs on) through every SpMV storage format, bitwise against scipy's
csr_matvec order (the oracle's vector order for 'vector').

RCCL refuses two ranks on one GPU, so the driver's 8-GPU run is the first to execute the real
exchange; this test covers what differs per rank on the device — ghost-extended column spaces,
the offsets the rowpat/sell_dict/sorted encoders see at slab boundaries, and the format
DistributedHierarchy picks for each local operator — for world sizes 2, 3 and 8.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

FORMATS = (("csr_stream", 0), ("sell", 1), ("sell", 512), ("sorted", 0), ("sell_dict", 1),
           ("rowpat", 0), ("long", 0), ("vector", 64), ("vector", 256))


@pytest.fixture(scope="module")
def hier():
    from mlamg import problems
    from mlamg.hierarchy import Hierarchy
    A = problems.poisson_3d_7pt(36)
    H = Hierarchy.build(A, alpha=0.1, max_coarse=200)
    assert H.n_levels >= 3
    return A, H


def _check_formats(M_host, label, oracle, required=()):
    from mlamg import _lib
    from mlamg.sparse import DeviceCSR
    M = DeviceCSR.from_scipy(M_host, check=False)
    x = np.random.RandomState(M_host.nnz % 1000).randn(M_host.shape[1])
    xd = torch.as_tensor(x).cuda()
    ran = []
    for fmt, arg in FORMATS:
        try:
            M.set_format(fmt, arg)
        except _lib.MlamgError as e:
            assert e.code == _lib.MLAMG_EUNSUPPORTED, f"{label} {fmt}: {e}"
            assert fmt not in required, f"{label}: {fmt} refused"
            continue
        y = M.matvec(xd).cpu().numpy()
        ref = oracle.vec_matvec(M_host, x, arg) if fmt == "vector" else oracle.csr_matvec(M_host, x)
        assert np.array_equal(y, ref), f"{label} {fmt}/{arg}: max |d| {np.abs(y - ref).max()}"
        ran.append(fmt)
    return ran


@pytest.mark.parametrize("world", (2, 3, 8))
def test_local_operators_every_format(hier, oracle, world):
    from mlamg import partition
    A, H = hier
    K = len(H.levels)
    As = [A] + [H.levels[l].A.to_scipy() for l in range(1, K)]
    Ps = [H.levels[l].P.to_scipy() for l in range(K)]
    seeds = [H.levels[l].seeds for l in range(K)]
    for rank in range(world):
        parts = partition.build_levels(As, Ps, seeds, world, rank)
        for p in parts:
            tag = f"world {world} rank {rank} level {p['level']}"
            ran = _check_formats(p["A_loc"], f"{tag} A_loc", oracle,
                                 required=("csr_stream", "sorted", "rowpat") if p["level"] == 0 else ())
            assert "csr_stream" in ran
            _check_formats(p["P_loc"], f"{tag} P_loc", oracle)
            _check_formats(p["R_own"], f"{tag} R_own", oracle)


@pytest.mark.parametrize("world", (2, 8))
def test_local_rowpat_attached_dinv(hier, world):
    """The fine local operator keeps the stencil's row-pair patterns across the ghost columns
    (constant ghost offsets on z-slab boundaries), so DistributedHierarchy can attach the
    Jacobi weights to it exactly as on one GPU."""
    from mlamg import partition
    from mlamg.sparse import DeviceCSR
    A, H = hier
    for rank in range(world):
        p = partition.build_levels([A], [H.levels[0].P.to_scipy()], [H.levels[0].seeds], world,
                                   rank)[0]
        M = DeviceCSR.from_scipy(p["A_loc"], check=False).set_format("rowpat")
        dinv = H.levels[0].dinv[p["lo"]:p["hi"]].clone()
        assert M.attach_dinv(dinv), f"world {world} rank {rank}: weights not pattern-constant"


@pytest.mark.slow
def test_c4_slab_partition_level0(oracle):
    """The bench's C4 fine level (216^3) split over 8 GPUs: every rank's local operator is
    accepted by the row-pair format and reproduces scipy's rows bitwise."""
    import scipy.sparse as sp
    from mlamg import partition, problems
    from mlamg.sparse import DeviceCSR
    A = problems.poisson_3d_7pt(216)
    ranges = partition.row_ranges(A.shape[0], 8)
    his = np.array([h for _, h in ranges])
    for rank in (0, 3, 7):
        lo, hi = ranges[rank]
        blk = A[lo:hi]
        cols = np.unique(blk.indices)
        ghosts = cols[(cols < lo) | (cols >= hi)]
        loc = partition._remap(blk, lo, hi, ghosts)
        assert set(np.unique(partition.owner_of(ghosts, his))) <= {rank - 1, rank + 1}
        M = DeviceCSR.from_scipy(loc, check=False).set_format("rowpat")
        x = np.random.RandomState(rank).randn(loc.shape[1])
        y = M.matvec(torch.as_tensor(x).cuda()).cpu().numpy()
        assert np.array_equal(y, oracle.csr_matvec(sp.csr_matrix(loc), x)), f"rank {rank}"


@pytest.mark.parametrize("seed", (0, 1))
def test_rowpat_rows_in_stored_not_ascending_order(oracle, seed):
    """rowpat on rows whose stored order is not ascending in column (a fixed shuffle of a 2D
    stencil's entries in every row, plus rows of the shuffled and the sorted kind mixed): the
    pair merge keeps each row's stored order, so results stay bitwise scipy's."""
    import scipy.sparse as sp
    from mlamg import problems
    from mlamg.sparse import DeviceCSR
    A = problems.poisson_2d_5pt(40).tocsr()
    rs = np.random.RandomState(seed)
    ip, ij, ax = A.indptr, A.indices.copy(), A.data.copy()
    perm5 = rs.permutation(5)
    for r in range(A.shape[0]):
        a, b = ip[r], ip[r + 1]
        if b - a == 5 and (r % 7 != 3):
            ij[a:b] = ij[a:b][perm5]
            ax[a:b] = ax[a:b][perm5]
    M_host = sp.csr_matrix((ax, ij, ip.copy()), shape=A.shape)
    M = DeviceCSR.from_scipy(M_host, check=False).set_format("rowpat")
    x = rs.randn(A.shape[1])
    y = M.matvec(torch.as_tensor(x).cuda()).cpu().numpy()
    assert np.array_equal(y, oracle.csr_matvec(M_host, x))


@pytest.mark.parametrize("m,world", [(48, 3), (216, 8)])
def test_slab_local_operators_take_uniform_form(m, world):
    """Row-partitioned 3-D 7-point slabs: a middle or last rank's local operator reaches its
    ghost planes at offsets of their own (+n_own below, +2F above), so the uniform row-pair form
    takes them as alternate offsets of the two far slots on the first / last plane's pairs
    (build_rowpat). Every rank's operator must take the uniform form (its format
    bytes: x, y, one id byte per pair and the mask table) and reproduce the CSR-stream rows
    bitwise."""
    import torch
    from mlamg import partition, problems
    from mlamg.sparse import DeviceCSR
    A = problems.poisson_3d_7pt(m)
    ranges = partition.row_ranges(A.shape[0], world)
    for rank in sorted({0, world // 2, world - 1}):
        lo, hi = ranges[rank]
        blk = A[lo:hi]
        cols = np.unique(blk.indices)
        ghosts = cols[(cols < lo) | (cols >= hi)]
        loc = partition._remap(blk, lo, hi, ghosts)
        M = DeviceCSR.from_scipy(loc, check=False).set_format("rowpat")
        n, mc = loc.shape
        uni_bytes = 8.0 * mc + 8.0 * n + float((n + 1) // 2) + 512.0
        assert M.format_bytes() == uni_bytes, f"rank {rank}: not the uniform form"
        R = DeviceCSR.from_scipy(loc, check=False).set_format("csr_stream")
        x = torch.as_tensor(np.random.RandomState(rank).randn(mc)).cuda()
        assert torch.equal(M.matvec(x), R.matvec(x)), f"rank {rank}"
