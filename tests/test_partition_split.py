"""CPU: the row split behind the halo / interior overlap (mlamg.partition.interior_split,
SURVEY.md §8e): the longest run of rows reading only owned columns, even-aligned ends."""
import numpy as np
import scipy.sparse as sp

from mlamg import partition, problems


def _split_check(M, n_owned, cut):
    lo, hi = cut
    assert lo % 2 == 0 and hi % 2 == 0 and 0 <= lo < hi <= M.shape[0]
    mid = M[lo:hi]
    assert mid.nnz == 0 or mid.indices.max() < n_owned


def test_slab_split_c4_like():
    """z-slab partition of a 3D 7-point operator: the interior is every plane but the slab's
    first and last (the first rank has no lower neighbour)."""
    m = 12
    A = problems.poisson_3d_7pt(m).tocsr()
    n = A.shape[0]
    world = 3
    ranges = partition.row_ranges(n, world)
    for r, (lo, hi) in enumerate(ranges):
        xg = partition._ghost_sets(A[lo:hi].indices, lo, hi)
        A_loc = partition._remap(A[lo:hi], lo, hi, xg)
        cut = partition.interior_split(A_loc, hi - lo)
        assert cut is not None
        _split_check(A_loc, hi - lo, cut)
        plane = m * m
        want_lo = 0 if r == 0 else plane
        want_hi = (hi - lo) if r == world - 1 else (hi - lo) - plane
        # even rounding moves at most one row into each boundary part
        assert want_lo <= cut[0] <= want_lo + 1 and want_hi - 1 <= cut[1] <= want_hi


def test_split_none_cases():
    A = problems.poisson_2d_5pt(8).tocsr()
    assert partition.interior_split(A, A.shape[1]) is None           # no ghost column
    B = sp.csr_matrix(np.ones((6, 8)))
    assert partition.interior_split(B, 4) is None                      # every row reads a ghost
    assert partition.interior_split(sp.csr_matrix((0, 4)), 4) is None  # no rows


def test_split_picks_longest_run_and_min_frac():
    n, n_owned = 40, 40
    rows, cols = [], []
    for i in range(n):
        rows.append(i)
        cols.append(i)
    for i in (3, 10, 11, 30):           # rows reading a ghost column
        rows.append(i)
        cols.append(n_owned + 1)
    M = sp.csr_matrix((np.ones(len(rows)), (rows, cols)), shape=(n, n_owned + 2))
    cut = partition.interior_split(M, n_owned, min_frac=0.3)
    assert cut == (12, 30)               # run [12, 30): 18 rows, even ends
    _split_check(M, n_owned, cut)
    assert partition.interior_split(M, n_owned, min_frac=0.5) is None
