"""Row partition of the fine level across GPUs and the halo maps it needs (host logic, numpy).

The reference has no domain decomposition (its only parallelism is a task farm over independent
grids, ns/parallel/pool.py:139-186); this is the north star's fine-level row split (SURVEY.md
§8e). Every rank holds the full hierarchy (setup is deterministic and replicated), so every rank
can derive every other rank's needs locally and no setup communication is required.

Per rank r (rows [lo_r, hi_r) of the fine level, contiguous, near-equal):
  A_loc   rows lo..hi of A0, columns renumbered into x_ext = [owned (hi-lo) | ghosts]
  P_loc   rows lo..hi of P0 (columns = full coarse index space, replicated coarse vector)
  R_own   rows c_lo..c_hi of R0 = P0^T (coarse rows whose aggregate seed lies in [lo, hi)),
          columns renumbered into r_ext = [owned | r-ghosts]
  x halo  ghosts of A_loc: for each neighbour q, ascending global indices owned by q
  r halo  ghosts of R_own, same layout
Ghost order = ascending global index, which is also grouped by owner (owners are contiguous).
Because local rows keep their stored column order, every local product sums exactly like the
single-GPU kernel: the distributed iterate is bitwise the single-GPU iterate.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp


def row_ranges(n, world):
    """Contiguous near-equal row blocks [lo, hi) per rank."""
    base, extra = divmod(n, world)
    sizes = [base + (1 if r < extra else 0) for r in range(world)]
    bounds = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    return [(int(bounds[r]), int(bounds[r + 1])) for r in range(world)]


def owner_of(idx, bounds_hi):
    """Rank owning each global index (bounds_hi = array of hi per rank)."""
    return np.searchsorted(bounds_hi, idx, side="right")


class Halo:
    """Ghost layout of one rank: recv from neighbours into ext[n_own:], send owned entries."""

    def __init__(self, n_own, ghosts, ghost_owner, sends):
        self.n_own = n_own
        self.ghosts = ghosts                # global ids, ascending
        self.ghost_owner = ghost_owner
        self.sends = sends                  # {q: local indices (into owned) to send to q}
        nbrs = sorted(set(np.unique(ghost_owner).tolist()) | set(sends.keys()))
        self.neighbors = nbrs
        self.recv_counts = [int(np.sum(ghost_owner == q)) for q in nbrs]
        self.send_counts = [len(sends.get(q, ())) for q in nbrs]
        self.send_idx = (np.concatenate([np.asarray(sends.get(q, []), np.int32) for q in nbrs])
                         if nbrs else np.zeros(0, np.int32)).astype(np.int32)

    @property
    def n_ghost(self):
        return len(self.ghosts)


def _ghost_sets(M_rows_cols, lo, hi):
    cols = np.unique(M_rows_cols)
    return cols[(cols < lo) | (cols >= hi)]


def _remap(M, lo, hi, ghosts):
    """Renumber columns: owned j -> j - lo, ghost g -> n_own + position(g). Stored order kept."""
    n_own = hi - lo
    cols = M.indices.astype(np.int64)
    out = np.empty_like(cols)
    own = (cols >= lo) & (cols < hi)
    out[own] = cols[own] - lo
    gi = np.searchsorted(ghosts, cols[~own])
    out[~own] = n_own + gi
    return sp.csr_matrix((M.data, out.astype(np.int32), M.indptr.copy()),
                         shape=(M.shape[0], n_own + len(ghosts)))


def _halos(ghosts_all, ranges, r):
    """Halo of rank r in an index space split by `ranges`, given every rank's ghost set."""
    lo, hi = ranges[r]
    his = np.array([h for _, h in ranges], dtype=np.int64)
    sends = {}
    for q in range(len(ranges)):
        if q == r:
            continue
        g = ghosts_all[q]
        need = g[(g >= lo) & (g < hi)]
        if len(need):
            sends[q] = (need - lo).astype(np.int32)
    return Halo(hi - lo, ghosts_all[r], owner_of(ghosts_all[r], his), sends)


def _seed_ranges(seeds, ranges, nc):
    seeds = np.asarray(seeds, dtype=np.int64)
    if len(seeds) != nc or (len(seeds) > 1 and np.any(np.diff(seeds) <= 0)):
        raise ValueError("coarse unknowns must be ordered by strictly increasing seed node")
    b = [int(np.searchsorted(seeds, lo)) for lo, _ in ranges] + [nc]
    return [(b[r], b[r + 1]) for r in range(len(ranges))]


def build_levels(As, Ps, seeds_list, world, rank):
    """Partition maps of the first K = len(As) levels for `rank` (list of per-level dicts).

    Level 0 rows: near-equal contiguous blocks. Level l+1 rows: the coarse unknowns whose seed
    lies in the rank's level-l rows (contiguous because seeds are sorted). P_loc holds the rows
    of P_l for the owned rows AND the x-ghost rows (in x_ext order): prolonging into the ghosts
    locally reproduces their owners' update bit for bit, so no x halo is needed after the coarse
    correction. For l < K-1 its columns are renumbered into [owned level-(l+1) rows | P-ghosts]
    with a halo of x_{l+1}; the last partitioned level's P keeps global columns (the level below
    is replicated on every rank, gathered with an allgatherv of the owned coarse segments).
    """
    K = len(As)
    ranges = row_ranges(As[0].shape[0], world)
    out = []
    for l in range(K):
        A = As[l].tocsr()
        P = Ps[l].tocsr()
        n, nc = A.shape[0], P.shape[1]
        c_ranges = _seed_ranges(seeds_list[l], ranges, nc)
        R = P.T.tocsr()
        R.sort_indices()
        xg, rg, pg, prow = [], [], [], []
        for q, (lo, hi) in enumerate(ranges):
            xg.append(_ghost_sets(A[lo:hi].indices, lo, hi))
            clo, chi = c_ranges[q]
            rg.append(_ghost_sets(R[clo:chi].indices, lo, hi))
            rows = np.concatenate([np.arange(lo, hi), xg[q]]).astype(np.int64)
            prow.append(rows)
            pg.append(_ghost_sets(P[rows].indices, clo, chi))
        lo, hi = ranges[rank]
        clo, chi = c_ranges[rank]
        last = l == K - 1
        d = {
            "level": l, "rank": rank, "world": world, "lo": lo, "hi": hi, "n": n, "nc": nc,
            "c_lo": clo, "c_hi": chi, "c_ranges": c_ranges, "ranges": ranges,
            "A_loc": _remap(A[lo:hi], lo, hi, xg[rank]),
            "R_own": _remap(R[clo:chi], lo, hi, rg[rank]),
            "halo_x": _halos(xg, ranges, rank),
            "halo_r": _halos(rg, ranges, rank),
        }
        P_ext = P[prow[rank]]  # owned rows, then the x-ghost rows (x_ext order)
        if last:
            d["P_loc"] = P_ext.tocsr()
            d["halo_p"] = None
        else:
            d["P_loc"] = _remap(P_ext, clo, chi, pg[rank])
            d["halo_p"] = _halos(pg, c_ranges, rank)
        out.append(d)
        ranges = c_ranges
    return out


def build(A0, P0, seeds, world, rank=None):
    """Partition maps for all ranks (or one rank). A0: n x n CSR, P0: n x nc CSR, seeds: sorted
    seed node of each coarse unknown (aggregate j's seed is seeds[j]).

    Returns a list (per rank) of dicts, or the dict of `rank`.
    """
    A0 = A0.tocsr()
    P0 = P0.tocsr()
    n = A0.shape[0]
    nc = P0.shape[1]
    seeds = np.asarray(seeds, dtype=np.int64)
    if len(seeds) != nc or (len(seeds) > 1 and np.any(np.diff(seeds) <= 0)):
        raise ValueError("coarse unknowns must be ordered by strictly increasing seed node")
    R0 = P0.T.tocsr()
    R0.sort_indices()
    ranges = row_ranges(n, world)
    his = np.array([h for _, h in ranges], dtype=np.int64)
    # coarse ownership by seed owner: contiguous because seeds are sorted
    c_bounds = [int(np.searchsorted(seeds, lo)) for lo, _ in ranges] + [nc]
    c_ranges = [(c_bounds[r], c_bounds[r + 1]) for r in range(world)]
    # ghost sets of every rank (needed to derive send lists)
    xg, rg = [], []
    for r, (lo, hi) in enumerate(ranges):
        Ar = A0[lo:hi]
        xg.append(_ghost_sets(Ar.indices, lo, hi))
        clo, chi = c_ranges[r]
        Rr = R0[clo:chi]
        rg.append(_ghost_sets(Rr.indices, lo, hi))
    out = []
    for r, (lo, hi) in enumerate(ranges):
        if rank is not None and r != rank:
            out.append(None)
            continue
        clo, chi = c_ranges[r]
        sends_x, sends_r = {}, {}
        for q in range(world):
            if q == r:
                continue
            need = xg[q][(xg[q] >= lo) & (xg[q] < hi)]
            if len(need):
                sends_x[q] = (need - lo).astype(np.int32)
            need = rg[q][(rg[q] >= lo) & (rg[q] < hi)]
            if len(need):
                sends_r[q] = (need - lo).astype(np.int32)
        hx = Halo(hi - lo, xg[r], owner_of(xg[r], his), sends_x)
        hr = Halo(hi - lo, rg[r], owner_of(rg[r], his), sends_r)
        A_loc = _remap(A0[lo:hi], lo, hi, xg[r])
        R_own = _remap(R0[clo:chi], lo, hi, rg[r])
        P_loc = P0[lo:hi].copy()
        out.append({
            "rank": r, "world": world, "lo": lo, "hi": hi, "n": n, "nc": nc,
            "c_lo": clo, "c_hi": chi, "c_ranges": c_ranges, "ranges": ranges,
            "A_loc": A_loc, "P_loc": P_loc, "R_own": R_own, "halo_x": hx, "halo_r": hr,
        })
    return out[rank] if rank is not None else out


def interior_split(M, n_owned_cols, min_frac=0.5):
    """Row split of a local operator for overlapping its halo exchange: the
    longest run of rows whose columns are all owned (< n_owned_cols), as (lo, hi) with both ends
    even (the row-pair kernels load epilogue vectors as 16-byte pairs; rounding only moves
    interior rows into the boundary parts). None when that run is shorter than min_frac of the
    rows or no row reads a ghost."""
    M = M.tocsr()
    n = M.shape[0]
    if n == 0:
        return None
    ghost = np.zeros(n, dtype=bool)
    lens = np.diff(M.indptr)
    rows = np.repeat(np.arange(n), lens)
    ghost[rows[M.indices >= n_owned_cols]] = True
    if not ghost.any():
        return None
    # runs of interior rows: boundaries where ghost flips
    interior = ~ghost
    edges = np.flatnonzero(np.diff(np.concatenate(([0], interior.astype(np.int8), [0]))))
    starts, ends = edges[0::2], edges[1::2]
    if len(starts) == 0:
        return None
    k = int(np.argmax(ends - starts))
    lo, hi = int(starts[k]), int(ends[k])
    lo += lo & 1
    hi -= hi & 1
    if hi - lo < max(2, min_frac * n):
        return None
    return lo, hi


# ---------------------------------------------------------------- vectorised (torch) build
# The same partition maps computed with torch tensor ops on the operators' own device arrays
# (VERDICT r05 Weak #6: the numpy build above took 5.1 s per rank at C4 — np.unique over every
# rank's 70 M column indices — and needed host copies of every partitioned operator). Every
# rank's ghost sets come from ONE pass over each operator: the entries whose column lies in
# another rank's range, keyed (owner of the row, column) and made unique; the rank then cuts
# only its own rows. Bitwise the same maps as build_levels (tests/test_partition_torch.py).

class TCSR:
    """A CSR matrix as three torch tensors (crow int64 or int32, col int32, val float64)."""

    __slots__ = ("crow", "col", "val", "shape")

    def __init__(self, crow, col, val, shape):
        self.crow, self.col, self.val, self.shape = crow, col, val, (int(shape[0]), int(shape[1]))

    @property
    def nnz(self):
        return int(self.col.numel())

    def rows(self, a, b):
        """Rows [a, b) (a view of col / val)."""
        s, e = int(self.crow[a]), int(self.crow[b])
        return TCSR(self.crow[a:b + 1] - s, self.col[s:e], self.val[s:e], (b - a, self.shape[1]))

    def to_scipy(self):
        return sp.csr_matrix((self.val.cpu().numpy(), self.col.cpu().numpy(),
                              self.crow.cpu().numpy()), shape=self.shape)

    @classmethod
    def from_scipy(cls, M, device="cpu"):
        import torch
        M = M.tocsr()
        return cls(torch.as_tensor(M.indptr.astype(np.int64), device=device),
                   torch.as_tensor(M.indices.astype(np.int32), device=device),
                   torch.as_tensor(M.data.astype(np.float64), device=device), M.shape)


def _t_owner(idx, his_t):
    import torch
    return torch.searchsorted(his_t, idx, right=True)


def _t_entry_owner(crow, bounds):
    """Owner rank of every entry of a CSR whose rows are split at `bounds` (lo of each rank +
    the end): entries are contiguous per rank."""
    import torch
    cuts = crow[torch.as_tensor(bounds, dtype=torch.int64, device=crow.device)].to(torch.int64)
    counts = cuts[1:] - cuts[:-1]
    return torch.repeat_interleave(torch.arange(len(bounds) - 1, device=crow.device), counts)


def _t_split_keys(keys, n, world):
    """Unique (rank, index) keys rank * n + index -> per-rank ascending index arrays."""
    import torch
    keys = torch.unique(keys)
    q = torch.div(keys, n, rounding_mode="floor")
    idx = keys - q * n
    counts = torch.bincount(q, minlength=world).cpu().numpy()
    parts = torch.split(idx, counts.tolist())
    return [p for p in parts]


def _t_cross_keys(M, row_bounds, col_his, n_cols):
    """keys (owner of the entry's row) * n_cols + column for entries whose column another rank
    owns."""
    import torch
    ro = _t_entry_owner(M.crow, row_bounds)
    col = M.col.to(torch.int64)
    co = _t_owner(col, col_his)
    cross = co != ro
    return ro[cross] * n_cols + col[cross]


def _t_gather_rows(M, rows):
    """The rows `rows` (int64 tensor, any order) of M, in that order."""
    import torch
    crow = M.crow.to(torch.int64)
    starts = crow[rows]
    lens = crow[rows + 1] - starts
    new_crow = torch.zeros(len(rows) + 1, dtype=torch.int64, device=crow.device)
    new_crow[1:] = torch.cumsum(lens, 0)
    total = int(new_crow[-1])
    pos = torch.arange(total, device=crow.device) - torch.repeat_interleave(new_crow[:-1], lens)
    src = torch.repeat_interleave(starts, lens) + pos
    return TCSR(new_crow, M.col[src], M.val[src], (len(rows), M.shape[1])), src, lens


def _t_remap(M, lo, hi, ghosts):
    """_remap on a TCSR: owned j -> j - lo, ghost g -> n_own + position(g); stored order kept."""
    import torch
    n_own = hi - lo
    col = M.col.to(torch.int64)
    own = (col >= lo) & (col < hi)
    out = torch.where(own, col - lo, n_own + torch.searchsorted(ghosts, col))
    return TCSR(M.crow, out.to(torch.int32), M.val, (M.shape[0], n_own + len(ghosts)))


def _t_halos(ghosts_all, ranges, r):
    """_halos from per-rank ghost tensors (moved to the host: they are small)."""
    g = [t.cpu().numpy().astype(np.int64) for t in ghosts_all]
    return _halos(g, ranges, r)


def build_levels_torch(As, Ps, Rs, seeds_list, world, rank):
    """build_levels for `rank` from TCSR operators (any torch device): As[l] n x n, Ps[l] n x nc,
    Rs[l] = P_l^T with ascending columns in every row (the device transpose's order, scipy's
    P.T.tocsr()). Returns the same per-level dicts, with TCSR matrices for A_loc / R_own / P_loc
    (on the operators' device)."""
    import torch
    K = len(As)
    ranges = row_ranges(As[0].shape[0], world)
    out = []
    for l in range(K):
        A, P, R = As[l], Ps[l], Rs[l]
        dev = A.col.device
        n, nc = A.shape[0], P.shape[1]
        c_ranges = _seed_ranges(seeds_list[l], ranges, nc)
        rb = [lo for lo, _ in ranges] + [n]
        cb = [lo for lo, _ in c_ranges] + [nc]
        his = torch.as_tensor([h for _, h in ranges], dtype=torch.int64, device=dev)
        chis = torch.as_tensor([h for _, h in c_ranges], dtype=torch.int64, device=dev)
        # x ghosts: columns of A outside the row owner's range; r ghosts: fine columns of R
        # (rows split by coarse ranges) outside the fine range of the row's owner
        xg = _t_split_keys(_t_cross_keys(A, rb, his, n), n, world)
        rg = _t_split_keys(_t_cross_keys(R, cb, his, n), n, world)
        # P rows of rank q: its owned rows, then its x-ghost rows; P ghosts = coarse columns of
        # those rows outside q's coarse range
        last = l == K - 1
        pg = None
        if not last:
            keys = [_t_cross_keys(P, rb, chis, nc)]
            for q in range(world):
                if len(xg[q]):
                    Pq, _, _ = _t_gather_rows(P, xg[q])
                    c = Pq.col.to(torch.int64)
                    keys.append(q * nc + c[(c < c_ranges[q][0]) | (c >= c_ranges[q][1])])
            pg = _t_split_keys(torch.cat(keys), nc, world)
        lo, hi = ranges[rank]
        clo, chi = c_ranges[rank]
        d = {
            "level": l, "rank": rank, "world": world, "lo": lo, "hi": hi, "n": n, "nc": nc,
            "c_lo": clo, "c_hi": chi, "c_ranges": c_ranges, "ranges": ranges,
            "A_loc": _t_remap(A.rows(lo, hi), lo, hi, xg[rank]),
            "R_own": _t_remap(R.rows(clo, chi), lo, hi, rg[rank]),
            "halo_x": _t_halos(xg, ranges, rank),
            "halo_r": _t_halos(rg, ranges, rank),
        }
        prow = torch.cat([torch.arange(lo, hi, device=dev, dtype=torch.int64), xg[rank]])
        P_ext, _, _ = _t_gather_rows(P, prow)
        if last:
            d["P_loc"] = P_ext
            d["halo_p"] = None
        else:
            d["P_loc"] = _t_remap(P_ext, clo, chi, pg[rank])
            d["halo_p"] = _t_halos(pg, c_ranges, rank)
        out.append(d)
        ranges = c_ranges
    return out


def interior_split_torch(M, n_owned_cols, min_frac=0.5):
    """interior_split on a TCSR (the per-row ghost test on M's device, the run search on the
    host)."""
    import torch
    n = M.shape[0]
    if n == 0:
        return None
    lens = (M.crow[1:] - M.crow[:-1]).to(torch.int64)
    rows = torch.repeat_interleave(torch.arange(n, device=M.col.device), lens)
    ghost = torch.zeros(n, dtype=torch.bool, device=M.col.device)
    ghost[rows[M.col.to(torch.int64) >= n_owned_cols]] = True
    ghost = ghost.cpu().numpy()
    if not ghost.any():
        return None
    interior = ~ghost
    edges = np.flatnonzero(np.diff(np.concatenate(([0], interior.astype(np.int8), [0]))))
    starts, ends = edges[0::2], edges[1::2]
    if len(starts) == 0:
        return None
    k = int(np.argmax(ends - starts))
    lo, hi = int(starts[k]), int(ends[k])
    lo += lo & 1
    hi -= hi & 1
    if hi - lo < max(2, min_frac * n):
        return None
    return lo, hi
