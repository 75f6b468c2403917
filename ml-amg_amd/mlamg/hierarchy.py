"""Device AMG hierarchy: setup on the GPU and the V-cycle executor (mlamg_hier_*).

Setup per level follows the reference's aggregation-based SA recipe, all on the device:
  C = strength(A)                                    utils/common.py:25-31 ('invabs', 'abs', 'unit',
                                                     'evolution', 'olson')
  seeds = RandomState(seed).permutation(n)[:ceil(alpha*n)]       graph.py:230-231; evaluate_dataset.py:80-85
  (dist, label) = Bellman-Ford(C, seeds)            graph.py:7-53   (or Lloyd: graph.py:156-239)
  Agg = aggregate operator(label)                   graph.py:56-86
  omega = (4/3)/lambda_max(Dinv A);  P = (I - omega Dinv A) Agg    multigrid.py:102-108
  R = P^T;  A_c = (R A) P                            multigrid.py:165
until n <= max_coarse; the last operator is inverted densely (multigrid.py:168 factorized).
The cycle is the Jacobi V(1,1) of ns/preconditioner/MLAMG.py:143-197 applied recursively.

Seeds are RandomState(seed).permutation(n)[:k] bit for bit, the reference seeding (numpy's
MT19937 draws on the host, the shuffle's first k positions resolved on the device: graph.
legacy_permutation); with sort_seeds=True (default for the multilevel solver) they are sorted so that
coarse unknowns follow the fine ordering (better locality, contiguous ownership per GPU).
"""
from __future__ import annotations

import ctypes
import math
import statistics
import time

import numpy as np
import scipy.sparse as sp
import torch

from . import _lib
from ._lib import MLAMG_EUNSUPPORTED, MlamgError, _tol_arg, call, ptr, stream_ptr
from .graph import (aggregate_op_device, bellman_ford_device, labels_to_columns,
                    legacy_permutation, lloyd_cluster_device, modified_bellman_ford_device)
from .multigrid import lambda_max_dinv_a
from .sparse import DeviceCSR, _device, as_device, galerkin, to_device_vec

STRENGTH_MODES = {"abs": 0, "invabs": 1, "unit": 2, "same": 3}


def strength(A_dev, mode="invabs", rho=None):
    """Strength graph of a device operator: the elementwise measures of utils/common.py:26,28,29
    or the evolution measures of :27,30 ('evolution', 'olson'; rho(D^-1 A) = rho, default the
    device Lanczos value)."""
    if mode in ("evolution", "olson"):
        from .strength import evolution_device
        return evolution_device(A_dev, mode, rho=rho)
    h = ctypes.c_void_p()
    call("mlamg_strength", A_dev.handle, STRENGTH_MODES[mode], ctypes.byref(h), stream_ptr())
    return DeviceCSR(h)


class CoarseSolveError(RuntimeError):
    """The coarsest solve cannot be done as asked (PCG on a non-symmetric operator too large
    for the dense solver) or a PCG coarse solve broke down (operator not positive definite)."""
    code = MLAMG_EUNSUPPORTED


def csr_symmetric(M, rtol=0.0):
    """True when the device CSR M is symmetric to `rtol` (mlamg_csr_symmetric)."""
    ok = ctypes.c_int()
    call("mlamg_csr_symmetric", M.handle, float(rtol), ctypes.byref(ok), stream_ptr())
    return bool(ok.value)


def _pyamg_empty_level(H, L, A_dev, agg, cpts, rounds, Bv, lvl, improve_iterations, rho,
                       omega):
    """pyamg_sa's level when standard aggregation finds no aggregate: an n x 1 empty AggOp
    (pyamg's standard_aggregation return), T = 0, B_c = [0], P = 0 (n x 1), R = P^T, A_c =
    [[0]]. The level keeps its symmetric block Gauss-Seidel smoother (pyamg still smooths it;
    for the operators this happens on — no off-diagonal couplings — the sweep is an exact
    solve). Appends L to H and returns (A_c, B_c)."""
    from .multigrid import GaussSeidel
    n = A_dev.shape[0]
    dev = _device()
    L.Agg = DeviceCSR.from_scipy(sp.csr_matrix((n, 1)))
    L.agg_col = agg
    L.seeds = cpts[:0]
    L.n_seeds = 1
    L.bf_sweeps = int(rounds.value)
    if lvl == 0 and improve_iterations > 0:
        L.gs = GaussSeidel(A_dev, "symmetric", block=True)
        L.gs.sweep(Bv, torch.zeros_like(Bv), int(improve_iterations))
    L.B = Bv
    dinv = torch.empty(n, dtype=torch.float64, device=dev)
    call("mlamg_diag_pinv", A_dev.handle, ptr(dinv), stream_ptr())
    if rho == "lanczos":
        # rho(D^-1 A) of an operator without off-diagonal couplings: 1 where a_ii != 0
        L.lam = 1.0 if bool((dinv != 0).any()) else 0.0
    elif rho == "arnoldi":  # pyamg's estimate (draws from numpy's global generator)
        from .strength import approximate_spectral_radius
        h = ctypes.c_void_p()
        call("mlamg_csr_scale_rows", A_dev.handle, ptr(dinv), 0, ctypes.byref(h), stream_ptr())
        L.lam = approximate_spectral_radius(DeviceCSR(h))
    else:
        r = _level_item(rho, lvl) if isinstance(rho, (list, tuple)) else rho
        if r is None:
            raise ValueError(f"no rho given for level {lvl}")
        L.lam = float(r)
    L.omega = omega / L.lam if L.lam else 0.0
    L.P = DeviceCSR.from_scipy(sp.csr_matrix((n, 1)))
    L.R = DeviceCSR.from_scipy(sp.csr_matrix((1, n)))
    L.dinv = dinv
    H.galerkin_s.append(0.0)
    H.levels.append(L)
    return (DeviceCSR.from_scipy(sp.csr_matrix((1, 1))),
            torch.zeros(1, dtype=torch.float64, device=dev))


class Level:
    __slots__ = ("A", "dinv", "P", "R", "Agg", "omega", "lam", "lanczos_iters", "n_seeds",
                 "bf_sweeps", "seeds", "gs", "labels", "agg_col", "B", "sa_prolong")

    def __init__(self, A):
        self.A = A
        self.dinv = None
        self.P = self.R = self.Agg = None
        self.omega = self.lam = None
        self.lanczos_iters = 0
        self.n_seeds = 0
        self.bf_sweeps = 0
        self.seeds = None
        self.gs = None
        self.labels = None  # per-node aggregate seed (node id, -1 none) when built by BF
        self.agg_col = None  # per-node aggregate column (int32 device tensor, -1 none)
        self.B = None  # near-nullspace candidate fitted at this level (pyamg_sa)
        self.sa_prolong = False  # P = (I - omega D^-1 A) Agg formed here (mlamg_sa_smoother)


_PHASES = ("count", "alloc", "expand", "sort", "runsum", "emit", "finalize", "free")


def _setup_phases(reset=False):
    """Accumulated SpGEMM phase wall times (ms) since the last reset (mlamg_setup_phase_times)."""
    buf = (ctypes.c_double * len(_PHASES))()
    call("mlamg_setup_phase_times", buf, len(_PHASES), int(bool(reset)))
    return {k: round(float(v), 2) for k, v in zip(_PHASES, buf)}


def _level_item(spec, lvl):
    """The level-`lvl` entry of a per-level specification (None, one item = level 0, or a
    list / tuple of items)."""
    if spec is None:
        return None
    if isinstance(spec, (list, tuple)):
        return spec[lvl] if lvl < len(spec) else None
    return spec if lvl == 0 else None


def _aggregate_operator(agg, n):
    """Agg (n x k, ones) on the device from a label vector (-1 = unaggregated) or a matrix."""
    if isinstance(agg, DeviceCSR):
        return agg
    if sp.issparse(agg):
        if agg.shape[0] != n:
            raise ValueError(f"aggregate matrix has {agg.shape[0]} rows, the operator {n}")
        A = sp.csr_matrix(agg, dtype=np.float64)
        A.data[:] = 1.0
        return DeviceCSR.from_scipy(A)
    lab = np.asarray(agg.cpu().numpy() if isinstance(agg, torch.Tensor) else agg).astype(np.int64)
    if lab.shape != (n,):
        raise ValueError(f"aggregate labels must have shape ({n},), got {lab.shape}")
    k = int(lab.max()) + 1 if lab.size else 0
    return aggregate_op_device(torch.as_tensor(lab.astype(np.int32)).to(_device()), k)


def rhs_arg(b):
    """The right-hand side handed to mlamg_hier_vcycle: None when every entry of b is +0.0
    (bit pattern 0, so -0.0 does not count) — the reference's convergence-factor problems
    (utils/common.py:74, utils/evaluate_dataset.py:92: b = zeros). The fine-level kernels then
    take b = +0.0 instead of streaming a vector of zeros; the results are the same bits. One
    reduction over b per call (no per-cycle cost)."""
    if b is None:
        return None
    if b.numel() and bool(torch.count_nonzero(b.reshape(-1).contiguous().view(torch.int64))):
        return b
    return None


class Hierarchy:
    """A multilevel (or two-level) smoothed-aggregation hierarchy resident on the GPU."""

    def __init__(self):
        self.levels = []
        self.Ac = None
        self.dense = None
        self.handle = None
        self.recipe = "mlamg_sa"  # Hierarchy.build / two_level; "pyamg_sa" from pyamg_sa()
        self.jacobi_weight = 2.0 / 3.0
        self.nu_pre = 1
        self.nu_post = 1
        self.timings = {}
        self.pcg = None
        self.inner = None
        self.coarse_gmres = False  # coarsest solve by GMRES + inner hierarchy (_make_coarse_gmres)
        self._breakdowns_seen = 0
        self._factored = {}

    # ------------------------------------------------------------------ construction
    @classmethod
    def two_level(cls, A, P, omega=2.0 / 3.0, nu_pre=1, nu_post=1, dinv_w=None,
                  smoother="jacobi", norm="residual", coarse="auto"):
        """Two-level cycle with a given P: MLAMG.amg_2_v (ns/preconditioner/MLAMG.py:120-122,
        smoother='jacobi') or multigrid.amg_2_v (multigrid.py:111-210, smoother='gauss_seidel';
        norm='x' records ||x||_2 per cycle, the error_tol mode). coarse='dense' forces the
        dense inverse (up to DENSE_LIMIT rows) where 'auto' would take PCG; coarse='gmres'
        the GMRES coarse solve (any A_c; Hierarchy._make_coarse_gmres)."""
        from .multigrid import GaussSeidel
        H = cls()
        H.jacobi_weight = omega
        tm, t0 = {}, time.perf_counter()
        L = Level(as_device(A))
        L.P = as_device(P)
        L.R = L.P.transpose()
        L.dinv = L.A.diag_inv(omega) if dinv_w is None else to_device_vec(dinv_w)
        H.levels.append(L)
        torch.cuda.synchronize()
        tm["upload"], t0 = time.perf_counter() - t0, time.perf_counter()
        H.Ac = galerkin(L.R, L.A, L.P)
        torch.cuda.synchronize()
        tm["galerkin"], t0 = time.perf_counter() - t0, time.perf_counter()
        n_c = H.Ac.shape[0]
        if coarse == "dense" and n_c > cls.DENSE_LIMIT:
            raise CoarseSolveError(f"coarse operator of {n_c} rows: the dense solver is limited "
                                   f"to {cls.DENSE_LIMIT} rows")
        if coarse not in ("auto", "dense", "gmres"):
            raise ValueError(f"unknown coarse solver {coarse!r}")
        H._finalize(nu_pre, nu_post,
                    dense_max=n_c if coarse == "dense" else cls.TWO_LEVEL_DENSE_MAX,
                    coarse="gmres" if coarse == "gmres" else None)
        torch.cuda.synchronize()
        tm["coarse_solver"], t0 = time.perf_counter() - t0, time.perf_counter()
        if smoother == "gauss_seidel":
            L.gs = GaussSeidel(L.A)
            call("mlamg_hier_set_level_smoother", H.handle, 0, L.gs.handle)
            torch.cuda.synchronize()
            tm["gauss_seidel"] = time.perf_counter() - t0
        elif smoother != "jacobi":
            raise ValueError(f"unknown smoother {smoother!r}")
        H.timings = tm
        if norm not in ("residual", "x"):
            raise ValueError(f"unknown norm {norm!r}")
        call("mlamg_hier_set_norm", H.handle, 0 if norm == "residual" else 1)
        return H

    EXACT_CANDIDATES = (("csr_stream", 0), ("sell", 1), ("sell", 512), ("sorted", 0),
                        ("sorted", 2), ("sell_dict", 1), ("sell_dict", 512), ("rowpat", 0))
    LONG_CANDIDATES = (("long", 0),)
    VECTOR_CANDIDATES = (("vector", 64), ("vector", 128), ("vector", 256), ("vector", 512))

    # bytes read between two timed launches of the autotune, so each one starts with the
    # operator and x out of the caches (L2 4 MB per XCD, MALL 256 MB) as in the cycle, where the
    # other levels' streams pass in between; a read leaves no dirty lines to write back during
    # the timed launch
    FLUSH_BYTES = 512 << 20

    @staticmethod
    def _time_format(M, fmt, arg, x, y, reps=5, kind="A", flush=None):
        """Median time of M's cycle operation in format fmt over `reps` launches, each after a
        cache flush (a read of `flush`): the residual epilogue for A (r = b - A x, as in the
        cycle; here b = y), y += M x for P, y = M x for R. Timing a launch repeated back to back
        measures cache-resident operators (any operator up to the MALL's size), which
        favoured formats that are not the fastest in the cycle."""
        M.set_format(fmt, arg)
        if kind == "A":
            def op():
                call("mlamg_residual", M.handle, ptr(y), ptr(x), ptr(y), None, stream_ptr())
        elif kind == "P":
            def op():
                call("mlamg_prolong_add", M.handle, ptr(x), ptr(y), stream_ptr())
        else:
            def op():
                M.matvec(x, out=y)
        op()
        s = torch.cuda.current_stream()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(reps)]
        sink = torch.empty((), dtype=flush.dtype, device=flush.device) if flush is not None else None
        for e0, e1 in ev:
            if flush is not None:
                torch.sum(flush, dim=0, out=sink)
            e0.record(s)
            op()
            e1.record(s)
        ev[-1][1].synchronize()
        return statistics.median(e0.elapsed_time(e1) for e0, e1 in ev) * 1e3  # us

    # Autotune pruning: the fewest bytes per stored nonzero a format can stream (sorted: 4-byte
    # packed index + a 1-byte value code when the values fit a dictionary; sell_dict: a 2-byte
    # code; rowpat: ~0, one byte per pair of rows; vector: 16-bit indices) at 7 TB/s: no
    # candidate can beat that from a cold cache (the autotune reads 512 MB, twice the MALL,
    # before each timed launch; 8 TB/s is the HBM peak, ~6.3 TB/s what streams reach, and the
    # fastest cold kernel measured here runs at 3.7 TB/s of its bytes). A pruned candidate costs
    # nothing but a timing chance: every format of the family computes the same bits. (Round 4:
    # 8 -> 7 TB/s, so that e.g. SELL and CSR-stream are no longer built and timed for P_0 / R_0,
    # whose sorted format already beats their bytes at 7 TB/s.)
    FORMAT_MIN_BYTES_PER_NNZ = {"csr_stream": 12.0, "sell": 12.0, "sorted": 5.0, "sell_dict": 2.0,
                                "rowpat": 0.0, "long": 12.0, "vector": 10.0}
    LB_PEAK_BPS = 7e12
    # a SELL / dictionary-SELL timed at more than this many times the best format so far skips
    # its sigma-sorted (row-length-ordered) variant
    SIGMA_SKIP_RATIO = 1.5

    @classmethod
    def _lower_bound_us(cls, M, kind, fmt):
        n_rows, n_cols = M.shape
        vec = 8.0 * (n_cols + n_rows + (n_rows if kind in ("A", "P") else 0))  # x, y (+ b / y in)
        return (cls.FORMAT_MIN_BYTES_PER_NNZ[fmt] * M.nnz + vec) / cls.LB_PEAK_BPS * 1e6

    # operators whose mean row has at least this many entries use the lane-parallel CSR-vector
    # family (canonical order, one result for every width); shorter rows use the exact-order
    # (scipy) family. A rule on the matrix, not a timing: measured on the C4 hierarchy
    # (tools/coarse_formats.py) the vector kernels win from R_2 (357 entries per row: 18 vs
    # 34 us) up and lose below (A_2, 187 per row: 79 vs 54 us).
    VEC_MIN_MEAN_ROW = 256

    # autotune decisions per operator signature (kind, shape, nnz, fingerprint of rows, columns
    # and value bits, candidate family): a hierarchy rebuilt on the same operator (a dataset loop
    # re-solving one grid, a distributed rank rebuilding rank 0's hierarchy) takes the same
    # kernel without re-timing (VERDICT r04 Next #7). The choice is a timing decision only —
    # every candidate of a family computes the same bits — so a stale entry costs speed, never
    # a result. Bounded; cleared by clear_tune_cache().
    _TUNE_CACHE = {}
    TUNE_CACHE_MAX = 256

    @classmethod
    def clear_tune_cache(cls):
        cls._TUNE_CACHE.clear()

    def apply_formats(self, fine_format="autotune", coarse_format="auto", vec_min_row=None,
                      first_level=0):
        """Choose the SpMV kernel of every operator.

        The candidates of one operator all compute the same bits, so the autotune — a timing
        decision — cannot change any result:
          * mean row length < vec_min_row (default VEC_MIN_MEAN_ROW): the exact-order family,
            scipy's left-to-right order (CSR-stream, SELL-64[-sigma], dictionary SELL,
            gather-sorted CSR-stream, row-pair patterns, long-row tiles) — bitwise A @ x;
          * otherwise (levels >= 1 only; coarse_format='auto'): the CSR-vector family, widths
            64..512 in one canonical lane-parallel order (oracle.c vec_matvec), for the long
            rows of coarse Galerkin operators where a one-lane chain is latency-bound.
        Which family applies is a rule on the matrix; coarse_format='exact' keeps every
        operator in the exact family. fine_format='autotune' times the family's kernels on each
        operator once and keeps the fastest (self.tuning); any other value forces that format.
        first_level: the global index of self.levels[0] (a hierarchy that continues another one,
        e.g. the replicated tail of the distributed setup: the family rule uses the global
        level index)."""
        if coarse_format not in ("auto", "exact", "vector"):
            raise ValueError(f"coarse_format must be 'auto' or 'exact', got {coarse_format!r}")
        vec_min_row = self.VEC_MIN_MEAN_ROW if vec_min_row is None else vec_min_row
        self.tuning = []
        dev = torch.device("cuda", torch.cuda.current_device())
        flush = (torch.ones(self.FLUSH_BYTES // 8, dtype=torch.float64, device=dev)
                 if fine_format == "autotune" else None)
        for i, L in enumerate(self.levels):
            row = {}
            for name, M in (("A", L.A), ("P", L.P), ("R", L.R)):
                if (i + first_level > 0 and coarse_format != "exact" and M.shape[0] <= (1 << 20)
                        and M.nnz >= vec_min_row * M.shape[0]):
                    cands = list(self.VECTOR_CANDIDATES)
                else:
                    cands = list(self.EXACT_CANDIDATES)
                    if M.nnz >= 16 * M.shape[0]:
                        cands += list(self.LONG_CANDIDATES)
                if fine_format != "autotune":
                    M.set_format(fine_format if fine_format != "vector" else "auto_exact")
                    row[name] = {"chosen": M.get_format()[:2]}
                    continue
                key = (name, M.shape, M.nnz, M.fingerprint(), tuple(cands))
                hit = self._TUNE_CACHE.get(key)
                if hit is not None:
                    fmt, arg = hit["chosen"].split("/")
                    M.set_format(fmt, int(arg))
                    row[name] = dict(hit, cached=True)
                    continue
                x = torch.randn(M.shape[1], dtype=torch.float64, device=dev)
                y = torch.zeros(M.shape[0], dtype=torch.float64, device=dev)
                times = {}
                # most compact formats first; a candidate whose bytes could not move in less
                # than the best time so far, even at LB_PEAK_BPS, is neither built nor timed
                # (a timing rule only: every candidate of the family computes the same bits)
                lbs = {c: self._lower_bound_us(M, name, c[0]) for c in cands}
                cands.sort(key=lambda c: lbs[c])
                pruned = []
                value_dict = False
                refused = set()
                for fmt, arg in cands:
                    if times and lbs[(fmt, arg)] >= min(times.values()):
                        pruned.append(f"{fmt}/{arg}")
                        continue
                    if fmt in refused or ((fmt, arg) == ("sorted", 2) and value_dict):
                        # builds that would be refused: a dictionary-SELL or sorted limit of
                        # one variant (too many column offsets or values, a row over a block)
                        # holds for the others, and block dictionaries are refused when the
                        # <= 256-value table applies (known from sorted/0). At C4 these
                        # refused builds were half the autotune (0.46 of 0.99 s).
                        pruned.append(f"{fmt}/{arg}")
                        continue
                    try:
                        t = self._time_format(M, fmt, arg, x, y, kind=name, flush=flush)
                        times[f"{fmt}/{arg}"] = t
                        if (fmt, arg) == ("sorted", 0):
                            value_dict = M.get_format()[1] == 1
                        if fmt in ("sell", "sell_dict") and arg == 1 and \
                                t > self.SIGMA_SKIP_RATIO * min(times.values()):
                            # the sigma-sorted variant only reorders rows by length: it does not
                            # close a gap this large to the best format (C4 A_0: its build
                            # alone took 0.18 s, and it ran at 106 against rowpat's 56 us)
                            refused.add(fmt)
                    except MlamgError as e:  # format limits (e.g. sorted: row > 4096 nnz)
                        if e.code != MLAMG_EUNSUPPORTED:
                            raise
                        if fmt in ("sell_dict", "sell") or (fmt, arg) == ("sorted", 0):
                            refused.add(fmt)
                best = min(times, key=times.get)
                fmt, arg = best.split("/")
                M.set_format(fmt, int(arg))
                row[name] = {"chosen": best, "us": {k: round(v, 2) for k, v in times.items()},
                             "pruned": pruned}
                if len(self._TUNE_CACHE) >= self.TUNE_CACHE_MAX:
                    self._TUNE_CACHE.pop(next(iter(self._TUNE_CACHE)))
                self._TUNE_CACHE[key] = row[name]
            self.tuning.append(row)
        self.attach_dinvs()

    def attach_dinvs(self):
        """Let every rowpat level operator take its Jacobi weights from its pattern table."""
        for L in self.levels:
            if L.A.get_format()[0] == "rowpat":
                L.A.attach_dinv(L.dinv)

    def set_factored_prolong(self, level=0, on=True):
        """Opt-in (VERDICT r04 Next #5): apply level `level`'s prolongation factored, x += t -
        (w / a_ii) (A t) with t = Agg e (P = (I - w D^-1 A) Agg, ns/lib/multigrid.py:102-108),
        through the level operator's uniform row-pair kernel (csrc/spmv.hip spmv_fadd) instead
        of streaming the explicit P. Same operator, different rounding: NOT bitwise the explicit
        P @ e (tests hold it to the oracle cycle at rtol 1e-11). Needs the level's aggregates
        (built here, not supplied as P) and a constant-stencil operator; raises MlamgError
        (EUNSUPPORTED) otherwise. on=False restores x += P e."""
        L = self.levels[level]
        if not on:
            call("mlamg_hier_set_factored_prolong", self.handle, int(level), None, None, None)
            self._factored.pop(level, None)
            return
        if self.recipe != "mlamg_sa" or not L.sa_prolong:
            # pyamg_sa's P = T - (w/rho) D^-1 A T smooths the normalised candidate T, not the
            # 0/1 aggregate operator: the factored form would be a different prolongator
            raise _lib.MlamgError(_lib.MLAMG_EUNSUPPORTED, "factored prolongation needs "
                                  "P = (I - w D^-1 A) Agg built by Hierarchy.build "
                                  f"(recipe {self.recipe!r}, level {level})")
        if L.agg_col is None or L.omega is None:
            raise ValueError("factored prolongation needs the level's aggregates and SA weight")
        ip, ij, ax = L.A.arrays()
        h = ctypes.c_void_p()
        n = L.A.shape[0]
        call("mlamg_csr_create", n, n, L.A.nnz, ctypes.c_void_p(ip), ctypes.c_void_p(ij),
             ctypes.c_void_p(ax), _lib.MLAMG_WRAP_DEVICE, ctypes.byref(h))
        A_uni = DeviceCSR(h, keep=(L.A,))  # wraps L.A's arrays: keep L.A alive
        A_uni.set_format("rowpat")
        c = L.A.diag_inv(L.omega)  # w / a_ii
        A_uni.attach_dinv(c)
        call("mlamg_hier_set_factored_prolong", self.handle, int(level), A_uni.handle,
             ptr(L.agg_col), ptr(c))
        self._factored[level] = (A_uni, c)

    def formats(self):
        return [{"A": L.A.get_format(), "P": L.P.get_format(), "R": L.R.get_format()}
                for L in self.levels]

    def set_formats(self, formats):
        """Apply a formats() list (e.g. rank 0's autotune result on every rank, so that the
        replicated hierarchies of a distributed run sum every row in the same order)."""
        if len(formats) != len(self.levels):
            raise ValueError("formats list does not match the number of levels")
        for L, f in zip(self.levels, formats):
            for name in ("A", "P", "R"):
                fmt, arg = f[name][0], f[name][1]
                getattr(L, name).set_format(fmt, int(arg))
        self.attach_dinvs()

    @classmethod
    def build(cls, A, *, alpha=0.1, strength_mode="invabs", aggregation="bellman_ford",
              max_coarse=1000, max_levels=10, jacobi_weight=2.0 / 3.0, seed=0, sort_seeds=True,
              lanczos_tol=1e-15, lanczos_iter=20000, lloyd_maxiter=10, nu_pre=1, nu_post=1,
              fine_format="autotune", coarse_format="auto", verbose=False, finalize=True,
              aggregates=None, prolongators=None, coarse_order="seed"):
        """Smoothed-aggregation hierarchy built on the GPU.

        Per level: strength -> seeds RandomState(seed).permutation(n)[:ceil(alpha n)] ->
        seeded Bellman-Ford (or Lloyd) aggregates -> SA prolongator P = (I - w D^-1 A) Agg with
        w = (4/3)/lambda_max(D^-1 A) (ns/lib/multigrid.py:102-108) -> A_c = P^T A P (:165).

        aggregation:
          'bellman_ford' (default): every level the order-independent seeded Bellman-Ford
              (label = smallest seed among tight predecessors), seeds sorted (sort_seeds);
          'reference': level 0 is the reference's "dumb" recipe of
              utils/evaluate_dataset.py:80-90 exactly — unsorted RandomState(seed) seeds, the
              in-place row-major push sweeps of ns/lib/graph.py:40-51 in fp32
              (mlamg_bellman_ford) and nearest_center_to_agg's columns (graph.py:56-86: column t
              = seeds[t]); coarser levels (no reference counterpart) as 'bellman_ford'.
              coarse_order='sorted' relabels the level-0 aggregates in ascending seed order
              (the same aggregates — each column is the same node set — permuted so coarse
              unknowns follow the fine ordering: locality, and the contiguous coarse ownership
              the distributed executor needs); 'seed' keeps the reference's column order;
          'lloyd': pyamg lloyd_cluster with the order-independent rule.

        aggregates / prolongators: supplied instead of computed, for the first levels — e.g. the
        learned aggregates of C5 or the learned P of the MLAMG PC
        (ns/preconditioner/MLAMG.py:105-121). Each is one item (level 0) or a list (levels
        0, 1, ...); an aggregate item is a label vector (node -> aggregate column, -1 = none)
        or an n x k 0/1 matrix (scipy or DeviceCSR), and is smoothed into P as above; a
        prolongator item is used as P as given (no smoothing). jacobi_weight="sa" smooths every
        level with its SA weight w instead of a fixed one."""
        if aggregation not in ("bellman_ford", "reference", "lloyd"):
            raise ValueError(f"unknown aggregation {aggregation!r}")
        if coarse_order not in ("seed", "sorted"):
            raise ValueError(f"coarse_order must be 'seed' or 'sorted', got {coarse_order!r}")
        H = cls()
        H.jacobi_weight = jacobi_weight
        H.aggregation = aggregation
        H.coarse_order = coarse_order
        t_all = time.perf_counter()
        A_dev = as_device(A)
        tm = {"aggregation": 0.0, "lambda_max": 0.0, "prolongator": 0.0, "galerkin": 0.0,
              "formats": 0.0, "dense": 0.0}
        _setup_phases(reset=True)
        H.galerkin_s = []
        while True:
            n = A_dev.shape[0]
            if n <= max_coarse or len(H.levels) + 1 >= max_levels:
                break
            L = Level(A_dev)
            lvl = len(H.levels)
            P_given = _level_item(prolongators, lvl)
            Agg_given = _level_item(aggregates, lvl)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if P_given is None and Agg_given is None:
                C = strength(A_dev, strength_mode)
                k = int(math.ceil(alpha * n))
                if isinstance(seed, (int, np.integer)) and 0 <= int(seed) < 2 ** 32:
                    # RandomState(seed).permutation(n)[:k], bit for bit (device, csrc/seeds.hip)
                    seeds = legacy_permutation(seed, n, k).cpu().numpy().astype(np.int64)
                else:  # a seed numpy takes otherwise (None, an array, a generator's state)
                    seeds = np.random.RandomState(seed).permutation(n)[:k]
                if aggregation == "reference" and lvl == 0:
                    # evaluate_dataset.py:80-90: push-order sweeps from the unsorted seeds
                    seeds_dev = torch.as_tensor(seeds.astype(np.int32)).to(_device())
                    _, lab, L.bf_sweeps = modified_bellman_ford_device(C, seeds_dev)
                    if coarse_order == "sorted":
                        seeds = np.sort(seeds)
                        seeds_dev = torch.as_tensor(seeds.astype(np.int32)).to(_device())
                    col = labels_to_columns(lab, seeds_dev)
                    L.labels = lab
                else:
                    if sort_seeds:
                        seeds = np.sort(seeds)
                    seeds_dev = torch.as_tensor(seeds.astype(np.int32)).to(_device())
                    if aggregation == "lloyd":
                        _, col, _, L.bf_sweeps = lloyd_cluster_device(C, seeds_dev,
                                                                      lloyd_maxiter, exact=False)
                    else:
                        _, lab, L.bf_sweeps = bellman_ford_device(C, seeds_dev)
                        col = labels_to_columns(lab, seeds_dev)
                        L.labels = lab
                L.seeds = seeds
                L.Agg = aggregate_op_device(col, k)
                L.agg_col = col
                L.n_seeds = k
                del C
            elif P_given is None:
                L.Agg = _aggregate_operator(Agg_given, n)
                L.n_seeds = L.Agg.shape[1]
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            if P_given is None or jacobi_weight == "sa":
                if lvl == 0 and fine_format in ("autotune", "rowpat"):
                    # Lanczos runs on the operator's own SpMV: a constant stencil gets its
                    # row-pair format now (the autotune below reuses or replaces it)
                    try:
                        A_dev.set_format("rowpat")
                    except _lib.MlamgError as e:
                        if e.code != _lib.MLAMG_EUNSUPPORTED:
                            raise
                L.lam, L.lanczos_iters = lambda_max_dinv_a(A_dev, max_iter=lanczos_iter,
                                                           tol=lanczos_tol)
                L.omega = (4.0 / 3.0) / abs(L.lam)
            t2 = time.perf_counter()
            if P_given is None:
                h = ctypes.c_void_p()
                call("mlamg_sa_smoother", A_dev.handle, float(L.omega), ctypes.byref(h),
                     stream_ptr())
                S = DeviceCSR(h)
                L.P = S @ L.Agg
                L.sa_prolong = True
                del S
            else:
                L.P = as_device(P_given)
                if L.P.shape[0] != n:
                    raise ValueError(f"level {lvl}: prolongator has {L.P.shape[0]} rows, "
                                     f"the operator {n}")
            if L.P.shape[1] >= n:
                raise ValueError(f"level {lvl}: P has {L.P.shape[1]} columns for {n} rows "
                                 "(no coarsening)")
            L.R = L.P.transpose()
            L.dinv = A_dev.diag_inv(L.omega if jacobi_weight == "sa" else jacobi_weight)
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            A_next = galerkin(L.R, A_dev, L.P)
            torch.cuda.synchronize()
            t4 = time.perf_counter()
            tm["aggregation"] += t1 - t0
            tm["lambda_max"] += t2 - t1
            tm["prolongator"] += t3 - t2
            tm["galerkin"] += t4 - t3
            H.galerkin_s.append(round(t4 - t3, 4))
            H.levels.append(L)
            if verbose:
                print(f"[mlamg] level {len(H.levels) - 1}: n={n} nnz={A_dev.nnz} "
                      f"seeds={L.n_seeds} bf_sweeps={L.bf_sweeps} lam={L.lam} "
                      f"({L.lanczos_iters} it) "
                      f"P nnz={L.P.nnz} -> n_c={A_next.shape[0]} nnz_c={A_next.nnz} "
                      f"[agg {t1 - t0:.2f}s lam {t2 - t1:.2f}s P {t3 - t2:.2f}s gal {t4 - t3:.2f}s]",
                      flush=True)
            A_dev = A_next
        H.Ac = A_dev
        # host-side view of the SpGEMM phases (Galerkin + SA products), then drop the cached
        # scratch blocks (several GB at C4) so the cycle phase does not hold them
        H.spgemm_phases_ms = _setup_phases(reset=True)
        call("mlamg_scratch_trim", None)
        if not finalize:  # setup only (e.g. to take P for a two-level cycle)
            return H
        t5 = time.perf_counter()
        H.apply_formats(fine_format, coarse_format)
        torch.cuda.synchronize()
        t6 = time.perf_counter()
        H._finalize(nu_pre, nu_post)
        torch.cuda.synchronize()
        tm["formats"] = t6 - t5
        tm["dense"] = time.perf_counter() - t6
        tm["total"] = time.perf_counter() - t_all
        H.timings = tm
        return H

    @classmethod
    def pyamg_sa(cls, A, *, max_levels=10, max_coarse=10, theta=0.0, omega=4.0 / 3.0,
                 improve_iterations=4, rho="lanczos", B=None, fine_format="csr_stream",
                 coarse_format="exact", verbose=False):
        """pyamg.aggregation.smoothed_aggregation_solver(A, max_levels=max_levels) with pyamg's
        defaults — the multilevel solver of the reference's PyAMG preconditioner
        (ns/preconditioner/PyAMG.py:94) — built on the GPU. Per level, while n > max_coarse
        and fewer than max_levels levels:
          C = symmetric_strength_of_connection(A, theta)          mlamg_symmetric_strength
          AggOp = standard_aggregation(C)                          mlamg_standard_aggregation
          level 0: B <- 4 symmetric block Gauss-Seidel sweeps on A B = 0 from B = ones
                   (improve_candidates, level 0 only)              mlamg_gs_create_ex
          T, B_c = fit_candidates(AggOp, B)                        mlamg_fit_candidates
          P = T - (omega / rho) (D^-1 A) T  (jacobi_prolongation_smoother: D^-1 A by row
              scaling with get_diagonal(inv=True), scaled by omega / rho, times T, subtracted)
          R = P^T;  A_c = (R A) P
        Coarsest level: scipy.linalg.pinv(A_c) applied as a dense product (pyamg's 'pinv'
        coarse solver; the same scipy call). Smoother: symmetric block Gauss-Seidel, one
        iteration before and after the coarse correction (pyamg's presmoother/postsmoother).
        rho: rho(D^-1 A); 'lanczos' (default) the converged device Lanczos value, 'arnoldi'
        pyamg's approximate_spectral_radius estimate (15-step Arnoldi from np.random.rand: draws
        from numpy's global generator, as pyamg does), or a number / per-level list.
        pyamg is absent here: parity unpinned; every setup kernel is bitwise the oracle's
        restatement (oracle/oracle.c pyamg_*). Summation orders of pyamg's BSR products are not
        restated (the Galerkin product sums over k ascending, as scipy's CSR/CSC kernels do)."""
        from .multigrid import GaussSeidel
        if max_levels < 1:
            raise ValueError("max_levels must be >= 1")
        H = cls()
        H.recipe = "pyamg_sa"
        H.jacobi_weight = None
        t_all = time.perf_counter()
        A_dev = as_device(A)
        dev = _device()
        n0 = A_dev.shape[0]
        if B is None:
            Bv = torch.ones(n0, dtype=torch.float64, device=dev)
        else:
            Bn = np.asarray(B, dtype=np.float64)
            if Bn.size != n0:
                raise NotImplementedError("one near-nullspace candidate (B of shape (n, 1))")
            Bv = to_device_vec(Bn.reshape(-1)).clone()
        tm = {"strength": 0.0, "aggregation": 0.0, "candidates": 0.0, "rho": 0.0,
              "prolongator": 0.0, "galerkin": 0.0}
        H.galerkin_s = []
        while A_dev.shape[0] > max_coarse and len(H.levels) + 1 < max_levels:
            n = A_dev.shape[0]
            lvl = len(H.levels)
            L = Level(A_dev)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            h = ctypes.c_void_p()
            call("mlamg_symmetric_strength", A_dev.handle, float(theta), ctypes.byref(h),
                 stream_ptr())
            C = DeviceCSR(h)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            agg = torch.empty(n, dtype=torch.int32, device=dev)
            cpts = torch.empty(n, dtype=torch.int32, device=dev)
            k, rounds = ctypes.c_int64(), ctypes.c_int32()
            call("mlamg_standard_aggregation", C.handle, ptr(agg), ptr(cpts), ctypes.byref(k),
                 ctypes.byref(rounds), stream_ptr())
            del C
            k = int(k.value)
            if k == 0:
                # no node has an off-diagonal strength entry (a diagonal or fully decoupled
                # operator): pyamg's standard_aggregation returns an n x 1 empty AggOp, so
                # T = 0, B_c = 0, P = 0 and A_c = [[0]], whose pinv is 0 (a zero coarse
                # correction); the level keeps its smoother
                A_dev, Bv = _pyamg_empty_level(H, L, A_dev, agg, cpts, rounds, Bv, lvl,
                                               improve_iterations, rho, omega)
                continue
            L.Agg = aggregate_op_device(agg, k)
            L.agg_col = agg
            L.seeds = cpts[:k]
            L.n_seeds = k
            L.bf_sweeps = int(rounds.value)
            t2 = time.perf_counter()
            if lvl == 0 and improve_iterations > 0:
                # the same symmetric block sweep later smooths this level: one handle
                L.gs = GaussSeidel(A_dev, "symmetric", block=True)
                L.gs.sweep(Bv, torch.zeros_like(Bv), int(improve_iterations))
            L.B = Bv
            h = ctypes.c_void_p()
            Bc = torch.empty(k, dtype=torch.float64, device=dev)
            call("mlamg_fit_candidates", L.Agg.handle, ptr(Bv), 1e-10, ctypes.byref(h), ptr(Bc),
                 stream_ptr())
            T = DeviceCSR(h)
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            dinv = torch.empty(n, dtype=torch.float64, device=dev)
            call("mlamg_diag_pinv", A_dev.handle, ptr(dinv), stream_ptr())
            h = ctypes.c_void_p()
            call("mlamg_csr_scale_rows", A_dev.handle, ptr(dinv), 0, ctypes.byref(h),
                 stream_ptr())
            DinvA = DeviceCSR(h)
            if rho == "lanczos":
                # pyamg's own estimate is a 15-step Arnoldi value to a relative 1e-2
                # (approximate_spectral_radius's tol); 1e-6 is far tighter
                lam, L.lanczos_iters = lambda_max_dinv_a(A_dev, tol=1e-6)
                L.lam = abs(lam)
            elif rho == "arnoldi":
                from .strength import approximate_spectral_radius
                L.lam = approximate_spectral_radius(DinvA)
            else:
                r = _level_item(rho, lvl) if isinstance(rho, (list, tuple)) else rho
                if r is None:
                    raise ValueError(f"no rho given for level {lvl}")
                L.lam = float(r)
            t4 = time.perf_counter()
            L.omega = omega / L.lam
            h = ctypes.c_void_p()
            cvec = torch.full((n,), L.omega, dtype=torch.float64, device=dev)
            call("mlamg_csr_scale_rows", DinvA.handle, ptr(cvec), 0, ctypes.byref(h),
                 stream_ptr())
            DinvA = DeviceCSR(h)
            M = DinvA @ T
            del DinvA
            h = ctypes.c_void_p()
            call("mlamg_csr_sub", T.handle, M.handle, ctypes.byref(h), stream_ptr())
            L.P = DeviceCSR(h)
            del M, T
            L.R = L.P.transpose()
            L.dinv = dinv
            torch.cuda.synchronize()
            t5 = time.perf_counter()
            A_next = galerkin(L.R, A_dev, L.P)
            torch.cuda.synchronize()
            t6 = time.perf_counter()
            for key, dt in (("strength", t1 - t0), ("aggregation", t2 - t1),
                            ("candidates", t3 - t2), ("rho", t4 - t3),
                            ("prolongator", t5 - t4), ("galerkin", t6 - t5)):
                tm[key] += dt
            H.galerkin_s.append(round(t6 - t5, 4))
            H.levels.append(L)
            if verbose:
                print(f"[mlamg pyamg_sa] level {lvl}: n={n} nnz={A_dev.nnz} aggregates={k} "
                      f"rounds={L.bf_sweeps} rho={L.lam:.6g} P nnz={L.P.nnz} -> "
                      f"n_c={A_next.shape[0]} nnz_c={A_next.nnz}", flush=True)
            A_dev = A_next
            Bv = Bc
        H.Ac = A_dev
        H.B_coarse = Bv
        call("mlamg_scratch_trim", None)
        t7 = time.perf_counter()
        if H.levels:
            H.apply_formats(fine_format, coarse_format)
        t8 = time.perf_counter()
        H._finalize_pinv()
        torch.cuda.synchronize()
        tm["formats"] = t8 - t7
        tm["coarse_and_smoothers"] = time.perf_counter() - t8
        tm["total"] = time.perf_counter() - t_all
        H.timings = tm
        return H

    def _finalize_pinv(self):
        """pyamg's default coarse solver ('pinv': scipy.linalg.pinv of the dense A_c, applied as
        a product) and symmetric block Gauss-Seidel V(1,1) smoothing on every level."""
        import scipy.linalg
        from .multigrid import GaussSeidel
        self.nu_pre = self.nu_post = 1
        Ad = self.Ac.to_scipy().toarray()
        Pinv = np.ascontiguousarray(scipy.linalg.pinv(Ad), dtype=np.float64)
        self.coarse_pinv = Pinv
        h = ctypes.c_void_p()
        call("mlamg_dense_create_matrix", Pinv.ctypes.data_as(ctypes.c_void_p),
             int(Pinv.shape[0]), ctypes.byref(h), stream_ptr())
        self.dense = h
        hh = ctypes.c_void_p()
        call("mlamg_hier_create", ctypes.byref(hh))
        self.handle = hh
        for L in self.levels:
            call("mlamg_hier_add_level", hh, L.A.handle, ptr(L.dinv), L.P.handle, L.R.handle)
        call("mlamg_hier_set_coarse", hh, self.Ac.handle, self.dense)
        call("mlamg_hier_set_smoothing", hh, 1, 1)
        for i, L in enumerate(self.levels):
            if L.gs is None:
                L.gs = GaussSeidel(L.A, "symmetric", block=True)
            call("mlamg_hier_set_level_smoother", hh, i, L.gs.handle)

    # coarsest solve: a dense inverse up to this many rows (its setup is O(n_c^3)), above it
    # PCG preconditioned by an inner hierarchy of the coarse operator (csrc/pcg.hip)
    DENSE_MAX = 4096
    # the reference's two-level solve factors A_H once for ~30 cycles: there the O(n_c^3) dense
    # factor (device-wide, fp64 matrix cores) beats a PCG solve per cycle up to larger n_c
    TWO_LEVEL_DENSE_MAX = 10240
    COARSE_RTOL = 1e-12
    # the PCG preconditioner's hierarchy stops coarsening at this size (its coarsest operator is
    # then solved by the dense inverse)
    PCG_INNER_MAX_COARSE = 4096
    PCG_INNER_NU = 2  # V(nu, nu) preconditioner cycle (symmetric for any nu)

    # the dense solver's size limit (dense.hip mlamg_dense_create): an operator PCG may not take
    # (not symmetric) still gets an exact inverse up to this size
    DENSE_LIMIT = 32768
    SYMMETRY_RTOL = 1e-12  # dense.hip's "symmetric to rounding" test

    # coarsest solve of an operator that is not SPD and beyond DENSE_LIMIT rows: restarted GMRES
    # (restart GMRES_RESTART, at most GMRES_MAXITER restart cycles) preconditioned by one V-cycle
    # of an inner hierarchy, to ||r|| <= GMRES_RTOL ||b||; a solve whose final relative residual
    # stays above GMRES_FAIL_RTOL is a failed coarse solve (CoarseSolveError, like a SuperLU
    # factorisation failure)
    GMRES_RTOL = 1e-14
    GMRES_RESTART = 50
    GMRES_MAXITER = 20
    GMRES_FAIL_RTOL = 1e-10

    def _finalize(self, nu_pre, nu_post, dense_max=None, coarse_rtol=None, coarse=None):
        """coarse: None chooses (dense inverse up to dense_max rows; above, PCG for a symmetric
        A_c, else the dense inverse up to DENSE_LIMIT rows, else GMRES); 'gmres' forces GMRES."""
        self.nu_pre, self.nu_post = nu_pre, nu_post
        dense_max = self.DENSE_MAX if dense_max is None else dense_max
        n_c = self.Ac.shape[0]
        use_gmres = coarse == "gmres"
        if not use_gmres and n_c > dense_max and not csr_symmetric(self.Ac, self.SYMMETRY_RTOL):
            # PCG needs an SPD A_c (a Galerkin P^T A P of an SPD A is symmetric to rounding);
            # SuperLU, which the reference uses, takes any nonsingular A_H: an exact dense
            # inverse up to DENSE_LIMIT rows, GMRES beyond
            if n_c > self.DENSE_LIMIT:
                use_gmres = True
            else:
                dense_max = n_c
        if use_gmres:
            self._make_coarse_gmres()
        elif n_c <= dense_max:
            h = ctypes.c_void_p()
            call("mlamg_dense_create", self.Ac.handle, ctypes.byref(h), stream_ptr())
            self.dense = h
        else:
            self._make_coarse_pcg(self.COARSE_RTOL if coarse_rtol is None else coarse_rtol)
        hh = ctypes.c_void_p()
        call("mlamg_hier_create", ctypes.byref(hh))
        self.handle = hh
        for L in self.levels:
            call("mlamg_hier_add_level", hh, L.A.handle, ptr(L.dinv), L.P.handle, L.R.handle)
        if self.dense is not None:
            call("mlamg_hier_set_coarse", hh, self.Ac.handle, self.dense)
        elif self.pcg is not None:
            call("mlamg_hier_set_coarse_pcg", hh, self.Ac.handle, self.pcg)
        else:
            call("mlamg_hier_set_coarse_gmres", hh, self.Ac.handle, self.inner.handle,
                 float(self.GMRES_RTOL), float(self.GMRES_FAIL_RTOL), int(self.GMRES_RESTART),
                 int(self.GMRES_MAXITER))
        call("mlamg_hier_set_smoothing", hh, int(nu_pre), int(nu_post))

    def _make_coarse_gmres(self):
        """Coarsest solve for a coarse operator that is not SPD (non-symmetric, or indefinite:
        PCG broke down) and too large for the dense inverse: GMRES on A_c preconditioned by one
        V(2,2) cycle of an inner smoothed-aggregation hierarchy of A_c (weighted Jacobi w = 2/3,
        a dense coarsest inverse) — the reference factors any nonsingular A_H with SuperLU
        (ns/lib/multigrid.py:165-170)."""
        self.inner = Hierarchy.build(self.Ac, alpha=0.1, max_coarse=self.PCG_INNER_MAX_COARSE,
                                     jacobi_weight=2.0 / 3.0, lanczos_tol=1e-8,
                                     nu_pre=self.PCG_INNER_NU, nu_post=self.PCG_INNER_NU,
                                     fine_format="csr_stream", coarse_format="exact")
        self.coarse_gmres = True

    def _make_coarse_pcg(self, rtol, maxit=200):
        """Coarsest solve for an operator too large for the dense inverse (the reference
        factorises any size with SuperLU, ns/lib/multigrid.py:168): PCG on A_c with one V-cycle
        of an inner smoothed-aggregation hierarchy of A_c as preconditioner, to
        ||r|| <= rtol ||b||. The inner hierarchy smooths with the per-level SA weight
        w = (4/3)/lambda_max(D^-1 A) (w * lambda_max < 2: a convergent, symmetric V-cycle, i.e.
        an SPD preconditioner for an SPD A_c)."""
        self.inner = Hierarchy.build(self.Ac, alpha=0.1, max_coarse=self.PCG_INNER_MAX_COARSE,
                                     jacobi_weight="sa", lanczos_tol=1e-8,
                                     nu_pre=self.PCG_INNER_NU,
                                     nu_post=self.PCG_INNER_NU,
                                     fine_format="csr_stream", coarse_format="exact")
        h = ctypes.c_void_p()
        call("mlamg_pcg_create", self.Ac.handle, self.inner.handle, float(rtol), int(maxit),
             ctypes.byref(h))
        self.pcg = h

    def coarse_stats(self):
        """PCG / GMRES coarse solver statistics (None with a dense coarse inverse): iterations
        of the last solve, solves that stopped at maxit, total iterations, largest final
        relative residual (GMRES: also the number of solves)."""
        if getattr(self, "coarse_gmres", False) and self.handle:
            sv, a, c, b = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
            d = ctypes.c_double()
            call("mlamg_hier_coarse_gmres_stats", self.handle, ctypes.byref(sv), ctypes.byref(a),
                 ctypes.byref(c), ctypes.byref(b), ctypes.byref(d))
            return {"solver": "gmres", "solves": sv.value, "last_iters": a.value,
                    "not_converged": b.value, "total_iters": c.value,
                    "max_rel_residual": d.value, "breakdowns": 0}
        if getattr(self, "pcg", None) is None:
            return None
        a, b, c = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        d = ctypes.c_double()
        e = ctypes.c_int32()
        call("mlamg_pcg_stats", self.pcg, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c),
             ctypes.byref(d), stream_ptr())
        call("mlamg_pcg_breakdowns", self.pcg, ctypes.byref(e), stream_ptr())
        return {"last_iters": a.value, "not_converged": b.value, "total_iters": c.value,
                "max_rel_residual": d.value, "breakdowns": e.value}

    def check_coarse(self):
        """Raise if a PCG coarse solve broke down (A_c or its preconditioner not positive
        definite: the iterate is not a solve of the coarse system). Syncs."""
        if self.pcg is None and not self.coarse_gmres:
            return
        st = self.coarse_stats()
        if st.get("solver") == "gmres":  # a failed solve already ended its call (_gmres_call)
            return
        if st is not None and st["breakdowns"] > self._breakdowns_seen:
            self._breakdowns_seen = st["breakdowns"]
            raise CoarseSolveError(f"PCG coarse solve broke down ({st['breakdowns']} solves): "
                                   "the coarse operator is not positive definite")

    # ------------------------------------------------------------------ cycling
    def _solve_call(self, fn, *args):
        """A C-ABI call that runs this hierarchy's cycles: a GMRES coarse solve that did not
        converge ends it with EINVAL ("did not converge") -> CoarseSolveError (the reference's
        factorisation failure, ns/lib/multigrid.py:167-170)."""
        try:
            return call(fn, *args)
        except MlamgError as e:
            if self.coarse_gmres and "did not converge" in str(e):
                raise CoarseSolveError(str(e)) from None
            raise

    def cycle(self, b, x, n_cycles, tol=None, use_graph=True, history=True):
        """Run up to n_cycles V-cycles in place on x (device tensors). Returns the residual
        history ||b - A x||_2 after each cycle (numpy, truncated at convergence). tol=None runs
        every cycle; a number (0 included) stops after the first cycle whose norm is <= tol."""
        dev = x.device
        hist = torch.zeros(max(n_cycles, 1), dtype=torch.float64, device=dev) if history else None
        done = ctypes.c_int32()
        self._solve_call("mlamg_hier_vcycle", self.handle, ptr(rhs_arg(b)), ptr(x),
                         int(n_cycles), _tol_arg(tol), ptr(hist), ctypes.byref(done),
                         int(bool(use_graph)), stream_ptr())
        self.check_coarse()
        if not history:
            return None
        return hist[: int(done.value)].cpu().numpy()

    def cycle_async(self, b, x, n_cycles, use_graph=True, zero_rhs=None):
        """Launch n_cycles V-cycles without reading anything back (for timing). zero_rhs: None
        = detect an all-zero b (rhs_arg: one reduction and a sync), True / False = as given
        (False streams b even when it is zero: the general-b kernels)."""
        if zero_rhs is None:
            bb = rhs_arg(b)
        else:
            bb = None if zero_rhs else b
            if zero_rhs and b is not None and bool(torch.count_nonzero(b.view(torch.int64))):
                raise ValueError("zero_rhs=True with a nonzero b")
        self._solve_call("mlamg_hier_vcycle", self.handle, ptr(bb), ptr(x), int(n_cycles),
                         _tol_arg(None), None, None, int(bool(use_graph)), stream_ptr())

    def solve(self, b, x0=None, tol=1e-8, maxiter=500, return_history=False):
        """Stationary V-cycle iteration until ||b - A x||_2 <= tol (absolute, MLAMG.py:194);
        tol=None runs all maxiter cycles."""
        bd = to_device_vec(b)
        xd = torch.zeros_like(bd) if x0 is None else to_device_vec(x0).clone()
        hist = self.cycle(bd, xd, maxiter, tol=tol)
        x = xd.cpu().numpy() if not isinstance(b, torch.Tensor) else xd
        return (x, hist) if return_history else x

    def gmres(self, b, x0=None, rtol=1e-5, restart=20, maxiter=None, return_info=False):
        """GMRES on A x = b preconditioned by one V-cycle of this hierarchy (mlamg_gmres:
        scipy.sparse.linalg.gmres's algorithm — left-preconditioned, restarted MGS — with
        ||b - A x|| <= rtol ||b||; the Krylov acceleration of ns/preconditioner/PyAMG.py:119).
        x0=None starts from 0. Returns x (numpy in -> numpy out, tensor in -> tensor out), plus
        {"info", "inner_iters", "presid"} (presid: preconditioned residual estimate / ||b|| per
        Krylov step) with return_info=True."""
        A = self.levels[0].A if self.levels else self.Ac
        bd = to_device_vec(b)
        xd = torch.zeros_like(bd) if x0 is None else to_device_vec(x0).clone()
        n = bd.numel()
        cap = 4096
        hist = (ctypes.c_double * cap)()
        info, inner = ctypes.c_int(), ctypes.c_int()
        self._solve_call("mlamg_gmres", A.handle, self.handle, ptr(bd), ptr(xd), float(rtol),
                         int(restart), int(maxiter or 0), int(x0 is None), ctypes.byref(info),
                         ctypes.byref(inner), hist, cap, stream_ptr())
        self.check_coarse()  # a broken-down coarse solve inside the preconditioner
        x = xd if isinstance(b, torch.Tensor) else xd.cpu().numpy()
        if not return_info:
            return x
        k = min(inner.value, cap)
        return x, {"info": info.value, "inner_iters": inner.value,
                   "presid": np.array(hist[:k])}

    def gmres_householder(self, b, x0=None, tol=1e-5, maxiter=None, return_info=False):
        """pyamg.krylov.gmres(A, b, x0, tol, maxiter, M=one V-cycle) with its default
        Householder orthogonalisation (mlamg_gmres_householder): what pyamg's
        MultilevelSolver.solve(b, tol, accel='gmres') runs (ns/preconditioner/PyAMG.py:119).
        Returns x (numpy in -> numpy out, tensor in -> tensor out), plus {"info", "iters",
        "residuals"} (preconditioned residual norms: initial, per step, final) with
        return_info=True."""
        A = self.levels[0].A if self.levels else self.Ac
        bd = to_device_vec(b)
        xd = torch.zeros_like(bd) if x0 is None else to_device_vec(x0).clone()
        cap = 4096
        hist = (ctypes.c_double * cap)()
        info, iters = ctypes.c_int(), ctypes.c_int()
        self._solve_call("mlamg_gmres_householder", A.handle, self.handle, ptr(bd), ptr(xd),
                         float(tol), int(maxiter or 0), int(x0 is None), ctypes.byref(info),
                         ctypes.byref(iters), hist, cap, stream_ptr())
        self.check_coarse()
        x = xd if isinstance(b, torch.Tensor) else xd.cpu().numpy()
        if not return_info:
            return x
        # recorded: the initial norm, one per step except the last (the budget's last step, or
        # the step whose estimate met tol: pyamg breaks before appending it), the final norm
        it = iters.value
        k = min(1 if it == 0 else it + 1, cap)
        return x, {"info": info.value, "iters": it, "residuals": np.array(hist[:k])}

    def precondition(self, b):
        """One V-cycle from a zero guess: the action of the preconditioner on b."""
        bd = to_device_vec(b)
        xd = torch.zeros_like(bd)
        self.cycle(bd, xd, 1, history=False)
        return xd if isinstance(b, torch.Tensor) else xd.cpu().numpy()

    def cycle_bytes(self, stored=False):
        """Bytes of one V-cycle. stored=False: operators priced as CSR (a
        CSR-equivalent figure); stored=True: priced as stored (the cycle's HBM roofline bytes)."""
        v = ctypes.c_double()
        call("mlamg_hier_cycle_format_bytes" if stored else "mlamg_hier_cycle_bytes",
             self.handle, ctypes.byref(v))
        return float(v.value)

    # ------------------------------------------------------------------ info
    @property
    def n_levels(self):
        return len(self.levels) + 1

    def operator_complexity(self):
        nnz = sum(L.A.nnz for L in self.levels) + self.Ac.nnz
        return nnz / self.levels[0].A.nnz if self.levels else 1.0

    def describe(self):
        rows = []
        for i, L in enumerate(self.levels):
            rows.append({"level": i, "n": L.A.shape[0], "nnz": L.A.nnz,
                         "P_nnz": L.P.nnz, "omega": L.omega, "lambda_max": L.lam,
                         "lanczos_iters": L.lanczos_iters, "bf_sweeps": L.bf_sweeps})
        rows.append({"level": len(self.levels), "n": self.Ac.shape[0], "nnz": self.Ac.nnz,
                     "coarse": "dense inverse" if self.dense is not None
                     else ("GMRES, inner SA hierarchy" if self.coarse_gmres
                           else "PCG, inner SA hierarchy")})
        return rows

    def __del__(self):
        for attr, fn in (("handle", "mlamg_hier_destroy"), ("dense", "mlamg_dense_destroy"),
                         ("pcg", "mlamg_pcg_destroy")):
            h = getattr(self, attr, None)
            if h:
                try:
                    getattr(_lib.lib, fn)(h)
                except Exception:
                    pass
                setattr(self, attr, None)
