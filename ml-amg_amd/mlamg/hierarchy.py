"""Device AMG hierarchy: setup on the GPU and the V-cycle executor (mlamg_hier_*).

Setup per level follows the reference's aggregation-based SA recipe, all on the device:
  C = strength(A)                                    utils/common.py:25-31 ('invabs', 'abs', 'unit')
  seeds = RandomState(seed).permutation(n)[:ceil(alpha*n)]       graph.py:230-231; evaluate_dataset.py:80-85
  (dist, label) = Bellman-Ford(C, seeds)            graph.py:7-53   (or Lloyd: graph.py:156-239)
  Agg = aggregate operator(label)                   graph.py:56-86
  omega = (4/3)/lambda_max(Dinv A);  P = (I - omega Dinv A) Agg    multigrid.py:102-108
  R = P^T;  A_c = (R A) P                            multigrid.py:165
until n <= max_coarse; the last operator is inverted densely (multigrid.py:168 factorized).
The cycle is the Jacobi V(1,1) of ns/preconditioner/MLAMG.py:143-197 applied recursively.

Seeds are drawn on the host with numpy's RandomState for bit-exact reproducibility against the
reference seeding; with sort_seeds=True (default for the multilevel solver) they are sorted so that
coarse unknowns follow the fine ordering (better locality, contiguous ownership per GPU).
"""
from __future__ import annotations

import ctypes
import math
import time

import numpy as np
import torch

from . import _lib
from ._lib import MLAMG_EUNSUPPORTED, MlamgError, _tol_arg, call, ptr, stream_ptr
from .graph import aggregate_op_device, bellman_ford_device, labels_to_columns, lloyd_cluster_device
from .multigrid import lambda_max_dinv_a
from .sparse import DeviceCSR, _device, as_device, galerkin, to_device_vec

STRENGTH_MODES = {"abs": 0, "invabs": 1, "unit": 2, "same": 3}


def strength(A_dev, mode="invabs"):
    h = ctypes.c_void_p()
    call("mlamg_strength", A_dev.handle, STRENGTH_MODES[mode], ctypes.byref(h), stream_ptr())
    return DeviceCSR(h)


class Level:
    __slots__ = ("A", "dinv", "P", "R", "Agg", "omega", "lam", "lanczos_iters", "n_seeds",
                 "bf_sweeps", "seeds", "gs")

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


class Hierarchy:
    """A multilevel (or two-level) smoothed-aggregation hierarchy resident on the GPU."""

    def __init__(self):
        self.levels = []
        self.Ac = None
        self.dense = None
        self.handle = None
        self.jacobi_weight = 2.0 / 3.0
        self.nu_pre = 1
        self.nu_post = 1
        self.timings = {}

    # ------------------------------------------------------------------ construction
    @classmethod
    def two_level(cls, A, P, omega=2.0 / 3.0, nu_pre=1, nu_post=1, dinv_w=None,
                  smoother="jacobi", norm="residual"):
        """Two-level cycle with a given P: MLAMG.amg_2_v (ns/preconditioner/MLAMG.py:120-122,
        smoother='jacobi') or multigrid.amg_2_v (multigrid.py:111-210, smoother='gauss_seidel';
        norm='x' records ||x||_2 per cycle, the error_tol mode)."""
        from .multigrid import GaussSeidel
        H = cls()
        H.jacobi_weight = omega
        L = Level(as_device(A))
        L.P = as_device(P)
        L.R = L.P.transpose()
        L.dinv = L.A.diag_inv(omega) if dinv_w is None else to_device_vec(dinv_w)
        H.levels.append(L)
        H.Ac = galerkin(L.R, L.A, L.P)
        H._finalize(nu_pre, nu_post)
        if smoother == "gauss_seidel":
            L.gs = GaussSeidel(L.A)
            call("mlamg_hier_set_level_smoother", H.handle, 0, L.gs.handle)
        elif smoother != "jacobi":
            raise ValueError(f"unknown smoother {smoother!r}")
        if norm not in ("residual", "x"):
            raise ValueError(f"unknown norm {norm!r}")
        call("mlamg_hier_set_norm", H.handle, 0 if norm == "residual" else 1)
        return H

    EXACT_CANDIDATES = (("csr_stream", 0), ("sell", 1), ("sell", 512), ("sorted", 0),
                        ("sell_dict", 1), ("sell_dict", 512), ("rowpat", 0))
    VECTOR_CANDIDATES = (("vector", 8), ("vector", 16), ("vector", 32), ("vector", 64),
                         ("vector", 128), ("vector", 256), ("vector", 512))

    @staticmethod
    def _time_format(M, fmt, arg, x, y, reps=5, kind="A"):
        """Average time of M's cycle operation in format fmt: the residual epilogue for A
        (r = b - A x, as in the cycle; here b = y), y += M x for P, y = M x for R."""
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
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            op()
        e1.record(s)
        e1.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3  # us

    def apply_formats(self, fine_format="autotune", coarse_format="vector", vec_min_row=16):
        """Choose the SpMV kernel of every operator.

        Level-0 operators (A0, P0, R0: the ones with a scipy counterpart in the reference
        cycle) always keep scipy's summation order: CSR-stream, SELL-64, SELL-64-sigma or
        gather-sorted CSR-stream, all bitwise scipy. Coarser levels (the multilevel extension, no reference counterpart) may
        also use the CSR-vector kernel for A_l and R_l when coarse_format='vector' and their
        mean row length is >= vec_min_row; its fixed order is restated by the oracle.
        fine_format='autotune' times every admissible kernel on each operator once and keeps
        the fastest (results in self.tuning); any other value forces that format."""
        self.tuning = []
        dev = torch.device("cuda", torch.cuda.current_device())
        for i, L in enumerate(self.levels):
            row = {}
            for name, M in (("A", L.A), ("P", L.P), ("R", L.R)):
                cands = list(self.EXACT_CANDIDATES)
                if (i > 0 and name in ("A", "R") and coarse_format == "vector"
                        and M.nnz >= vec_min_row * M.shape[0]):
                    cands += list(self.VECTOR_CANDIDATES)
                if fine_format != "autotune":
                    M.set_format(fine_format if fine_format != "vector" else "auto_exact")
                    row[name] = {"chosen": M.get_format()[:2]}
                    continue
                x = torch.randn(M.shape[1], dtype=torch.float64, device=dev)
                y = torch.zeros(M.shape[0], dtype=torch.float64, device=dev)
                times = {}
                for fmt, arg in cands:
                    try:
                        times[f"{fmt}/{arg}"] = self._time_format(M, fmt, arg, x, y,
                                                                  kind=name)
                    except MlamgError as e:  # format limits (e.g. sorted: row > 4096 nnz)
                        if e.code != MLAMG_EUNSUPPORTED:
                            raise
                best = min(times, key=times.get)
                fmt, arg = best.split("/")
                M.set_format(fmt, int(arg))
                row[name] = {"chosen": best, "us": {k: round(v, 2) for k, v in times.items()}}
            self.tuning.append(row)
        self.attach_dinvs()

    def attach_dinvs(self):
        """Let every rowpat level operator take its Jacobi weights from its pattern table."""
        for L in self.levels:
            if L.A.get_format()[0] == "rowpat":
                L.A.attach_dinv(L.dinv)

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
              fine_format="autotune", coarse_format="vector", verbose=False, finalize=True):
        H = cls()
        H.jacobi_weight = jacobi_weight
        t_all = time.perf_counter()
        A_dev = as_device(A)
        tm = {"aggregation": 0.0, "lambda_max": 0.0, "prolongator": 0.0, "galerkin": 0.0,
              "formats": 0.0, "dense": 0.0}
        while True:
            n = A_dev.shape[0]
            if n <= max_coarse or len(H.levels) + 1 >= max_levels:
                break
            L = Level(A_dev)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            C = strength(A_dev, strength_mode)
            k = int(math.ceil(alpha * n))
            seeds = np.random.RandomState(seed).permutation(n)[:k]
            if sort_seeds:
                seeds = np.sort(seeds)
            L.seeds = seeds
            seeds_dev = torch.as_tensor(seeds.astype(np.int32)).to(_device())
            if aggregation == "bellman_ford":
                _, lab, L.bf_sweeps = bellman_ford_device(C, seeds_dev)
                col = labels_to_columns(lab, seeds_dev)
            elif aggregation == "lloyd":
                _, col, _, L.bf_sweeps = lloyd_cluster_device(C, seeds_dev, lloyd_maxiter)
            else:
                raise ValueError(f"unknown aggregation {aggregation!r}")
            L.Agg = aggregate_op_device(col, k)
            L.n_seeds = k
            del C
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            L.lam, L.lanczos_iters = lambda_max_dinv_a(A_dev, max_iter=lanczos_iter, tol=lanczos_tol)
            L.omega = (4.0 / 3.0) / abs(L.lam)
            t2 = time.perf_counter()
            h = ctypes.c_void_p()
            call("mlamg_sa_smoother", A_dev.handle, float(L.omega), ctypes.byref(h), stream_ptr())
            S = DeviceCSR(h)
            L.P = S @ L.Agg
            del S
            L.R = L.P.transpose()
            L.dinv = A_dev.diag_inv(jacobi_weight)
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            A_next = galerkin(L.R, A_dev, L.P)
            torch.cuda.synchronize()
            t4 = time.perf_counter()
            tm["aggregation"] += t1 - t0
            tm["lambda_max"] += t2 - t1
            tm["prolongator"] += t3 - t2
            tm["galerkin"] += t4 - t3
            H.levels.append(L)
            if verbose:
                print(f"[mlamg] level {len(H.levels) - 1}: n={n} nnz={A_dev.nnz} seeds={k} "
                      f"bf_sweeps={L.bf_sweeps} lam={L.lam:.15g} ({L.lanczos_iters} it) "
                      f"P nnz={L.P.nnz} -> n_c={A_next.shape[0]} nnz_c={A_next.nnz} "
                      f"[agg {t1 - t0:.2f}s lam {t2 - t1:.2f}s P {t3 - t2:.2f}s gal {t4 - t3:.2f}s]",
                      flush=True)
            A_dev = A_next
        H.Ac = A_dev
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

    def _finalize(self, nu_pre, nu_post):
        self.nu_pre, self.nu_post = nu_pre, nu_post
        h = ctypes.c_void_p()
        call("mlamg_dense_create", self.Ac.handle, ctypes.byref(h), stream_ptr())
        self.dense = h
        hh = ctypes.c_void_p()
        call("mlamg_hier_create", ctypes.byref(hh))
        self.handle = hh
        for L in self.levels:
            call("mlamg_hier_add_level", hh, L.A.handle, ptr(L.dinv), L.P.handle, L.R.handle)
        call("mlamg_hier_set_coarse", hh, self.Ac.handle, self.dense)
        call("mlamg_hier_set_smoothing", hh, int(nu_pre), int(nu_post))

    # ------------------------------------------------------------------ cycling
    def cycle(self, b, x, n_cycles, tol=None, use_graph=True, history=True):
        """Run up to n_cycles V-cycles in place on x (device tensors). Returns the residual
        history ||b - A x||_2 after each cycle (numpy, truncated at convergence). tol=None runs
        every cycle; a number (0 included) stops after the first cycle whose norm is <= tol."""
        dev = x.device
        hist = torch.zeros(max(n_cycles, 1), dtype=torch.float64, device=dev) if history else None
        done = ctypes.c_int32()
        call("mlamg_hier_vcycle", self.handle, ptr(b), ptr(x), int(n_cycles), _tol_arg(tol),
             ptr(hist), ctypes.byref(done), int(bool(use_graph)), stream_ptr())
        if not history:
            return None
        return hist[: int(done.value)].cpu().numpy()

    def cycle_async(self, b, x, n_cycles, use_graph=True):
        """Launch n_cycles V-cycles without reading anything back (for timing)."""
        call("mlamg_hier_vcycle", self.handle, ptr(b), ptr(x), int(n_cycles), _tol_arg(None),
             None, None, int(bool(use_graph)), stream_ptr())

    def solve(self, b, x0=None, tol=1e-8, maxiter=500, return_history=False):
        """Stationary V-cycle iteration until ||b - A x||_2 <= tol (absolute, MLAMG.py:194);
        tol=None runs all maxiter cycles."""
        bd = to_device_vec(b)
        xd = torch.zeros_like(bd) if x0 is None else to_device_vec(x0).clone()
        hist = self.cycle(bd, xd, maxiter, tol=tol)
        x = xd.cpu().numpy() if not isinstance(b, torch.Tensor) else xd
        return (x, hist) if return_history else x

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
                     "coarse": "dense inverse"})
        return rows

    def __del__(self):
        for attr, fn in (("handle", "mlamg_hier_destroy"), ("dense", "mlamg_dense_destroy")):
            h = getattr(self, attr, None)
            if h:
                try:
                    getattr(_lib.lib, fn)(h)
                except Exception:
                    pass
                setattr(self, attr, None)
