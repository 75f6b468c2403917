"""Drop-in mirror of ns/lib/multigrid.py running on the MI355X.

Same names, argument meaning, return values and error behaviour as the reference; every sparse
operation runs in libmlamg_hip (HIP kernels for gfx950). scipy matrices / numpy vectors go in and
come out, like the reference; `DeviceCSR` operands and torch cuda tensors are also accepted.

  jacobi                     ns/lib/multigrid.py:15-45
  gauss_seidel               ns/lib/multigrid.py:58-90 (pyamg gauss_seidel order)
  smoothed_aggregation_jacobi ns/lib/multigrid.py:102-108
  amg_2_v                    ns/lib/multigrid.py:111-210
  jacobi_torch, gauss_seidel_torch, amg_2_v_torch   ns/lib/multigrid.py:48,93,213 (torch ops as
                             in the reference; not on the V-cycle path)
"""
from __future__ import annotations

import ctypes

import numpy as np
import scipy.sparse as sp
import torch

from . import _lib
from ._lib import call, ptr, stream_ptr
from .sparse import DeviceCSR, as_device, galerkin, to_device_vec


def _as_numpy_out(x_dev, like):
    out = x_dev.cpu().numpy()
    if isinstance(like, np.ndarray):
        like[...] = out
        return like
    return out


def _dinv_vector(A_dev, Dinv):
    """Diagonal of the reference's Dinv argument as a device vector (fl(1/a_ii))."""
    if Dinv is None:
        return A_dev.diag_inv(1.0)
    if sp.issparse(Dinv):
        d = np.asarray(Dinv.diagonal(), dtype=np.float64)
    else:
        d = np.asarray(Dinv, dtype=np.float64)
        if d.ndim == 2:
            d = np.diagonal(d).copy()
    return to_device_vec(d)


def _scale(d, omega):
    # `omega * Dinv` scales the dia data: fl(omega * d)
    return d * omega


def jacobi(A, b, x, Dinv=None, omega=0.666, nu=2):
    """Weighted Jacobi, ns/lib/multigrid.py:15-45:  x += w*Dinv@b - ((w*Dinv)@A)@x, nu times.

    The explicit product (w*Dinv)@A is formed on the device with scipy's row order, so the
    result is bitwise the reference's. x (numpy) is updated in place and returned.
    """
    A_dev = as_device(A)
    d = _dinv_vector(A_dev, Dinv)
    dw = _scale(d, omega)
    h = ctypes.c_void_p()
    call("mlamg_csr_scale_rows", A_dev.handle, ptr(dw), 1, ctypes.byref(h), stream_ptr())
    M = DeviceCSR(h)
    xd = to_device_vec(x)
    bd = to_device_vec(b)
    tmp = torch.empty_like(xd)
    call("mlamg_jacobi_explicit", M.handle, ptr(dw), ptr(bd), ptr(xd), ptr(tmp), int(nu),
         stream_ptr())
    if isinstance(x, torch.Tensor):
        x.copy_(xd)
        return x
    return _as_numpy_out(xd, x)


class GaussSeidel:
    """Level-scheduled Gauss-Seidel: pyamg relaxation.gauss_seidel semantics (block=False, the
    reference driver's forward sweep), or relaxation.block_gauss_seidel with 1 x 1 blocks
    (block=True: pyamg's smoothed-aggregation smoother). sweep: 'forward', 'backward' or
    'symmetric' (forward then backward, per iteration)."""

    SWEEPS = {"forward": 0, "backward": 1, "symmetric": 2}

    def __init__(self, A_dev, sweep="forward", block=False):
        if sweep not in self.SWEEPS:
            raise ValueError("valid sweep directions are 'forward', 'backward', and 'symmetric'")
        self.A = A_dev
        self.sweep_dir = sweep
        self.block = bool(block)
        h = ctypes.c_void_p()
        call("mlamg_gs_create_ex", A_dev.handle, self.SWEEPS[sweep], int(self.block),
             ctypes.byref(h), stream_ptr())
        self.handle = h
        n = ctypes.c_int32()
        call("mlamg_gs_levels", h, ctypes.byref(n))
        self.n_levels = int(n.value)

    def sweep(self, x, b, iterations=1):
        call("mlamg_gs_sweep", self.handle, ptr(x), ptr(b), int(iterations), stream_ptr())
        return x

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            try:
                _lib.lib.mlamg_gs_destroy(h)
            except Exception:
                pass
            self.handle = None


def gauss_seidel(A, b, x, L=None, U=None, nu=2):
    """Gauss-Seidel, ns/lib/multigrid.py:58-90 (nu forward sweeps; L/U are ignored)."""
    A_dev = as_device(A)
    gs = GaussSeidel(A_dev)
    xd = to_device_vec(x)
    bd = to_device_vec(b)
    gs.sweep(xd, bd, nu)
    out = xd.cpu().numpy()
    return out


def lambda_max_dinv_a(A, max_iter=20000, tol=1e-15, seed=0):
    """Largest eigenvalue of Dinv@A (ARPACK eigs k=1 'LM' at ns/lib/multigrid.py:105)."""
    A_dev = as_device(A)
    lam = ctypes.c_double()
    its = ctypes.c_int()
    call("mlamg_lambda_max_dinvA", A_dev.handle, int(max_iter), float(tol), int(seed),
         ctypes.byref(lam), ctypes.byref(its), stream_ptr())
    return float(lam.value), int(its.value)


def sa_omega(A, **kw):
    lam, _ = lambda_max_dinv_a(A, **kw)
    return (4.0 / 3.0) / abs(lam)


def smoothed_aggregation_jacobi_device(A_dev, Agg_dev, omega=None):
    """P = (I - omega*Dinv@A) @ Agg on the device; omega = (4/3)/lambda_max(Dinv@A)."""
    if omega is None:
        omega = sa_omega(A_dev)
    h = ctypes.c_void_p()
    call("mlamg_sa_smoother", A_dev.handle, float(omega), ctypes.byref(h), stream_ptr())
    S = DeviceCSR(h)
    return S @ Agg_dev, omega


def smoothed_aggregation_jacobi(A, Agg):
    """ns/lib/multigrid.py:102-108; returns a scipy CSR like the reference."""
    A_dev = as_device(A)
    Agg_dev = as_device(sp.csr_matrix(Agg, dtype=np.float64) if sp.issparse(Agg) else Agg)
    P, _ = smoothed_aggregation_jacobi_device(A_dev, Agg_dev)
    return P.to_scipy()


def conv_factor(err):
    """Convergence-factor formula of ns/lib/multigrid.py:201-208, quirks included."""
    if len(err) != 1:
        try:
            err_n = min(len(err) // 3, 10)
            conv = (err[-1] / err[-err_n]) ** (1 / (err_n - 1))
        except Exception:  # the reference's bare except: divide by zero, empty history
            conv = 0
    else:
        conv = 0
    return conv


class TwoLevel:
    """Device state of one amg_2_v call: A, P, R = P^T, A_H = (R@A)@P and its dense inverse."""

    def __init__(self, A, P):
        self.A = as_device(A)
        self.P = as_device(P)
        self.R = self.P.transpose()
        self.A_H = galerkin(self.R, self.A, self.P)
        h = ctypes.c_void_p()
        call("mlamg_dense_create", self.A_H.handle, ctypes.byref(h), stream_ptr())
        self.dense = h
        self.n = self.A.shape[0]
        self.nc = self.P.shape[1]

    def coarse_correct(self, x, b, r, rc, ec):
        """x += P @ A_H^-1 (P.T @ (b - A@x))  (ns/lib/multigrid.py:181)."""
        s = stream_ptr()
        call("mlamg_residual", self.A.handle, ptr(b), ptr(x), ptr(r), None, s)
        call("mlamg_restrict", self.R.handle, ptr(r), ptr(rc), s)
        call("mlamg_dense_solve", self.dense, ptr(rc), ptr(ec), s)
        call("mlamg_prolong_add", self.P.handle, ptr(ec), ptr(x), s)

    def __del__(self):
        h = getattr(self, "dense", None)
        if h:
            try:
                _lib.lib.mlamg_dense_destroy(h)
            except Exception:
                pass
            self.dense = None


def lsqr(A, b, atol=1e-6, btol=1e-6, conlim=1e8, iter_lim=None, AT=None):
    """scipy.sparse.linalg.lsqr(A, b)[:3] (damp = 0, x0 = 0) on the device: (x, istop, itn).

    A and b may be scipy/numpy or device objects; AT (optional DeviceCSR) is A's transpose, the
    operator of scipy's rmatvec. x comes back as a device tensor when b is one, else numpy."""
    A_dev = as_device(A)
    AT = A_dev.transpose() if AT is None else AT
    bd = to_device_vec(b)
    xd = torch.empty(A_dev.shape[1], dtype=torch.float64, device=bd.device)
    istop, itn = ctypes.c_int(), ctypes.c_int()
    call("mlamg_lsqr", A_dev.handle, AT.handle, ptr(bd), ptr(xd), float(atol), float(btol),
         float(conlim), int(iter_lim or 0), ctypes.byref(istop), ctypes.byref(itn), stream_ptr())
    x = xd if isinstance(b, torch.Tensor) else xd.cpu().numpy()
    return x, int(istop.value), int(itn.value)


def _amg_2_v_singular(A, P, b, x, nu_pre, nu_post, jacobi_weight, res_tol, tol, max_iter,
                      smoother):
    """The singular branch of ns/lib/multigrid.py:111-210 (Neumann problems, constant
    nullspace): coarse correction x += P @ lsqr(P.T@A@P, P.T@(b - A@x))[0] (:178-179), mean
    removal after post-smoothing (:186-187), no factorization. Device-resident; one host read of
    the norm per cycle for the tolerance test."""
    A_dev, P_dev = as_device(A), as_device(P)
    R = P_dev.transpose()
    A_H = galerkin(R, A_dev, P_dev)
    A_HT = A_H.transpose()
    s = stream_ptr()
    xd = to_device_vec(x).clone()  # x = x.copy()  (:171)
    bd = to_device_vec(b)
    n, nc = A_dev.shape[0], P_dev.shape[1]
    r = torch.empty(n, dtype=torch.float64, device=xd.device)
    t = torch.empty_like(r)
    rc = torch.empty(nc, dtype=torch.float64, device=xd.device)
    ec = torch.empty_like(rc)
    nrm = torch.zeros(1, dtype=torch.float64, device=xd.device)
    istop, itn = ctypes.c_int(), ctypes.c_int()
    if smoother == "gauss_seidel":
        gs = GaussSeidel(A_dev)

        def smooth(nu):
            if nu > 0:
                gs.sweep(xd, bd, nu)
    else:
        dw = A_dev.diag_inv(jacobi_weight)

        def smooth(nu):
            if nu > 0:
                call("mlamg_jacobi", A_dev.handle, ptr(dw), ptr(bd), ptr(xd), ptr(t), int(nu), s)
    err = np.zeros(max_iter)
    for i in range(max_iter):
        smooth(nu_pre)
        call("mlamg_residual", A_dev.handle, ptr(bd), ptr(xd), ptr(r), None, s)
        call("mlamg_restrict", R.handle, ptr(r), ptr(rc), s)
        call("mlamg_lsqr", A_H.handle, A_HT.handle, ptr(rc), ptr(ec), 1e-6, 1e-6, 1e8, 0,
             ctypes.byref(istop), ctypes.byref(itn), s)
        call("mlamg_prolong_add", P_dev.handle, ptr(ec), ptr(xd), s)
        smooth(nu_post)
        call("mlamg_remove_mean", ptr(xd), int(n), s)
        if res_tol is not None:
            call("mlamg_residual", A_dev.handle, ptr(bd), ptr(xd), ptr(r), ptr(nrm), s)
        else:
            call("mlamg_norm2", ptr(xd), int(n), ptr(nrm), s)
        e = float(nrm.item())
        err[i] = e
        if e <= tol:
            err = err[:i + 1]
            break
    return xd.cpu().numpy(), conv_factor(err), err, len(err)


_BATCH_LIMITS = None


def _batch_limits():
    global _BATCH_LIMITS
    if _BATCH_LIMITS is None:
        n, nc, k = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int()
        call("mlamg_amg2v_batch_limits", ctypes.byref(n), ctypes.byref(nc), ctypes.byref(k))
        _BATCH_LIMITS = (int(n.value), int(nc.value), int(k.value))
    return _BATCH_LIMITS


_CSR_TYPES = (sp.csr_matrix,) + ((sp.csr_array,) if hasattr(sp, "csr_array") else ())
_F64, _I32 = np.dtype(np.float64), np.dtype(np.int32)


def _fused_arrays(A, P, b, x, max_nc=None):
    """The fused solver's host arrays of one amg_2_v problem, or None outside its limits:
    (n, n_c, [A.indptr, A.indices, A.data, P.indptr, P.indices, P.data, b, x]) with int32
    indices, fp64 values, C-contiguous, A's rows duplicate-free in their stored order.
    Canonical int32 / fp64 CSR inputs (what the reference's generators produce) are used as
    they are, without copies."""
    from .sparse import canonical_rows
    if not (sp.issparse(A) and sp.issparse(P)):
        return None
    max_n, lim_nc, _ = _batch_limits()
    max_nc = lim_nc if max_nc is None else min(max_nc, lim_nc)
    n, m = A.shape
    n2, nc = P.shape
    if not (n == m == n2 and 1 <= n <= max_n and 1 <= nc <= max_nc and nc <= n):
        return None
    if A.__class__ not in _CSR_TYPES or not A.has_canonical_format:
        A = canonical_rows(A)
    if P.__class__ not in _CSR_TYPES:
        P = sp.csr_matrix(P)
    if A.nnz >= 2**31 or P.nnz >= 2**31:
        return None
    arrs = []
    for v, dt in ((A.indptr, _I32), (A.indices, _I32), (A.data, _F64), (P.indptr, _I32),
                  (P.indices, _I32), (P.data, _F64)):
        if v.dtype != dt or not v.flags.c_contiguous:
            v = np.ascontiguousarray(v, dtype=dt)
        arrs.append(v)
    for v in (b, x):
        if (v.__class__ is not np.ndarray or v.dtype != _F64 or v.ndim != 1
                or not v.flags.c_contiguous):
            v = np.ascontiguousarray(np.asarray(v, dtype=np.float64).ravel())
        if v.size != n:
            raise ValueError(f"amg_2_v: vector of size {v.size} for a system of {n} rows")
        arrs.append(v)
    return n, nc, arrs


# Engine choice for engine='auto' (measured on MI355X, profiles/r02/amg2v_timing.json): one
# workgroup runs a whole fused solve's smoothing and transfers, so a single call pays its serial
# sweep levels alone. Single calls with n_c > 300 factor the coarse operator on the whole GPU
# (csrc/dense.hip) and run phased cycles, whose coarse solve is spread over every CU. The fused
# engine then beats the per-operation hierarchy engine at every size the batched solver takes
# (32^2: 1.8 vs 5.9 ms; 64^2, n_c = 484: 4.1 vs 9.4 ms; 96^2, n_c = 1024: 9.3 vs 13.9 ms;
# 128^2, n_c = 1849: 19.8 vs 20.4 ms). In a batch the problems run side by side on the CUs, so
# up to n_c = 1024 the fused launch wins by a wide margin (48 grids 32^2-64^2: 8.8 ms vs 190 ms
# for 16 threads of the hierarchy engine).
FUSED_SINGLE_MAX_NC = 2048
FUSED_BATCH_MAX_NC = 1024


def _amg_2_v_fused(prepared, xs, pre, post, jacobi_weight, res_tol, error_tol, max_iter,
                   smoother):
    """Run amg_2_v on every problem of `prepared` (_fused_arrays outputs; xs the caller's initial
    guesses) in ONE device launch (csrc/batch.hip): one workgroup per problem does its Galerkin
    product, coarse inverse, cycles and tolerance test. Returns a list of (x, conv_factor, err,
    iters), or None when a problem is outside the kernel's limits (the caller then takes the
    hierarchy path)."""
    from ._hostptr import data_ptrs
    tol = res_tol if res_tol is not None else error_tol
    count = len(prepared)
    rec = np.zeros(count, dtype=_lib.AMG2V_DTYPE)  # mlamg_amg2v_problem[count], filled by column
    # the eight host buffers of every problem, their addresses in one call
    flat = [a for _, _, arrs in prepared for a in arrs]
    ptrs = np.empty(8 * count, dtype=np.uint64)
    data_ptrs(flat, ptrs)
    ptrs = ptrs.reshape(count, 8)
    for c, k in enumerate(("A_indptr", "A_indices", "A_data", "P_indptr", "P_indices", "P_data",
                           "b", "x0")):
        rec[k] = ptrs[:, c]
    ns = np.fromiter((p[0] for p in prepared), dtype=np.int64, count=count)
    rec["n"] = ns
    rec["n_c"] = np.fromiter((p[1] for p in prepared), dtype=np.int64, count=count)
    rec["A_nnz"] = np.fromiter((p[2][1].size for p in prepared), dtype=np.int64, count=count)
    rec["P_nnz"] = np.fromiter((p[2][4].size for p in prepared), dtype=np.int64, count=count)
    # outputs: one block for every x and one for every history
    xoff = np.zeros(count + 1, dtype=np.int64)
    np.cumsum(ns, out=xoff[1:])
    xbuf = np.empty(int(xoff[-1]))
    hlen = max(max_iter, 1)
    ebuf = np.empty((count, hlen))
    rec["x_out"] = xbuf.ctypes.data + 8 * xoff[:-1]
    rec["err_out"] = ebuf.ctypes.data + 8 * hlen * np.arange(count, dtype=np.int64)
    rc = _lib.lib.mlamg_amg2v_batch(rec.ctypes.data, count,
                                    0 if smoother == "gauss_seidel" else 1,
                                    int(pre), int(post), float(jacobi_weight),
                                    0 if res_tol is not None else 1, float(tol), int(max_iter),
                                    stream_ptr())
    del flat
    if rc == _lib.MLAMG_EUNSUPPORTED:
        return None
    _lib.check(rc, "mlamg_amg2v_batch")
    res = []
    status = rec["status_out"].tolist()
    iters = rec["iters_out"].tolist()
    xo = xoff.tolist()
    for q in range(count):
        if status[q] == 1:  # factorisation failure: multigrid.py:167-170
            res.append((xs[q], np.float64(1.), np.zeros(max_iter), 0))
            continue
        err = ebuf[q, :min(iters[q], max_iter)].copy()
        res.append((xbuf[xo[q]:xo[q + 1]], conv_factor(err), err, len(err)))
    return res


def amg_2_v(A, P, b, x,
            pre_smoothing_steps=1,
            post_smoothing_steps=1,
            jacobi_weight=0.666,
            res_tol=None,
            error_tol=None,
            max_iter=500,
            singular=False,
            *, smoother="gauss_seidel", use_graph=True, engine="auto"):
    """Two-level AMG solver, ns/lib/multigrid.py:111-210, on the GPU.

    smoother='gauss_seidel' (reference default: pyamg forward GS, :175,184) or 'jacobi'
    (weighted Jacobi x += w*Dinv(b - A x) with w = jacobi_weight, the MLAMG.py:143-146 form).
    Returns (x, conv_factor, err, num_iterations) exactly like the reference.

    engine='auto' runs problems within mlamg_amg2v_batch_limits (the reference's small-grid
    calls) as ONE fused device launch (csrc/batch.hip) and larger ones through a device
    Hierarchy (one kernel per operation; the coarse solve switches to PCG past
    Hierarchy.DENSE_MAX rows); 'fused' / 'hierarchy' force one of them. use_graph=False
    (hierarchy engine) launches the cycles eagerly instead of replaying a captured hipGraph.
    """
    if res_tol is None and error_tol is None:
        raise RuntimeError('One of res_tol or error_tol must be set!')
    tol = res_tol if res_tol is not None else error_tol
    if smoother not in ("gauss_seidel", "jacobi"):
        raise ValueError(f"unknown smoother {smoother!r}")
    if engine not in ("auto", "fused", "hierarchy"):
        raise ValueError(f"unknown engine {engine!r}")
    from . import broker
    if broker.enabled() and engine == "auto":
        # MLAMG_BROKER=1: the call goes to this GPU's broker process, which coalesces the calls
        # of concurrent worker processes into fused batch launches (mlamg/broker.py)
        def num(v):
            return None if v is None else float(v)
        return broker.solve(A, P, b, x, {
            "pre_smoothing_steps": int(pre_smoothing_steps),
            "post_smoothing_steps": int(post_smoothing_steps),
            "jacobi_weight": float(jacobi_weight), "res_tol": num(res_tol),
            "error_tol": num(error_tol), "max_iter": int(max_iter), "singular": bool(singular),
            "smoother": smoother})
    prep = None
    if engine != "hierarchy" and not singular:
        prep = _fused_arrays(A, P, b, x, None if engine == "fused" else FUSED_SINGLE_MAX_NC)
    if prep is not None:
        out = _amg_2_v_fused([prep], [x], pre_smoothing_steps, post_smoothing_steps,
                             jacobi_weight, res_tol, error_tol, max_iter, smoother)
        if out is not None:
            return out[0]
    if engine == "fused":
        raise ValueError("problem outside the fused solver's limits (mlamg_amg2v_batch_limits)")
    if singular:
        return _amg_2_v_singular(A, P, b, x, pre_smoothing_steps, post_smoothing_steps,
                                 jacobi_weight, res_tol, tol, max_iter, smoother)
    from .hierarchy import CoarseSolveError, Hierarchy

    def run(coarse):
        # the whole solve is one device call: cycles replayed from a captured graph, the
        # norm and tolerance test on the device (no host round trip per iteration)
        H = Hierarchy.two_level(A, P, omega=jacobi_weight, nu_pre=pre_smoothing_steps,
                                nu_post=post_smoothing_steps, smoother=smoother,
                                norm="residual" if res_tol is not None else "x", coarse=coarse)
        dev_x = to_device_vec(x).clone()  # x = x.copy()  (:171)
        dev_b = to_device_vec(b)
        err = H.cycle(dev_b, dev_x, max_iter, tol=tol, use_graph=use_graph)  # stops at e <= tol
        return dev_x.cpu().numpy(), conv_factor(err), err, len(err)

    failed = (x, np.float64(1.), np.zeros(max_iter), 0)  # multigrid.py:167-170
    try:
        return run("auto")
    except _lib.MlamgError as e:
        if e.code == _lib.MLAMG_EINVAL and "singular" in str(e):
            return failed  # the dense factorisation failed, as spla.factorized would
        raise
    except CoarseSolveError:
        pass
    # The PCG coarse solve broke down: A_H is not positive definite. SuperLU (the reference's
    # factorisation) solves any nonsingular A_H, so the coarse operator is inverted densely
    # instead (Gauss-Jordan with partial pivoting when it is not SPD) and the solve rerun, or,
    # beyond the dense solver's size, solved by GMRES with an inner hierarchy (to 1e-14
    # relative). The reference's failure return when the factorisation fails or GMRES does not
    # converge (no CoarseSolveError escapes — a dataset loop over amg_2_v expects the
    # (x, 1.0, zeros, 0) tuple, not an exception)
    try:
        return run("dense")
    except CoarseSolveError:
        pass
    except _lib.MlamgError as e:
        if e.code == _lib.MLAMG_EINVAL and "singular" in str(e):
            return failed
        raise
    try:
        return run("gmres")
    except CoarseSolveError:
        return failed


def amg_2_v_batch(problems, workers=8, **kw):
    """Many independent amg_2_v solves at once on one GPU — the reference's task farm
    (ns/parallel/pool.py:139-186: one grid per worker process, e.g. utils/evaluate_dataset.py
    over a dataset) as host threads sharing the device, each on its own HIP stream (the C calls
    release the GIL; scratch buffers are per thread), so the small latency-bound solves overlap.

    problems: iterable of (A, P, b, x) tuples; keyword arguments as amg_2_v. Returns the list of
    (x, conv_factor, err, num_iterations) in input order, each equal to a sequential amg_2_v.

    Problems within the fused solver's limits (all of the reference's small-grid datasets) run
    together in ONE launch, one workgroup each (csrc/batch.hip); the rest go through the
    threaded per-problem path below."""
    import threading
    from concurrent.futures import ThreadPoolExecutor
    problems = list(problems)
    engine = kw.pop("engine", "auto")
    if engine != "hierarchy" and problems:
        opts = dict(pre_smoothing_steps=1, post_smoothing_steps=1, jacobi_weight=0.666,
                    res_tol=None, error_tol=None, max_iter=500, singular=False,
                    smoother="gauss_seidel")
        unknown = set(kw) - set(opts) - {"use_graph"}
        if unknown:
            raise TypeError(f"unexpected keyword arguments {sorted(unknown)}")
        opts.update({k: v for k, v in kw.items() if k in opts})
        if opts["res_tol"] is None and opts["error_tol"] is None:
            raise RuntimeError('One of res_tol or error_tol must be set!')
        idx, prepared = [], []
        if not opts["singular"]:
            lim = None if engine == "fused" else FUSED_BATCH_MAX_NC
            for i, (A, P, b, x) in enumerate(problems):
                h = _fused_arrays(A, P, b, x, lim)
                if h is not None:
                    idx.append(i)
                    prepared.append(h)
        results = [None] * len(problems)
        if idx:
            out = _amg_2_v_fused(prepared, [problems[i][3] for i in idx],
                                 opts["pre_smoothing_steps"],
                                 opts["post_smoothing_steps"], opts["jacobi_weight"],
                                 opts["res_tol"], opts["error_tol"], opts["max_iter"],
                                 opts["smoother"])
            if out is not None:
                for i, o in zip(idx, out):
                    results[i] = o
        rest = [i for i in range(len(problems)) if results[i] is None]
        if not rest:
            return results
        sub = amg_2_v_batch([problems[i] for i in rest], workers=workers, engine="hierarchy",
                            **kw)
        for i, o in zip(rest, sub):
            results[i] = o
        return results
    dev = torch.cuda.current_device()
    local = threading.local()

    def run(args):
        if not hasattr(local, "stream"):
            torch.cuda.set_device(dev)
            local.stream = torch.cuda.Stream(device=dev)
        with torch.cuda.stream(local.stream):
            # eager launches: a stream capture must not overlap the other threads' synchronous
            # setup calls (allocations, blocking copies), and concurrency already hides launches
            out = amg_2_v(*args, use_graph=False, engine="hierarchy", **kw)
        local.stream.synchronize()
        return out

    if workers <= 1 or len(problems) <= 1:
        return [amg_2_v(*args, engine="hierarchy", **kw) for args in problems]
    with ThreadPoolExecutor(max_workers=int(workers)) as ex:
        return list(ex.map(run, problems))


def amg_2_v_jacobi(A, P, b, x, dinv_w=None, omega=2. / 3., pre_smoothing_steps=1,
                   post_smoothing_steps=1, max_iter=500, tol=1e-8, history=False):
    """MLAMG.amg_2_v (ns/preconditioner/MLAMG.py:148-197) through the device V-cycle executor.

    Stops after the first cycle with ||b - A x||_2 <= tol (absolute, :194). Returns x (numpy),
    plus the residual history when history=True.
    """
    from .hierarchy import Hierarchy
    H = Hierarchy.two_level(A, P, omega=omega, nu_pre=pre_smoothing_steps,
                            nu_post=post_smoothing_steps, dinv_w=dinv_w)
    xd = to_device_vec(x).clone()
    hist = H.cycle(to_device_vec(b), xd, max_iter, tol=tol)
    out = xd.cpu().numpy()
    return (out, hist) if history else out


# ---------------------------------------------------------------- torch variants (a5'')
# ns/lib/multigrid.py:48-55, 93-98, 213-245: the fp32 torch-sparse paths of the GNN training
# loop (train_dataset.py:111 branch). SURVEY.md §8(a) a5'' marks them "semantics only": they are
# kept here as the same torch operations (they run wherever the caller's tensors live, the GPU
# included) so that aliasing ns.lib.multigrid to this module leaves those callers working.
def jacobi_torch(A, b, x, Dinv=None, omega=0.666, nu=2):
    """ns/lib/multigrid.py:48-55 (x updated in place and returned). Dinv defaults to the stored
    diagonal itself, exactly as the reference does."""
    from .sparse import get_diagonal
    if Dinv is None:
        Dinv = get_diagonal(A)
    for _ in range(nu):
        x += omega * (Dinv * b) - omega * Dinv * (A @ x)
    return x


def gauss_seidel_torch(A, b, x, L=None, U=None, nu=2):
    """ns/lib/multigrid.py:93-98: x = tril(A)^-1 (b - triu(A, 1) x), nu times (dense triangular
    solve of the lower triangle, b as a column)."""
    from .sparse import triu
    if U is None:
        U = triu(A, 1)
    Ad = A.to_dense() if A.is_sparse else A
    for _ in range(nu):
        rhs = (b - U @ x).unsqueeze(1)
        x = torch.linalg.solve_triangular(torch.tril(Ad), rhs, upper=False).squeeze(1)
    return x


def amg_2_v_torch(A, P, b, x, pre_smoothing_steps=1, post_smoothing_steps=1,
                  jacobi_weight=0.666, error_tol=1e-10, max_iter=20):
    """ns/lib/multigrid.py:213-245: two-level Jacobi cycle on torch sparse tensors with a dense
    LU of P^T A P; returns (err[i] / err[i-3]) ** (1/2) like the reference (err = ||x||_2)."""
    from .sparse import get_diagonal
    device = A.device
    Dinv = 1. / get_diagonal(A)
    Pt = P.transpose(0, 1)
    A_H = torch.sparse.mm(torch.sparse.mm(Pt, A), P).to_dense()
    LU, piv = torch.linalg.lu_factor(A_H)
    err = torch.zeros(max_iter, device=device)
    i = 0
    for i in range(max_iter):
        x = jacobi_torch(A, b, x, Dinv, omega=jacobi_weight, nu=pre_smoothing_steps)
        r_H = torch.unsqueeze(Pt.matmul(b - A @ x), 1)
        e_H = torch.linalg.lu_solve(LU, piv, r_H)
        x += P.matmul(e_H.squeeze())
        x = jacobi_torch(A, b, x, Dinv, omega=jacobi_weight, nu=post_smoothing_steps)
        err[i] = torch.linalg.norm(x)
        if err[i] < error_tol:
            break
    n_err = 3
    return (err[i] / err[i - n_err]) ** (1 / (n_err - 1))
