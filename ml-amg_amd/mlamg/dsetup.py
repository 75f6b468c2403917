"""Distributed setup of the row-partitioned levels ("Setup").

The reference builds its hierarchy in one process (ns/lib/multigrid.py:96-108 + :165 for the
SA prolongator and P^T A P; ns/lib/graph.py:7-53 for the seeded Bellman-Ford). The replicated
path (Hierarchy.build on every rank, then partition.build_levels_torch) needs the whole fine
operator and the whole hierarchy on every GPU. Here each rank starts from ITS rows of A and
builds only its part of every partitioned level:

  strength      row-local (the rank's rows of C)
  seeds         RandomState(seed).permutation(n)[:ceil(alpha n)], sorted — drawn by every rank
                (device, csrc/seeds.hip), so the global seed list and the coarse ranges need no
                message
  Bellman-Ford  the order-independent sweeps of mlamg_bellman_ford_canon, one sweep at a time:
                forward halo of the ghost copies, a push sweep over the rank's rows, the ghost
                copies min-merged into their owners (reverse halo), an any-changed reduction —
                until no rank changes anything. Every relaxation is the monotone map
                d_j <- min(d_j, fl(d_i + w_ij)) (labels: min over tight edges), so any fair
                order ends on the same fixed point: distances, labels and aggregates are
                bitwise the single-GPU ones at any world size.
                aggregation='reference': level 0 is the reference's sequential push-order sweep
                (graph.py:40-51), which does not distribute; every rank runs it on the global
                level-0 strength graph (A0_global) and only that step is replicated.
  lambda_max    Lanczos in the D inner product (csrc/eig.hip's algorithm: same start vector,
                recurrences, bisection and stopping rule) with a halo per product and every
                scalar reduced as an allgather of per-rank partials summed in rank order: a
                few ulps from the single-GPU value, not bitwise (lams= overrides it, e.g.
                with the single-GPU values, and everything downstream is then bitwise)
  P             the rank's rows of (I - w D^-1 A) Agg (row-local SpGEMM over its ghost labels)
  A_c           (R A) P for the coarse rows the rank owns (their seed lies in its rows): P's
                entries routed to their column's owner form R's rows (ascending fine index,
                the device transpose's order), the foreign A rows R reaches and the foreign P
                rows R A reaches are fetched once; mlamg_galerkin then sums every owned row
                exactly as the single-GPU call does (csrc/spgemm.hip: row-wise, stored order)
  tail          the first level with fewer than min_rows rows is gathered to every rank and
                built replicated (Hierarchy.build; rank 0's kernel formats broadcast), as the
                executor runs it replicated

Operators are held "global-shaped": a DeviceCSR with the global row count whose rows outside
the rank's range are empty, every index global — the unchanged setup kernels (strength,
diag_inv, SA smoother, SpGEMM, Bellman-Ford sweeps) then run on them as they are, and each row
is computed exactly as in the single-GPU build.

The output (DistSetup) carries the same per-level partition maps partition.build_levels_torch
derives from a replicated hierarchy (tests/test_gpu_dsetup.py compares them array for array)
and feeds DistributedHierarchy.from_setup.

Transport (setup only, not the cycle): SetupComm — ThreadComm (ranks as host threads of one
process, for one-GPU tests and world 1) or TorchComm (torch.distributed: gloo with host copies,
or nccl with device tensors).
"""
from __future__ import annotations

import ctypes
import math
import threading
import time

import numpy as np
import torch

from . import partition
from ._lib import call, ptr, stream_ptr
from .graph import (aggregate_op_device, labels_to_columns, legacy_permutation,
                    modified_bellman_ford_device)
from .partition import TCSR
from .sparse import DeviceCSR, _device, galerkin


# ---------------------------------------------------------------------------------- transport
class ThreadGroup:
    """Shared state of `world` ranks running as threads of one process. The ranks take turns
    on the device (one lock, released only while a rank waits in a collective), so library
    calls never run concurrently."""

    def __init__(self, world):
        self.world = world
        self.barrier = threading.Barrier(world)
        self.box = {}
        self.lock = threading.Lock()


class ThreadComm:
    def __init__(self, group, rank, device=None):
        self.g = group
        self.world, self.rank = group.world, rank
        self.device = device if device is not None else _default_device()
        self.busy_s = 0.0  # time this rank held the device (its own work, without the waits)
        self._t = time.perf_counter()

    def _sync(self):
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        self.busy_s += time.perf_counter() - self._t
        self.g.lock.release()
        try:
            self.g.barrier.wait()
        finally:
            self.g.lock.acquire()
            self._t = time.perf_counter()

    def allgather_obj(self, obj):
        self.g.box[("ag", self.rank)] = obj
        self._sync()
        out = [self.g.box[("ag", q)] for q in range(self.world)]
        self._sync()
        return out

    def exchange(self, sends, recvs):
        """sends {q: tensor}, recvs {q: (numel, dtype)} -> {q: tensor on this device}."""
        for q, t in sends.items():
            if t.numel():
                self.g.box[("x", self.rank, q)] = t.clone()
        self._sync()
        out = {}
        for q, (cnt, dt) in recvs.items():
            if cnt:
                t = self.g.box[("x", q, self.rank)]
                if t.numel() != cnt or t.dtype != dt:
                    raise RuntimeError(f"exchange {q}->{self.rank}: expected {cnt} x {dt}, "
                                       f"got {t.numel()} x {t.dtype}")
                out[q] = t
            else:
                out[q] = torch.empty(0, dtype=dt, device=self.device)
        self._sync()
        for q in sends:
            self.g.box.pop(("x", self.rank, q), None)
        return out


def _default_device():
    return _device() if torch.cuda.is_available() else torch.device("cpu")


def run_threads(world, fn, device=None):
    """fn(comm) on `world` ranks as threads of this process; returns the per-rank results (the
    first exception raised by any rank is re-raised)."""
    g = ThreadGroup(world)
    out = [None] * world
    errs = []
    dev = torch.cuda.current_device() if torch.cuda.is_available() else None

    def body(r):
        if dev is not None:
            torch.cuda.set_device(dev)
        g.lock.acquire()
        try:
            comm = ThreadComm(g, r, device)
            out[r] = fn(comm)
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            comm.busy_s += time.perf_counter() - comm._t
        except BaseException as e:  # noqa: BLE001 — reported to the caller below
            errs.append((r, e))
            g.barrier.abort()  # peers blocked in a collective raise BrokenBarrierError
        finally:
            g.lock.release()

    ts = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errs:
        errs.sort(key=lambda e: isinstance(e[1], threading.BrokenBarrierError))
        raise errs[0][1]
    return out


class TorchComm:
    """Setup transport over torch.distributed (the process group already initialised). Point-
    to-point tensors go device-to-device on nccl (RCCL) and through host copies on gloo;
    objects through all_gather_object on a gloo group."""

    def __init__(self, group=None, device=None):
        import torch.distributed as dist
        self.dist = dist
        self.world, self.rank = dist.get_world_size(), dist.get_rank()
        self.nccl = dist.get_backend() == "nccl"
        self.device = device if device is not None else _default_device()
        self.obj_group = dist.new_group(backend="gloo") if self.nccl else group

    def allgather_obj(self, obj):
        out = [None] * self.world
        self.dist.all_gather_object(out, obj, group=self.obj_group)
        return out

    def exchange(self, sends, recvs):
        dev = self.device
        reqs, bufs = [], {}
        if self.rank in recvs:  # a rank's message to itself stays local
            bufs[("r", self.rank)] = sends[self.rank]
        for q, t in sorted(sends.items()):
            if t.numel() and q != self.rank:
                b = t.contiguous() if self.nccl else t.cpu().contiguous()
                bufs[("s", q)] = b
                reqs.append(self.dist.isend(b, dst=q))
        for q, (cnt, dt) in sorted(recvs.items()):
            if cnt and q != self.rank:
                b = torch.empty(cnt, dtype=dt, device=dev if self.nccl else "cpu")
                bufs[("r", q)] = b
                reqs.append(self.dist.irecv(b, src=q))
        for r in reqs:
            r.wait()
        return {q: (bufs[("r", q)].to(dev) if cnt else torch.empty(0, dtype=dt, device=dev))
                for q, (cnt, dt) in recvs.items()}


class SoloComm:
    """World 1 (no process group needed)."""

    world, rank = 1, 0

    def __init__(self, device=None):
        self.device = device if device is not None else _default_device()

    def allgather_obj(self, obj):
        return [obj]

    def exchange(self, sends, recvs):
        return {q: (sends[q] if cnt else torch.empty(0, dtype=dt, device=self.device))
                for q, (cnt, dt) in recvs.items()}


def setup_comm(world):
    """The setup transport of a torch.distributed job (SoloComm at world 1)."""
    return TorchComm() if world > 1 else SoloComm()


def _any(comm, flag):
    return any(comm.allgather_obj(bool(flag)))


def _allsum(comm, v):
    """Sum of one float per rank, in rank order (the same bits on every rank)."""
    s = 0.0
    for x in comm.allgather_obj(float(v)):
        s += x
    return s


# ---------------------------------------------------------------------------------- operators
def _gs_csr(rows, T, n_rows, n_cols):
    """Global-shaped DeviceCSR: rows `rows` (ascending int64, device) hold T's rows in order,
    every other row is empty."""
    dev = T.col.device
    lens = (T.crow[1:] - T.crow[:-1]).to(torch.int64)
    full = torch.zeros(n_rows, dtype=torch.int64, device=dev)
    if rows.numel():
        full[rows] = lens
    crow = torch.zeros(n_rows + 1, dtype=torch.int64, device=dev)
    crow[1:] = torch.cumsum(full, 0)
    return DeviceCSR.from_torch(crow.to(torch.int32).contiguous(),
                                T.col.to(torch.int32).contiguous(),
                                T.val.to(torch.float64).contiguous(), (n_rows, n_cols))


def _gs_own(M, lo, hi):
    """Rows [lo, hi) of a global-shaped DeviceCSR as a TCSR (row i -> i - lo)."""
    crow, col, val = M.to_torch()
    crow = crow.to(torch.int64)
    s, e = int(crow[lo]), int(crow[hi])
    return TCSR(crow[lo:hi + 1] - s, col[s:e], val[s:e], (hi - lo, M.shape[1]))


def _concat(T1, T2):
    crow = torch.cat([T1.crow.to(torch.int64), T2.crow[1:].to(torch.int64) + int(T1.crow[-1])])
    return TCSR(crow, torch.cat([T1.col, T2.col]), torch.cat([T1.val, T2.val]),
                (T1.shape[0] + T2.shape[0], T1.shape[1]))


def _merge_rows(ids1, T1, ids2, T2):
    """Rows of two TCSRs with disjoint global row ids, sorted by id."""
    ids = torch.cat([ids1, ids2])
    order = torch.argsort(ids)
    T, _, _ = partition._t_gather_rows(_concat(T1, T2), order)
    return ids[order], T


def _ghosts(T, lo, hi):
    """Ascending global columns of T outside [lo, hi) (device int64)."""
    c = T.col.to(torch.int64)
    return torch.unique(c[(c < lo) | (c >= hi)])


class GHalo:
    """One ghost set on globally indexed arrays: forward (owners -> ghost copies) and
    reverse-min (ghost copies -> owners, min-merged). Also the partition.Halo the executor
    takes (built from every rank's ghost list)."""

    def __init__(self, comm, ghosts, ranges):
        self.comm = comm
        r = comm.rank
        g_np = ghosts.cpu().numpy().astype(np.int64)
        allg = comm.allgather_obj(g_np)
        self.halo = partition._halos(allg, ranges, r)
        lo = ranges[r][0]
        dev = ghosts.device
        self.ghosts = ghosts
        self.send = {q: torch.as_tensor(idx.astype(np.int64) + lo, device=dev)
                     for q, idx in self.halo.sends.items()}
        owners = self.halo.ghost_owner
        self.recv = {int(q): torch.as_tensor(g_np[owners == q], device=dev)
                     for q in np.unique(owners)}

    def forward(self, arr):
        got = self.comm.exchange({q: arr[i] for q, i in self.send.items()},
                                 {q: (len(i), arr.dtype) for q, i in self.recv.items()})
        for q, t in got.items():
            if t.numel():
                arr[self.recv[q]] = t

    def reverse_min(self, arr):
        got = self.comm.exchange({q: arr[i] for q, i in self.recv.items()},
                                 {q: (len(i), arr.dtype) for q, i in self.send.items()})
        for q, t in got.items():
            if t.numel():
                i = self.send[q]
                arr[i] = torch.minimum(arr[i], t)

    def fetch_rows(self, M_own, lo):
        """The ghost rows of a row-partitioned operator (M_own: this rank's rows, TCSR) from
        their owners, in ghost order (ascending global index)."""
        sub = {q: partition._t_gather_rows(M_own, i - lo)[0] for q, i in self.send.items()}
        lens = self.comm.exchange(
            {q: (T.crow[1:] - T.crow[:-1]).to(torch.int64) for q, T in sub.items()},
            {q: (len(i), torch.int64) for q, i in self.recv.items()})
        cnt = {q: int(t.sum()) for q, t in lens.items()}
        cols = self.comm.exchange({q: T.col.to(torch.int32) for q, T in sub.items()},
                                  {q: (cnt[q], torch.int32) for q in self.recv})
        vals = self.comm.exchange({q: T.val.to(torch.float64) for q, T in sub.items()},
                                  {q: (cnt[q], torch.float64) for q in self.recv})
        dev = M_own.col.device
        qs = sorted(self.recv)
        ln = torch.cat([lens[q] for q in qs]) if qs else torch.zeros(0, dtype=torch.int64,
                                                                      device=dev)
        crow = torch.zeros(len(ln) + 1, dtype=torch.int64, device=dev)
        crow[1:] = torch.cumsum(ln, 0)
        col = (torch.cat([cols[q] for q in qs]) if qs
               else torch.zeros(0, dtype=torch.int32, device=dev))
        val = (torch.cat([vals[q] for q in qs]) if qs
               else torch.zeros(0, dtype=torch.float64, device=dev))
        return TCSR(crow, col, val, (len(ln), M_own.shape[1]))


# ---------------------------------------------------------------------------------- steps
class DeviceBF:
    """The four mlamg_bf_canon_* entry points (csrc/graph.hip) on a DeviceCSR graph."""

    def begin(self, C, seeds, w, dist, lab, is_seed):
        call("mlamg_bf_canon_begin", C.handle, ptr(seeds), int(seeds.numel()), ptr(w), ptr(dist),
             ptr(lab), ptr(is_seed), stream_ptr())

    def sweep(self, C, w, dist, changed):
        call("mlamg_bf_canon_sweep", C.handle, ptr(w), ptr(dist), ptr(changed), stream_ptr())

    def label(self, C, w, dist, is_seed, lab, changed):
        call("mlamg_bf_canon_label", C.handle, ptr(w), ptr(dist), ptr(is_seed), ptr(lab),
             ptr(changed), stream_ptr())

    def end(self, lab):
        call("mlamg_bf_canon_end", ptr(lab), int(lab.numel()), stream_ptr())


def bellman_ford_distributed(C, seeds_dev, hx, comm, kernels=None):
    """mlamg_bellman_ford_canon over the ranks (module doc). C: global-shaped strength graph of
    this rank's rows; seeds_dev: the global seed list (int32). Returns (labels int32 over all n
    — final on the rank's rows and its ghosts —, distance sweeps). kernels: the sweep kernels
    (default DeviceBF; tests/test_dsetup_transport.py drives the same protocol with a CPU
    restatement of them)."""
    kern = kernels if kernels is not None else DeviceBF()
    n = C.shape[0]
    dev = seeds_dev.device
    w = torch.empty(max(C.nnz, 1), dtype=torch.float32, device=dev)
    dist = torch.empty(n, dtype=torch.float32, device=dev)
    lab = torch.empty(n, dtype=torch.int32, device=dev)
    is_seed = torch.empty(n, dtype=torch.int32, device=dev)
    changed = torch.zeros(1, dtype=torch.int32, device=dev)
    kern.begin(C, seeds_dev, w, dist, lab, is_seed)
    sweeps = 0
    while True:
        hx.forward(dist)
        changed.zero_()
        kern.sweep(C, w, dist, changed)
        hx.reverse_min(dist)
        sweeps += 1
        if not _any(comm, int(changed.item())):
            break
    while True:
        hx.forward(lab)
        changed.zero_()
        kern.label(C, w, dist, is_seed, lab, changed)
        hx.reverse_min(lab)
        if not _any(comm, int(changed.item())):
            break
    hx.forward(lab)
    kern.end(lab)
    return lab, sweeps


def _splitmix_start(lo, hi, seed):
    """csrc/eig.hip k_lz_init's start vector for global rows [lo, hi)."""
    with np.errstate(over="ignore"):
        i = np.arange(lo, hi, dtype=np.uint64)
        x = np.uint64(seed) * np.uint64(0x100000001B3) + i
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
    return (x >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0) * 2.0 - 1.0


def _sturm_count(a, b, m, x):
    cnt = 0
    q = 1.0
    for i in range(m):
        bb = b[i] * b[i] if i > 0 else 0.0
        q = (a[i] - x) - (bb / q if i > 0 else 0.0)
        if q == 0.0:
            q = -1e-300
        if q < 0.0:
            cnt += 1
    return cnt


def _tridiag_max_eig(a, b, m):
    """csrc/eig.hip tridiag_max_eig (Gershgorin bracket, 200 bisection steps)."""
    lo = hi = a[0]
    for i in range(m):
        r = (abs(b[i]) if i > 0 else 0.0) + (abs(b[i + 1]) if i + 1 < m else 0.0)
        lo = min(lo, a[i] - r)
        hi = max(hi, a[i] + r)
    for _ in range(200):
        mid = 0.5 * (lo + hi)
        if mid <= lo or mid >= hi:
            break
        if _sturm_count(a, b, m, mid) == m:
            hi = mid
        else:
            lo = mid
    return hi


def lambda_max_distributed(Ag, hx, lo, hi, comm, max_iter=20000, tol=1e-15, seed=0):
    """lambda_max(D^-1 A) by csrc/eig.hip's Lanczos over the ranks (module doc). Ag: the rank's
    rows, global-shaped. Returns (lambda, iterations)."""
    n = Ag.shape[0]
    dev = _device()
    if n == 0:
        return 0.0, 0
    T = _gs_own(Ag, lo, hi)
    rows = torch.repeat_interleave(torch.arange(lo, hi, device=dev),
                                   (T.crow[1:] - T.crow[:-1]).to(torch.int64))
    on = T.col.to(torch.int64) == rows
    d = torch.zeros(n, dtype=torch.float64, device=dev)
    d_own = torch.zeros(hi - lo, dtype=torch.float64, device=dev)
    d_own.index_add_(0, rows[on] - lo, T.val[on])  # stored diagonal entries, summed
    d[lo:hi] = d_own
    dinv = 1.0 / d_own
    q = torch.zeros(n, dtype=torch.float64, device=dev)
    q[lo:hi] = torch.as_tensor(_splitmix_start(lo, hi, seed), device=dev)
    qprev = torch.zeros(n, dtype=torch.float64, device=dev)
    z = torch.zeros(n, dtype=torch.float64, device=dev)
    nrm0 = math.sqrt(_allsum(comm, float(torch.sum(d_own * (q[lo:hi] * q[lo:hi])))))
    q[lo:hi] *= (1.0 / nrm0) if nrm0 > 0.0 else 0.0
    m_max = min(int(max_iter), n)
    ha, hb = [], [0.0]
    theta_prev, theta = -1.0, 0.0
    j = 0
    while True:
        jend = min(m_max, j + 32)
        while j < jend:
            hx.forward(q)
            Ag.matvec(q, out=z)
            a = _allsum(comm, float(torch.dot(z[lo:hi], q[lo:hi])))
            w = (dinv * z[lo:hi] - a * q[lo:hi]) - hb[j] * qprev[lo:hi]
            b = math.sqrt(_allsum(comm, float(torch.sum(d_own * (w * w)))))
            ha.append(a)
            hb.append(b)
            w *= (1.0 / b) if b > 0.0 else 0.0
            qprev, q = q, qprev
            q[lo:hi] = w
            j += 1
        m, breakdown = j, False
        for i in range(1, j + 1):
            if not (hb[i] > 1e-14 * abs(ha[i - 1]) + 1e-300):
                m, breakdown = i, True
                break
        theta = _tridiag_max_eig(ha, hb, m)
        done = breakdown or j >= m_max
        if theta_prev > 0.0 and abs(theta - theta_prev) <= tol * abs(theta):
            done = True
        theta_prev = theta
        if done:
            return theta, j


def _route_transpose(comm, P_own, lo, n_fine, c_ranges):
    """This rank's rows of R = P^T (coarse rows [c_lo, c_hi), fine columns ascending within a
    row): every rank sends each of its P entries to the owner of its column."""
    dev = P_own.col.device
    r = comm.rank
    lens = (P_own.crow[1:] - P_own.crow[:-1]).to(torch.int64)
    fine = torch.repeat_interleave(torch.arange(lo, lo + P_own.shape[0], device=dev), lens)
    col = P_own.col.to(torch.int64)
    chis = torch.as_tensor([h for _, h in c_ranges], dtype=torch.int64, device=dev)
    dest = torch.searchsorted(chis, col, right=True)
    counts = torch.bincount(dest, minlength=comm.world).cpu().tolist()
    allc = comm.allgather_obj(counts)
    sends = {}
    for q in range(comm.world):
        m = dest == q
        sends[q] = (fine[m].to(torch.int32), col[m].to(torch.int32), P_own.val[m])
    recvs = {q: allc[q][r] for q in range(comm.world)}
    got = [comm.exchange({q: s[k] for q, s in sends.items()},
                         {q: (c, dt) for q, c in recvs.items()})
           for k, dt in ((0, torch.int32), (1, torch.int32), (2, torch.float64))]
    qs = range(comm.world)  # source rank order = ascending fine index
    f = torch.cat([got[0][q] for q in qs]).to(torch.int64)
    c = torch.cat([got[1][q] for q in qs]).to(torch.int64)
    v = torch.cat([got[2][q] for q in qs])
    clo, chi = c_ranges[r]
    c_sorted, order = torch.sort(c, stable=True)
    crow = torch.zeros(chi - clo + 1, dtype=torch.int64, device=dev)
    crow[1:] = torch.cumsum(torch.bincount(c_sorted - clo, minlength=chi - clo), 0)
    return TCSR(crow, f[order].to(torch.int32), v[order], (chi - clo, n_fine))


def _gather_rows_all(comm, T, n_cols):
    """Every rank's rows (in rank order) as one TCSR on T's device."""
    dev = T.col.device
    parts = comm.allgather_obj((T.crow.cpu().numpy(), T.col.cpu().numpy(), T.val.cpu().numpy()))
    crows, cols, vals, off = [np.zeros(1, np.int64)], [], [], 0
    for crow, col, val in parts:
        crows.append(crow[1:].astype(np.int64) + off)
        off += int(crow[-1])
        cols.append(col)
        vals.append(val)
    crow = np.concatenate(crows)
    return TCSR(torch.as_tensor(crow, device=dev),
                torch.as_tensor(np.concatenate(cols).astype(np.int32), device=dev),
                torch.as_tensor(np.concatenate(vals).astype(np.float64), device=dev),
                (len(crow) - 1, n_cols))


def _family(l, shape, nnz, coarse_format, vec_min_row):
    """Hierarchy.apply_formats's rule for the kernel family of an operator."""
    if (l > 0 and coarse_format != "exact" and shape[0] <= (1 << 20)
            and nnz >= vec_min_row * shape[0]):
        return "vector"
    return "exact"


class DistSetup:
    """Output of build_distributed for one rank (see module doc)."""

    def __init__(self):
        self.parts = []       # partition.build_levels_torch-shaped dicts, one per level
        self.dinv = []        # the rank's rows of each level's Jacobi weights (device)
        self.families = []    # {"A"|"P"|"R": "exact" | "vector"} per level
        self.seeds = []       # sorted global seed list per level (numpy int64)
        self.labels = []      # per-level global label arrays (device int32; final on own rows)
        self.lams, self.omegas, self.bf_sweeps, self.lanczos_iters = [], [], [], []
        self.own_rows = []    # per-level (A_own, P_own) TCSRs (global indices), for checks
        self.tail = None      # the replicated Hierarchy below the partitioned levels
        self.times = {}
        self.nu_pre = self.nu_post = 1


def build_distributed(A_own, n, comm, *, alpha=0.1, strength_mode="invabs",
                      aggregation="bellman_ford", A0_global=None, max_coarse=1000, max_levels=10,
                      jacobi_weight=2.0 / 3.0, seed=0, lanczos_tol=1e-15, lanczos_iter=20000,
                      min_rows=50000, lams=None, nu_pre=1, nu_post=1, fine_format="autotune",
                      coarse_format="auto", vec_min_row=None):
    """This rank's part of the hierarchy Hierarchy.build(A, ...) would build (sorted seeds),
    with the levels of >= min_rows rows (and always level 0) row-partitioned as
    DistributedHierarchy partitions them.

    A_own: partition.TCSR of this rank's rows [lo, hi) = partition.row_ranges(n, world)[rank]
    of the global operator (global column indices, on the device). aggregation: 'bellman_ford'
    (Hierarchy.build's default rule, fully distributed) or 'reference' (level 0 by the
    reference's push-order sweep on A0_global — a scipy / DeviceCSR of the whole level-0
    operator every rank holds — coarse unknowns in sorted seed order). lams: per-level
    lambda_max values to use instead of the distributed Lanczos."""
    from .hierarchy import Hierarchy, strength
    if aggregation not in ("bellman_ford", "reference"):
        raise ValueError("distributed setup: aggregation must be 'bellman_ford' or 'reference'")
    if aggregation == "reference" and A0_global is None:
        raise ValueError("aggregation='reference' needs A0_global (the push-order sweep of "
                         "graph.py:40-51 is sequential over the whole level-0 graph)")
    if not (isinstance(seed, (int, np.integer)) and 0 <= int(seed) < 2 ** 32):
        raise ValueError("distributed setup needs an integer seed in [0, 2**32)")
    vec_min_row = Hierarchy.VEC_MIN_MEAN_ROW if vec_min_row is None else vec_min_row
    world, rank = comm.world, comm.rank
    ranges = partition.row_ranges(n, world)
    if A_own.shape[0] != ranges[rank][1] - ranges[rank][0]:
        raise ValueError(f"rank {rank}: A_own has {A_own.shape[0]} rows, its range "
                         f"{ranges[rank]}")
    if n <= max_coarse or max_levels <= 1:
        raise ValueError("nothing to partition: the operator is the coarse operator itself")
    S = DistSetup()
    S.nu_pre, S.nu_post = nu_pre, nu_post
    tm = {"strength_seeds": 0.0, "bellman_ford": 0.0, "lambda_max": 0.0, "prolongator": 0.0,
          "transpose": 0.0, "galerkin": 0.0, "maps": 0.0, "tail": 0.0}
    t_all = time.perf_counter()
    dev = _device()
    l = 0
    while True:
        lo, hi = ranges[rank]
        t0 = time.perf_counter()
        rows_own = torch.arange(lo, hi, device=dev)
        Ag = _gs_csr(rows_own, A_own, n, n)
        xg = _ghosts(A_own, lo, hi)
        hx = GHalo(comm, xg, ranges)
        k = int(math.ceil(alpha * n))
        seeds_dev = legacy_permutation(int(seed), n, k)[:k]
        seeds_sorted, _ = torch.sort(seeds_dev)
        seeds_np = seeds_sorted.cpu().numpy().astype(np.int64)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if aggregation == "reference" and l == 0:
            from .sparse import as_device
            C0 = strength(as_device(A0_global), strength_mode)
            _, lab, sweeps = modified_bellman_ford_device(C0, seeds_dev)
            del C0
        else:
            C = strength(Ag, strength_mode)
            lab, sweeps = bellman_ford_distributed(C, seeds_sorted, hx, comm)
            del C
        col = labels_to_columns(lab, seeds_sorted)
        Agg = aggregate_op_device(col, k)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        if lams is not None:
            lam, its = float(lams[l]), 0
        else:
            lam, its = lambda_max_distributed(Ag, hx, lo, hi, comm, lanczos_iter, lanczos_tol)
        omega = (4.0 / 3.0) / abs(lam)
        t3 = time.perf_counter()
        h = ctypes.c_void_p()
        call("mlamg_sa_smoother", Ag.handle, float(omega), ctypes.byref(h), stream_ptr())
        Sg = DeviceCSR(h)
        Pg = Sg @ Agg
        del Sg, Agg
        P_own = _gs_own(Pg, lo, hi)
        dinv = Ag.diag_inv(omega if jacobi_weight == "sa" else jacobi_weight)[lo:hi].clone()
        c_ranges = partition._seed_ranges(seeds_np, ranges, k)
        clo, chi = c_ranges[rank]
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        R_own = _route_transpose(comm, P_own, lo, n, c_ranges)
        rg = _ghosts(R_own, lo, hi)
        hr = GHalo(comm, rg, ranges)
        torch.cuda.synchronize()
        t5 = time.perf_counter()
        # A rows R reaches, then P rows R A reaches (foreign columns of those A rows)
        A_r = hr.fetch_rows(A_own, lo)
        ids_a, A_ext = _merge_rows(rows_own, A_own, rg, A_r)
        pj = _ghosts(A_ext, lo, hi)
        hpj = GHalo(comm, pj, ranges)
        P_j = hpj.fetch_rows(P_own, lo)
        ids_p, P_ext_all = _merge_rows(rows_own, P_own, pj, P_j)
        Rg = _gs_csr(torch.arange(clo, chi, device=dev), R_own, k, n)
        Ag2 = _gs_csr(ids_a, A_ext, n, n)
        Pg2 = _gs_csr(ids_p, P_ext_all, n, k)
        Acg = galerkin(Rg, Ag2, Pg2)
        Ac_own = _gs_own(Acg, clo, chi)
        del Rg, Ag2, Pg2, Acg, A_ext
        torch.cuda.synchronize()
        t6 = time.perf_counter()
        # is the next level partitioned too? (DistributedHierarchy's rule on level sizes)
        next_is_level = k > max_coarse and l + 2 < max_levels
        last = not (next_is_level and k >= min_rows)
        # the executor's maps (partition.build_levels_torch's dict)
        prow = torch.cat([rows_own, xg])
        pos = torch.searchsorted(ids_p, prow)
        P_ext, _, _ = partition._t_gather_rows(P_ext_all, pos)
        d = {"level": l, "rank": rank, "world": world, "lo": lo, "hi": hi, "n": n, "nc": k,
             "c_lo": clo, "c_hi": chi, "c_ranges": c_ranges, "ranges": ranges,
             "A_loc": partition._t_remap(A_own, lo, hi, xg),
             "R_own": partition._t_remap(R_own, lo, hi, rg),
             "halo_x": hx.halo, "halo_r": hr.halo}
        if last:
            d["P_loc"] = P_ext
            d["halo_p"] = None
        else:
            pg = _ghosts(P_ext, clo, chi)
            d["P_loc"] = partition._t_remap(P_ext, clo, chi, pg)
            d["halo_p"] = GHalo(comm, pg, c_ranges).halo
        nnz = comm.allgather_obj((A_own.nnz, P_own.nnz))
        nnz_a, nnz_p = sum(a for a, _ in nnz), sum(p for _, p in nnz)
        S.families.append({"A": _family(l, (n, n), nnz_a, coarse_format, vec_min_row),
                           "P": _family(l, (n, k), nnz_p, coarse_format, vec_min_row),
                           "R": _family(l, (k, n), nnz_p, coarse_format, vec_min_row)})
        S.parts.append(d)
        S.dinv.append(dinv)
        S.seeds.append(seeds_np)
        S.labels.append(lab)
        S.lams.append(lam)
        S.omegas.append(omega)
        S.bf_sweeps.append(sweeps)
        S.lanczos_iters.append(its)
        S.own_rows.append((A_own, P_own))
        torch.cuda.synchronize()
        t7 = time.perf_counter()
        for key, dt in (("strength_seeds", t1 - t0), ("bellman_ford", t2 - t1),
                        ("lambda_max", t3 - t2), ("prolongator", t4 - t3),
                        ("transpose", t5 - t4), ("galerkin", t6 - t5), ("maps", t7 - t6)):
            tm[key] += dt
        if last:
            break
        A_own, n, ranges, l = Ac_own, k, c_ranges, l + 1
    # the replicated tail: the first unpartitioned level (or the coarse operator) everywhere
    t8 = time.perf_counter()
    Ac_all = _gather_rows_all(comm, Ac_own, k)
    Ac = DeviceCSR.from_torch(Ac_all.crow.to(torch.int32).contiguous(),
                              Ac_all.col.to(torch.int32).contiguous(),
                              Ac_all.val.contiguous(), (k, k))
    del Ac_all
    Ht = Hierarchy.build(Ac, alpha=alpha, strength_mode=strength_mode,
                         aggregation="bellman_ford", max_coarse=max_coarse,
                         max_levels=max_levels - (l + 1), jacobi_weight=jacobi_weight, seed=seed,
                         sort_seeds=True, lanczos_tol=lanczos_tol, lanczos_iter=lanczos_iter,
                         nu_pre=nu_pre, nu_post=nu_post, finalize=False)
    if rank == 0:
        Ht.apply_formats(fine_format, coarse_format, vec_min_row=vec_min_row,
                         first_level=l + 1)
    fmts = comm.allgather_obj(Ht.formats() if rank == 0 else None)[0]
    if rank != 0:
        Ht.set_formats(fmts)
    Ht._finalize(nu_pre, nu_post)
    torch.cuda.synchronize()
    tm["tail"] = time.perf_counter() - t8
    tm["total"] = time.perf_counter() - t_all
    S.tail = Ht
    S.times = {key: round(v, 4) for key, v in tm.items()}
    return S


def split_rows(A, world, rank, device=None):
    """Rows partition.row_ranges(n, world)[rank] of a scipy operator as a TCSR on the device
    (the input build_distributed takes; a real distributed caller assembles its rows itself)."""
    lo, hi = partition.row_ranges(A.shape[0], world)[rank]
    A = A.tocsr()
    return TCSR.from_scipy(A[lo:hi], device=device or _device())


__all__ = ["ThreadComm", "TorchComm", "SoloComm", "setup_comm", "run_threads", "build_distributed", "DistSetup", "DeviceBF",
           "bellman_ford_distributed", "lambda_max_distributed", "split_rows"]
