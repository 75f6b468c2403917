"""Multi-GPU V-cycle: the K finest levels row-partitioned over one process per GPU with RCCL halo
exchanges, the coarser levels replicated (C side: csrc/comm.hip).

The reference's only parallel backend is a task farm over independent problems
(ns/parallel/pool.py:139-186: pickled callables over multiprocessing pipes or mpi4py). Splitting
one problem across GPUs is new here. Bootstrap: torch.distributed (gloo, CPU) carries the
128-byte RCCL unique id and the benchmark barriers; all data-path traffic is RCCL (xGMI).
"""
from __future__ import annotations

import ctypes
import io
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

from . import _lib, partition
from ._lib import _tol_arg, call, ptr, stream_ptr
from .sparse import DeviceCSR


class Comm:
    """RCCL communicator created from a unique id broadcast over torch.distributed (gloo)."""

    def __init__(self, world, rank, phases=None):
        self.world, self.rank = world, rank
        if phases is not None:
            phases.enter("uid_broadcast")
        buf = ctypes.create_string_buffer(128)
        if rank == 0:
            call("mlamg_comm_unique_id", buf)
        obj = [bytes(buf.raw) if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(obj, src=0)
        uid = ctypes.create_string_buffer(obj[0], 128)
        if phases is not None:
            phases.enter("comm_create")
        h = ctypes.c_void_p()
        call("mlamg_comm_create", uid, int(world), int(rank), ctypes.byref(h))
        self.handle = h

    def info(self):
        return comm_info(self)

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            try:
                _lib.lib.mlamg_comm_destroy(h)
            except Exception:
                pass
            self.handle = None


def comm_info(comm):
    """{'nranks', 'rank', 'device', 'transport'} as the communicator's transport reports them
    (RCCL: ncclCommCount / ncclCommUserRank / ncclCommCuDevice)."""
    nr, rk, dv, tr = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    call("mlamg_comm_info", comm.handle, ctypes.byref(nr), ctypes.byref(rk), ctypes.byref(dv),
         ctypes.byref(tr))
    return {"nranks": nr.value, "rank": rk.value, "device": dv.value,
            "transport": ("rccl", "loopback", "null")[tr.value]}


class LoopbackGroup:
    """In-process test transport (include/mlamg.h mlamg_loop_group): `world` communicators whose
    ranks are host threads of this process sharing one GPU, each on its own stream. RCCL refuses
    two ranks on one device; this runs the distributed executor itself (csrc/comm.hip, eager
    mode) at world sizes > 1 on a single GPU."""

    def __init__(self, world):
        h = ctypes.c_void_p()
        call("mlamg_loop_group_create", int(world), ctypes.byref(h))
        self.handle = h
        self.world = world
        self.comms = [LoopbackComm(self, r) for r in range(world)]

    def close(self):
        for c in self.comms:
            c.close()
        if self.handle:
            call("mlamg_loop_group_destroy", self.handle)
            self.handle = None


class LoopbackComm:
    def __init__(self, group, rank):
        self.world, self.rank = group.world, rank
        h = ctypes.c_void_p()
        call("mlamg_comm_create_loopback", group.handle, int(rank), ctypes.byref(h))
        self.handle = h

    def close(self):
        if self.handle:
            _lib.lib.mlamg_comm_destroy(self.handle)
            self.handle = None


class NullComm:
    """Timing-only communicator (include/mlamg.h mlamg_comm_create_null): rank `rank` of `world`
    with every exchange skipped, to time one rank's device work of the distributed cycle on a
    single GPU. Results are not valid."""

    def __init__(self, world, rank):
        self.world, self.rank = world, rank
        h = ctypes.c_void_p()
        call("mlamg_comm_create_null", int(world), int(rank), ctypes.byref(h))
        self.handle = h

    def close(self):
        if self.handle:
            _lib.lib.mlamg_comm_destroy(self.handle)
            self.handle = None


class Halo:
    def __init__(self, comm, halo: partition.Halo):
        nn = len(halo.neighbors)
        self.nbr = np.asarray(halo.neighbors, dtype=np.int32)
        self.send_cnt = np.asarray(halo.send_counts, dtype=np.int64)
        self.recv_cnt = np.asarray(halo.recv_counts, dtype=np.int64)
        self.send_idx = np.ascontiguousarray(halo.send_idx, dtype=np.int32)
        h = ctypes.c_void_p()
        call("mlamg_halo_create", comm.handle, int(halo.n_own), int(nn),
             self.nbr.ctypes.data_as(ctypes.c_void_p), self.send_cnt.ctypes.data_as(ctypes.c_void_p),
             self.send_idx.ctypes.data_as(ctypes.c_void_p),
             self.recv_cnt.ctypes.data_as(ctypes.c_void_p), ctypes.byref(h))
        self.handle = h
        self.n_ghost = int(self.recv_cnt.sum())

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            try:
                _lib.lib.mlamg_halo_destroy(h)
            except Exception:
                pass
            self.handle = None


class DistributedHierarchy:
    """The K finest levels of a (replicated) Hierarchy split over `world` GPUs.

    Level l+1 rows are owned by the rank that owns their aggregate's seed node on level l, so
    restriction needs only an r-halo and prolongation a halo of the coarse correction; below
    level K-1 the owned coarse segments are allgathered and every rank runs the replicated
    coarse cycle. The iterate is bitwise the single-GPU Hierarchy.cycle iterate."""

    def __init__(self, H, comm, min_rows=50000, max_partitioned=None, A_host=None,
                 local_autotune=True, overlap_min_rows=2_000_000, partition_impl="torch"):
        """H: mlamg.hierarchy.Hierarchy built identically on every rank (sorted seeds, same
        kernel formats — see sync_formats). Levels with at least `min_rows` rows (at most
        `max_partitioned` of them) are row-partitioned; the rest are replicated.
        local_autotune: time every exact-order kernel on each rank's local operators (see
        tune_local) instead of reusing the global operator's choice.
        overlap_min_rows: local operators with at least this many rows are split into
        boundary | interior | boundary row blocks (partition.interior_split) so their halo
        exchange overlaps the interior rows (mlamg_dhier_set_split); None: no splits. A split
        costs two more launches and a stream fork/join per exchange (measured with the null
        communicator at world 8, C4: +7 us per split operator), so it pays only where the
        interior rows take longer than that: the default splits local operators of >= 2 M rows
        (C4 level 0 at world <= 4).
        partition_impl: 'torch' (default) builds the partition maps with torch ops on the
        operators' own device arrays (partition.build_levels_torch; the local operators never
        leave the GPU); 'numpy' downloads every partitioned operator and runs the host build
        (partition.build_levels, the reference implementation of the maps; A_host, if given,
        replaces the download of level 0). Both give the same maps. Phase wall times are kept
        in self.setup_times.
        Without a replicated hierarchy: DistributedHierarchy.from_setup (mlamg.dsetup)."""
        if not H.levels:
            raise ValueError("distributed cycle needs at least one level above the coarse solve")
        if (H.nu_pre, H.nu_post) != (1, 1):
            raise NotImplementedError("the distributed cycle is V(1,1)")
        if any(L.seeds is None for L in H.levels):
            raise ValueError("hierarchy was not built by Hierarchy.build (seeds unknown)")
        self.H = H
        self.setup = None
        self.comm = comm
        world, rank = comm.world, comm.rank
        K = 1
        while K < len(H.levels) and H.levels[K].A.shape[0] >= min_rows:
            K += 1
        if max_partitioned is not None:
            K = max(1, min(K, int(max_partitioned)))
        self.K = K
        if any(np.any(np.diff(H.levels[l].seeds) <= 0) for l in range(K)):
            # coarse rows follow their seed's owner: contiguous only with ascending seeds
            raise ValueError("the distributed cycle needs each partitioned level's coarse "
                             "unknowns in ascending seed order (Hierarchy.build with sorted "
                             "seeds; aggregation='reference' with coarse_order='sorted')")
        self.setup_times = st = {}
        t0 = time.perf_counter()
        seeds = [H.levels[l].seeds for l in range(K)]
        if partition_impl == "torch":
            def tc(M):
                crow, col, val = M.to_torch()
                return partition.TCSR(crow, col, val, M.shape)
            As = [tc(H.levels[l].A) for l in range(K)]
            Ps = [tc(H.levels[l].P) for l in range(K)]
            Rs = [tc(H.levels[l].R) for l in range(K)]
            torch.cuda.synchronize()
            st["download"] = time.perf_counter() - t0
            self.parts = parts = partition.build_levels_torch(As, Ps, Rs, seeds, world, rank)
            del As, Ps, Rs
        elif partition_impl == "numpy":
            As = [A_host if (l == 0 and A_host is not None) else H.levels[l].A.to_scipy()
                  for l in range(K)]
            Ps = [H.levels[l].P.to_scipy() for l in range(K)]
            st["download"] = time.perf_counter() - t0
            self.parts = parts = partition.build_levels(As, Ps, seeds, world, rank)
            del As, Ps
        else:
            raise ValueError(f"unknown partition_impl {partition_impl!r}")
        torch.cuda.synchronize()
        st["partition"] = time.perf_counter() - t0 - st["download"]
        globs = [{"A": H.levels[l].A, "P": H.levels[l].P, "R": H.levels[l].R, "family": None}
                 for l in range(K)]
        dinvs = [H.levels[l].dinv[p["lo"]:p["hi"]].clone() for l, p in enumerate(parts)]
        self._assemble(parts, globs, dinvs, H.levels[K:], H, local_autotune, overlap_min_rows,
                       t0)

    @classmethod
    def from_setup(cls, S, comm, local_autotune=True, overlap_min_rows=2_000_000):
        """The executor over a distributed setup (mlamg.dsetup.build_distributed): the rank's
        partition maps and Jacobi weights as built there, each local operator's kernel family
        by Hierarchy.apply_formats's rule on the global operator (S.families), the replicated
        tail S.tail. Without a replicated hierarchy there is no global operator to reuse a
        format from: every local operator is tuned within its family."""
        if (S.nu_pre, S.nu_post) != (1, 1):
            raise NotImplementedError("the distributed cycle is V(1,1)")
        self = cls.__new__(cls)
        self.H = None
        self.setup = S
        self.comm = comm
        self.K = len(S.parts)
        self.setup_times = {"download": 0.0, "partition": 0.0}
        self.parts = S.parts
        globs = [{"A": None, "P": None, "R": None, "family": f} for f in S.families]
        self._assemble(S.parts, globs, S.dinv, S.tail.levels, S.tail, local_autotune,
                       overlap_min_rows, time.perf_counter())
        return self

    def _assemble(self, parts, globs, dinvs, tail_levels, tail, local_autotune,
                  overlap_min_rows, t0):
        """Local operators (tuned), halos, the replicated coarse hierarchy and the C executor."""
        comm = self.comm
        st = self.setup_times
        t_ops = [0.0, 0.0]  # upload, local autotune
        p0 = parts[0]
        self.lo, self.hi = p0["lo"], p0["hi"]
        self.n_own = self.hi - self.lo

        self.tuning = []

        def like(M_glob, M_part, kind, family=None):
            t1 = time.perf_counter()
            M_loc = _device_csr(M_part)
            t2 = time.perf_counter()
            M, t = tune_local(M_glob, M_loc, kind, autotune=local_autotune, family=family)
            t_ops[0] += t2 - t1
            t_ops[1] += time.perf_counter() - t2
            self.tuning.append(t)
            return M

        self._keep = []
        last = parts[-1]
        # replicated coarse hierarchy: the levels below the partitioned ones + the coarse solve
        hh = ctypes.c_void_p()
        call("mlamg_hier_create", ctypes.byref(hh))
        self.coarse = hh
        for L in tail_levels:
            call("mlamg_hier_add_level", hh, L.A.handle, ptr(L.dinv), L.P.handle, L.R.handle)
        call("mlamg_hier_set_coarse", hh, tail.Ac.handle, tail.dense)
        call("mlamg_hier_set_smoothing", hh, int(tail.nu_pre), int(tail.nu_post))
        self.c_lo = np.array([a for a, _ in last["c_ranges"]], dtype=np.int64)
        self.c_hi = np.array([b for _, b in last["c_ranges"]], dtype=np.int64)
        d = ctypes.c_void_p()
        call("mlamg_dhier_create", comm.handle, hh, int(last["nc"]),
             self.c_lo.ctypes.data_as(ctypes.c_void_p), self.c_hi.ctypes.data_as(ctypes.c_void_p),
             ctypes.byref(d))
        self.handle = d
        self.ghosts = []
        self.splits = []
        for l, p in enumerate(parts):
            g = globs[l]
            fam = g["family"]
            A_loc = like(g["A"], p["A_loc"], "A", fam and fam["A"])
            P_loc = like(g["P"], p["P_loc"], "P", fam and fam["P"])
            R_own = like(g["R"], p["R_own"], "R", fam and fam["R"])
            dinv = dinvs[l]
            if A_loc.get_format()[0] == "rowpat":
                A_loc.attach_dinv(dinv)
            hx = Halo(comm, p["halo_x"])
            hr = Halo(comm, p["halo_r"])
            hp = Halo(comm, p["halo_p"]) if p["halo_p"] is not None else None
            self._keep.append((A_loc, P_loc, R_own, dinv, hx, hr, hp))
            self.ghosts.append((hx.n_ghost, hr.n_ghost, hp.n_ghost if hp else 0))
            call("mlamg_dhier_add_level", d, A_loc.handle, ptr(dinv), P_loc.handle, R_own.handle,
                 hx.handle, hr.handle, hp.handle if hp else None)
            if overlap_min_rows is not None:
                n_l = p["hi"] - p["lo"]
                ops = [(0, g["A"], p["A_loc"], n_l, dinv, fam and fam["A"]),
                       (1, g["R"], p["R_own"], n_l, None, fam and fam["R"])]
                if hp is not None:
                    ops.append((2, g["P"], p["P_loc"], p["c_hi"] - p["c_lo"], None,
                                fam and fam["P"]))
                for which, M_glob, M_host, n_owned, dv, fm in ops:
                    if M_host.shape[0] >= overlap_min_rows:
                        self._split(l, which, M_glob, M_host, n_owned, dv, like, fm)
            if l == 0:
                self.A_loc = A_loc
                self.hx = hx
        self.n_ext = self.n_own + self.hx.n_ghost
        torch.cuda.synchronize()
        st["upload"], st["local_autotune"] = t_ops
        st["total"] = time.perf_counter() - t0
        for p in parts:  # the maps' own copies of the local operators are not needed again
            p["A_loc"] = p["R_own"] = p["P_loc"] = None

    def _split(self, l, which, M_glob, M_host, n_owned, dinv, like, family=None):
        if isinstance(M_host, partition.TCSR):
            cut = partition.interior_split_torch(M_host, n_owned)
        else:
            cut = partition.interior_split(M_host, n_owned)
        if cut is None:
            return
        lo, hi = cut
        parts = []
        for a, b in ((0, lo), (lo, hi), (hi, M_host.shape[0])):
            if b == a:
                parts.append(None)
                continue
            Mp = M_host.rows(a, b) if isinstance(M_host, partition.TCSR) else M_host[a:b]
            M = like(M_glob, Mp, "APR"[which], family)
            self.tuning.pop()  # keep D.tuning = the whole operators' choices, 3 per level
            if dinv is not None and M.get_format()[0] == "rowpat":
                # a view: the epilogues are handed dinv + a, the very pointer attached
                M.attach_dinv(dinv[a:b])
            self._keep.append(M)
            parts.append(M)
        call("mlamg_dhier_set_split", self.handle, int(l), int(which),
             parts[0].handle if parts[0] else None, parts[1].handle,
             parts[2].handle if parts[2] else None)
        self.splits.append({"level": l, "op": "APR"[which], "rows": [0, lo, hi, M_host.shape[0]],
                            "formats": ["/".join(map(str, M.get_format()[:2])) if M else None
                                        for M in parts]})

    def set_overlap(self, on):
        """Overlap each split operator's halo exchange with its interior rows (default on)."""
        call("mlamg_dhier_set_overlap", self.handle, int(bool(on)))

    def new_x(self, x_own):
        x = torch.zeros(self.n_ext, dtype=torch.float64, device="cuda")
        x[: self.n_own].copy_(x_own)
        return x

    def set_coarse_graph(self, on):
        call("mlamg_dhier_set_coarse_graph", self.handle, int(bool(on)))

    def set_cycle_graph(self, on):
        """Replay each cycle from one captured hipGraph (kernels + RCCL calls)."""
        call("mlamg_dhier_set_cycle_graph", self.handle, int(bool(on)))

    def cycle(self, b_own, x_ext, n_cycles, tol=None, history=True):
        hist = torch.zeros(max(n_cycles, 1), dtype=torch.float64, device="cuda") if history else None
        done = ctypes.c_int32()
        from .hierarchy import rhs_arg
        call("mlamg_dhier_vcycle", self.handle, ptr(rhs_arg(b_own)), ptr(x_ext), int(n_cycles),
             _tol_arg(tol),
             ptr(hist), ctypes.byref(done) if history else None, stream_ptr())
        if not history:
            return None
        return hist[: int(done.value)].cpu().numpy()

    def __del__(self):
        for attr, fn in (("handle", "mlamg_dhier_destroy"), ("coarse", "mlamg_hier_destroy")):
            h = getattr(self, attr, None)
            if h:
                try:
                    getattr(_lib.lib, fn)(h)
                except Exception:
                    pass
                setattr(self, attr, None)


def rank_memory():
    """This rank's memory: device bytes in use (hipMemGetInfo: everything the process holds on
    its GPU, the library's own allocations included), torch's peak allocation, and the host
    process's peak resident set."""
    import resource
    free, total = torch.cuda.mem_get_info()
    return {"device_used_GB": round((total - free) / 1e9, 3),
            "torch_peak_GB": round(torch.cuda.max_memory_allocated() / 1e9, 3),
            "host_peak_rss_GB": round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6, 3)}


def _device_csr(M):
    """A partition map's local operator (scipy CSR or partition.TCSR) as a DeviceCSR."""
    if isinstance(M, partition.TCSR):
        if M.col.is_cuda:
            return DeviceCSR.from_torch(M.crow.to(torch.int32).contiguous(),
                                        M.col.to(torch.int32).contiguous(),
                                        M.val.contiguous(), M.shape)
        M = M.to_scipy()
    return DeviceCSR.from_scipy(M, check=False)


def tune_local(M_glob, M_loc, kind, autotune=True, family=None):
    """Kernel for one rank's local operator. The local operator keeps every row's stored
    entry order, so any kernel of the global operator's family reproduces its rows bit for bit:
    the exact-order family (CSR-stream, SELL, sorted, dictionary SELL, row-pair patterns,
    long-row tiles: scipy's order) or the CSR-vector family (one canonical order for every
    width). With autotune the fastest of the family on the local operator is kept (ghost
    columns change what the encoders accept and how well they pack). Returns
    (M_loc, {"chosen": ..., "us": {...}}).
    M_glob None (a distributed setup: no global operator on the rank): `family` ('exact' or
    'vector', Hierarchy.apply_formats's rule on the global operator) names the family; the
    search starts from its first candidate."""
    from .hierarchy import Hierarchy
    if M_glob is None:
        if family not in ("exact", "vector"):
            raise ValueError("tune_local without a global operator needs family='exact' or "
                             "'vector'")
        fmt, arg = ("vector", 64) if family == "vector" else ("csr_stream", 0)
    else:
        fmt, arg, _ = M_glob.get_format()
    if (autotune and M_glob is not None and M_loc.shape == M_glob.shape
            and M_loc.nnz == M_glob.nnz
            and M_loc.fingerprint() == M_glob.fingerprint()):
        # the rank's operator IS the global one (world 1, or a level a rank owns whole, e.g. the
        # whole coarse index space): the global autotune's choice, nothing to time
        M_loc.set_format(fmt, arg)
        return M_loc, {"chosen": "/".join(map(str, M_loc.get_format()[:2])), "reused": True}
    if not autotune:
        try:
            M_loc.set_format(fmt, arg)
        except _lib.MlamgError as e:  # e.g. sorted: ghost columns too far from owned
            if e.code != _lib.MLAMG_EUNSUPPORTED or fmt == "vector":
                raise
            M_loc.set_format("csr_stream")  # same summation order
        return M_loc, {"chosen": "/".join(map(str, M_loc.get_format()[:2]))}
    x = torch.randn(M_loc.shape[1], dtype=torch.float64, device="cuda")
    y = torch.zeros(M_loc.shape[0], dtype=torch.float64, device="cuda")
    if kind == "A" and M_loc.shape[0] != M_loc.shape[1]:
        kind = "R"  # ghost columns: mlamg_residual is square-only, time y = A x instead
    times = {}
    if fmt == "vector":
        cands = list(Hierarchy.VECTOR_CANDIDATES)
    else:
        cands = list(Hierarchy.EXACT_CANDIDATES)
        if M_loc.nnz >= 16 * max(M_loc.shape[0], 1):
            cands += list(Hierarchy.LONG_CANDIDATES)
    # as Hierarchy.apply_formats: the global choice first, then the rest in order of their byte
    # lower bound; a candidate that could not beat the best time even at LB_PEAK_BPS is skipped
    # (a timing rule only: every candidate of the family computes the same bits)
    lbs = {c: Hierarchy._lower_bound_us(M_loc, kind, c[0]) for c in cands}
    cands.sort(key=lambda c: (c != (fmt, arg), lbs[c]))
    pruned, refused = [], set()
    for f, a in cands:
        if (times and lbs[(f, a)] >= min(times.values())) or f in refused:
            pruned.append(f"{f}/{a}")
            continue
        try:
            times[f"{f}/{a}"] = Hierarchy._time_format(M_loc, f, a, x, y, kind=kind)
        except _lib.MlamgError as e:
            if e.code != _lib.MLAMG_EUNSUPPORTED:
                raise
            refused.add(f)
    best = min(times, key=times.get)
    f, a = best.split("/")
    M_loc.set_format(f, int(a))
    return M_loc, {"chosen": best, "us": {k: round(v, 2) for k, v in times.items()},
                   "pruned": pruned}


def sync_formats(H, world):
    """Give every rank rank 0's SpMV kernel choice (autotune timings differ between GPUs)."""
    if world > 1:
        obj = [H.formats()]
        dist.broadcast_object_list(obj, src=0)
        H.set_formats(obj[0])


def finalize_replicated(H, world, rank):
    """Kernel formats and the coarse solver of a hierarchy built with finalize=False on every
    rank: rank 0 runs the format autotune and broadcasts its choice, the other ranks take it
    without timing anything (VERDICT r04 Weak #7: each rank used to repeat the ~1 s autotune
    and then discard it for rank 0's), then every rank builds the coarse solver. Returns the
    seconds this rank spent."""
    t0 = time.perf_counter()
    if rank == 0 or world == 1:
        H.apply_formats("autotune", "auto")
    if world > 1:
        obj = [H.formats() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        if rank != 0:
            H.set_formats(obj[0])
    H._finalize(H.nu_pre, H.nu_post)
    torch.cuda.synchronize()
    return time.perf_counter() - t0


EXIT_DIST_TIMEOUT = 5
EXIT_DIST_FAILED = 6

# the phases of a distributed bench run, in order, with their wall-time budgets (s) — generous
# multiples of what C4 takes (the replicated build ~5 s, partition ~20 s, verify ~2 s); a phase
# that overruns is a hang (e.g. a peer that never joined an RCCL call) and ends the rank
DIST_PHASES = (("init", 300), ("build", 900), ("sync_formats", 300), ("uid_broadcast", 300),
               ("comm_create", 600), ("partition", 900), ("verify", 600), ("warmup", 300),
               ("timed", 600), ("roofline", 300), ("gather", 300), ("report", 900),
               ("teardown", 300))


def dist_timeout_s():
    """Timeout of every gloo collective (init, barriers, object broadcasts): the environment's
    MLAMG_DIST_TIMEOUT_S, default 600 s (torch's own default is 30 min)."""
    return float(os.environ.get("MLAMG_DIST_TIMEOUT_S", "600"))


class PhaseLog:
    """Rank-tagged phase markers on stderr and a watchdog (VERDICT r04 Weak #5).

    enter(name) prints `[mlamg rank r/w] phase <name> t=<s>` on every rank and starts that
    phase's budget (DIST_PHASES x MLAMG_PHASE_TIMEOUT_SCALE). A watchdog thread ends the process
    with EXIT_DIST_TIMEOUT, after printing the phase it was in, when a phase overruns its budget
    — e.g. a rank blocked in an RCCL call whose peer never arrives (ctypes and torch release the
    GIL while they wait, so the thread runs). fail() is the same exit for an error caught in the
    main thread (a gloo collective that timed out). The rank exits; it never re-executes or
    restarts itself, and a launcher (torch.distributed.run, bench.py's self-launch) then stops
    the other ranks."""

    def __init__(self, rank, world, scale=None, stream=None):
        import threading
        self.rank, self.world = rank, world
        self.scale = (float(os.environ.get("MLAMG_PHASE_TIMEOUT_SCALE", "1"))
                      if scale is None else float(scale))
        self.budgets = dict(DIST_PHASES)
        self.stream = stream if stream is not None else sys.stderr
        self.t0 = time.monotonic()
        self.name, self.started, self.deadline = "start", self.t0, None
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._th = threading.Thread(target=self._watch, daemon=True, name="mlamg-phase-watchdog")
        self._th.start()
        try:  # a launcher's SIGTERM (another rank failed): dump where every thread is, then die
            import faulthandler
            import signal
            faulthandler.register(signal.SIGTERM, file=self.stream, all_threads=True, chain=True)
        except (AttributeError, ValueError, OSError, io.UnsupportedOperation):
            pass

    def _say(self, msg):
        print(f"[mlamg rank {self.rank}/{self.world}] {msg}", file=self.stream, flush=True)

    def enter(self, name):
        now = time.monotonic()
        budget = self.budgets.get(name, 600) * self.scale
        with self._lock:
            prev, self.name, self.started, self.deadline = self.name, name, now, now + budget
        self._say(f"phase {name} t={now - self.t0:.1f}s (previous {prev}; budget {budget:.0f}s)")

    def selftest_stall_point(self):
        """phase_selftest only: MLAMG_SELFTEST_STALL=rank:phase makes that rank hang here."""
        stall = os.environ.get("MLAMG_SELFTEST_STALL")
        if stall and stall == f"{self.rank}:{self.name}":
            self._say(f"test hook: stalling in phase {self.name}")
            while True:
                time.sleep(1.0)

    def done(self):
        self._stop.set()
        self._say(f"done t={time.monotonic() - self.t0:.1f}s")

    def fail(self, why, code=EXIT_DIST_FAILED):
        with self._lock:
            name, started = self.name, self.started
        self._say(f"FAILED in phase {name} after {time.monotonic() - started:.1f}s "
                  f"(t={time.monotonic() - self.t0:.1f}s): {why}; exiting {code}")
        try:
            sys.stdout.flush()
        finally:
            os._exit(code)

    def _watch(self):
        while not self._stop.wait(0.1):
            with self._lock:
                late = self.deadline is not None and time.monotonic() > self.deadline
                name = self.name
            if late:
                self.fail(f"phase {name} exceeded its budget of "
                          f"{self.budgets.get(name, 600) * self.scale:.0f}s", EXIT_DIST_TIMEOUT)


def init_process_group(world, rank):
    if world > 1 and not dist.is_initialized():
        import datetime
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", world_size=world, rank=rank,
                                timeout=datetime.timedelta(seconds=dist_timeout_s()))


def _barrier(world):
    if world > 1:
        dist.barrier()


def _max(v, world):
    if world == 1:
        return v
    t = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def phase_selftest(world, rank):
    """bench.py --phase-selftest (CPU, gloo; no GPU work): every phase of a distributed bench
    run in order, each opened by a barrier, under the same PhaseLog — with
    MLAMG_SELFTEST_STALL=r:name rank r hangs in that phase (after its barrier, as a rank whose
    work in the phase never returns) and must exit non-zero naming it; its peer waits in the
    next phase's barrier (tests/test_bench_launch.py)."""
    ph = PhaseLog(rank, world)
    try:
        for name, _ in DIST_PHASES:
            ph.enter(name)
            if name == "init":
                init_process_group(world, rank)
            elif world > 1:
                dist.barrier()
            ph.selftest_stall_point()
        ph.done()
    except Exception as e:  # a gloo collective that timed out or lost its peer
        ph.fail(f"{type(e).__name__}: {e}")
    if rank == 0:
        print(json.dumps({"phase_selftest": True, "n_gpus": world,
                          "phases": [n for n, _ in DIST_PHASES]}), flush=True)
    if world > 1:
        dist.destroy_process_group()


class DistributedMismatch(RuntimeError):
    """The distributed cycle does not reproduce the single-GPU iterate on any executor path:
    bench.py must not time or print a throughput for it (it exits non-zero)."""


def verify_paths(check, D, graph_on, overlap_on):
    """Run check() (all ranks agree: its result is MIN-reduced over ranks) on the fastest
    executor path, falling back to overlap off, then to eager launches. Returns the
    (graph_on, overlap_on) that reproduce the single-GPU iterate; raises DistributedMismatch
    when none does — never time a path that computes a different answer."""
    ok = check()
    if not ok and overlap_on:
        overlap_on = False
        D.set_overlap(False)
        ok = check()
    if not ok and graph_on:
        graph_on = False
        D.set_cycle_graph(False)
        ok = check()
    if not ok:
        raise DistributedMismatch(
            "distributed V-cycle differs from the single-GPU iterate with overlap off and "
            "eager launches; refusing to report a throughput")
    return graph_on, overlap_on


def bench_main(args, world, rank, local_rank, metric, hbm_peak, phases=None):
    """bench.py for N > 1: strong scaling of one C4 problem over N GPUs. Returns
    (out, H, x0, teardown): `out` is the JSON dict on rank 0 (None elsewhere), H the replicated
    single-GPU hierarchy (rank 0's CPU baseline runs on it), teardown() ends the run (barrier,
    process group). Every rank reports its own fine-level SpMV roofline (cold launches timed by
    their dispatch packet, as the N = 1 line) and its communicator's rank count as RCCL itself
    reports it (ncclCommCount); rank 0 gathers them. `phases` (PhaseLog): every rank marks each
    phase on stderr and a phase that overruns its budget ends the rank (DIST_PHASES)."""
    from . import problems
    from .hierarchy import Hierarchy
    from .timing import time_kernel, time_kernel_cold

    ph = phases if phases is not None else PhaseLog(rank, world)

    def log(*a):
        if rank == 0:
            print("[bench]", *a, file=sys.stderr, flush=True)

    ph.enter("init")
    init_process_group(world, rank)
    torch.cuda.set_device(local_rank)
    ph.enter("build")
    n1 = args.n
    A = problems.poisson_3d_7pt(n1)
    n = A.shape[0]
    t0 = time.perf_counter()
    omr = getattr(args, "overlap_min_rows", 2_000_000)
    aggregation = getattr(args, "aggregation", "bellman_ford")
    dist_setup = bool(getattr(args, "dist_setup", False))
    H = None
    if dist_setup:
        # SURVEY.md §8(e) setup: each rank builds its rows of the partitioned levels
        # (mlamg.dsetup); only the tail below them is replicated
        from . import dsetup
        scomm = dsetup.setup_comm(world)
        S = dsetup.build_distributed(
            dsetup.split_rows(A, world, rank), n, scomm, alpha=args.alpha,
            strength_mode="invabs", aggregation=aggregation,
            A0_global=A if aggregation == "reference" else None, max_coarse=args.max_coarse,
            min_rows=args.dist_min_rows)
        setup_s = time.perf_counter() - t0
        log("distributed setup phases (s, rank 0): " + json.dumps(S.times))
        comm = Comm(world, rank, phases=ph)
        cinfo = comm.info()
        ph.enter("partition")
        t1 = time.perf_counter()
        D = DistributedHierarchy.from_setup(S, comm, overlap_min_rows=None if omr < 0 else omr)
        n_levels = len(S.parts) + S.tail.n_levels
    else:
        H = Hierarchy.build(A, alpha=args.alpha, strength_mode="invabs",
                            max_coarse=args.max_coarse, aggregation=aggregation,
                            coarse_order=getattr(args, "coarse_order", "sorted"),
                            finalize=False)
        ph.enter("sync_formats")
        finalize_replicated(H, world, rank)
        setup_s = time.perf_counter() - t0
        comm = Comm(world, rank, phases=ph)
        cinfo = comm.info()
        ph.enter("partition")
        t1 = time.perf_counter()
        D = DistributedHierarchy(H, comm, min_rows=args.dist_min_rows, A_host=A,
                                 overlap_min_rows=None if omr < 0 else omr)
        n_levels = H.n_levels
    part_s = time.perf_counter() - t1
    log("partition phases (s): " + json.dumps({k: round(v, 3) for k, v in D.setup_times.items()}))
    log(f"setup {setup_s:.1f}s ({'distributed' if dist_setup else 'replicated'}), "
        f"partition+upload {part_s:.1f}s; {D.K} of {n_levels} levels partitioned; rank rows "
        f"{D.lo}..{D.hi}; ghosts (x, r, p) per level {D.ghosts}; communicator {cinfo}")
    ph.enter("verify")
    x0 = np.random.RandomState(0).randn(n)
    x0 /= np.linalg.norm(x0)
    b_own = torch.zeros(D.n_own, dtype=torch.float64, device="cuda")
    ncheck = 5
    if dist_setup:
        # no replicated hierarchy to compare with: the timed path must reproduce the eager,
        # overlap-free cycle of the same distributed hierarchy bit for bit (the setup itself is
        # bitwise the replicated build given the same lambda_max: tests/test_gpu_dsetup.py)
        D.set_cycle_graph(False)
        D.set_overlap(False)
        x_ref = D.new_x(torch.as_tensor(x0[D.lo:D.hi]))
        h_single = D.cycle(b_own, x_ref, ncheck)
        x_ref_own = x_ref[: D.n_own].clone()
        D.set_overlap(True)
        ref_name = "eager distributed"
    else:
        # correctness: the distributed iterate equals the single-GPU iterate (replicated here)
        b_full = torch.zeros(n, dtype=torch.float64, device="cuda")
        x_full = torch.as_tensor(x0).cuda()
        h_single = H.cycle(b_full, x_full, ncheck, use_graph=True)
        x_ref_own = x_full[D.lo:D.hi]
        ref_name = "single-GPU"

    def check():
        x_ext = D.new_x(torch.as_tensor(x0[D.lo:D.hi]))
        try:
            h_dist = D.cycle(b_own, x_ext, ncheck)
        except _lib.MlamgError as e:
            log(f"distributed cycle failed: {e}")
            h_dist = np.full(ncheck, np.nan)
        same_x = bool(torch.equal(x_ext[: D.n_own], x_ref_own))
        same_h = bool(len(h_dist) == len(h_single)
                      and np.allclose(h_dist, h_single, rtol=1e-10, atol=0))
        ok = torch.tensor([1.0 if (same_x and same_h) else 0.0])
        if world > 1:
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        log(f"distributed vs {ref_name} after {ncheck} cycles: x bitwise "
            f"{same_x}, history {same_h} ({h_dist[-1]:.6e} vs {h_single[-1]:.6e})")
        return bool(ok.item() == 1.0)

    graph_on = not args.no_graph
    overlap_on = bool(D.splits)
    D.set_cycle_graph(graph_on)
    graph_on, overlap_on = verify_paths(check, D, graph_on, overlap_on)
    ok_all = True
    x_ref_own = None
    # timing
    ph.enter("warmup")
    x_ext = D.new_x(torch.as_tensor(x0[D.lo:D.hi]))
    D.cycle(b_own, x_ext, args.warmup, history=False)
    torch.cuda.synchronize()
    _barrier(world)
    ph.enter("timed")
    torch.cuda.synchronize()
    ta = time.perf_counter()
    D.cycle(b_own, x_ext, args.steps, history=False)
    torch.cuda.synchronize()
    _barrier(world)
    dt = _max(time.perf_counter() - ta, world)
    # per-rank fine-level SpMV (local rows) for the roofline: cold launches (a 512 MB read
    # before each), each timed by its own dispatch packet — the N = 1 line's method; warm
    # back-to-back launches beside it (the local operator can sit in the MALL at world 8)
    ph.enter("roofline")
    xs = torch.randn(D.n_ext, dtype=torch.float64, device="cuda")
    ys = torch.empty(D.n_own, dtype=torch.float64, device="cuda")
    t_spmv, t_med, t_ev = time_kernel_cold(lambda: D.A_loc.matvec(xs, out=ys), reps=20)
    t_warm = time_kernel(lambda: D.A_loc.matvec(xs, out=ys), reps=50)
    B = D.A_loc.format_bytes()  # bytes the chosen storage format streams for y = A_loc x_ext
    B_csr = 12.0 * D.A_loc.nnz + 4.0 * (D.n_own + 1) + 8.0 * D.n_ext + 8.0 * D.n_own
    mine = {"rank": rank, "rccl_nranks": cinfo["nranks"], "rccl_rank": cinfo["rank"],
            "device": cinfo["device"], "transport": cinfo["transport"],
            "rows": [int(D.lo), int(D.hi)], "format": D.A_loc.get_format()[0],
            "format_bytes": B, "us": round(t_spmv * 1e6, 2),
            "median_us": round(t_med * 1e6, 2), "stream_event_us": round(t_ev * 1e6, 2),
            "warm_us": round(t_warm * 1e6, 2),
            "GBps": round(B / t_spmv / 1e9, 1), "frac": round(B / t_spmv / 1e9 / hbm_peak, 4),
            "warm_frac": round(B / t_warm / 1e9 / hbm_peak, 4),
            "partition_s": {k: round(v, 3) for k, v in D.setup_times.items()},
            "memory": rank_memory()}
    ph.enter("gather")
    per_rank = [None] * world
    if world > 1:
        dist.all_gather_object(per_rank, mine)
    else:
        per_rank = [mine]
    out = None
    if rank == 0:
        slow = min(per_rank, key=lambda r: r["GBps"])
        pmc = _load_rank_pmc(world, slow["format"], slow["format_bytes"])
        out = {
            "metric": metric,
            "value": round(args.steps / dt, 3),
            "unit": "V-cycles/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {
                "workload": f"C4: 3D 7-point Laplace {n1}^3 ({n} DoF), SA-AMG V(1,1) weighted "
                            f"Jacobi, {D.K} finest levels row-split over {world} GPUs + RCCL "
                            f"halos, {n_levels - D.K} coarser levels replicated; aggregation "
                            f"{aggregation} (coarse order sorted); setup "
                            f"{'distributed' if dist_setup else 'replicated'}",
                "aggregation": aggregation,
                "setup": "distributed" if dist_setup else "replicated",
                "partitioned_levels": D.K,
                "overlap_splits": [(s["level"], s["op"]) for s in D.splits] if overlap_on else [],
                "n": n, "levels": n_levels, "parallelism": f"rowsplit{world}",
                "dist_matches_single_gpu": bool(ok_all),
                "cycle_graph": graph_on,
                "rccl_nranks": sorted({r["rccl_nranks"] for r in per_rank}),
                "devices": [r["device"] for r in per_rank],
                "rank0_local_formats": [
                    {k: t["chosen"] for k, t in zip("APR", D.tuning[3 * l:3 * l + 3])}
                    for l in range(D.K)],
            },
            "roofline": {
                "bound": "hbm", "kernel": f"fine-level SpMV ({slow['format']}), local rows "
                                          f"(slowest rank {slow['rank']})",
                "achieved": slow["GBps"], "peak": hbm_peak, "unit": "GB/s",
                "frac": slow["frac"],
                "traffic": pmc.get("hbm_bytes_per_launch") if pmc else None,
                "algorithmic_bytes_per_launch": slow["format_bytes"],
                "csr_algorithmic_bytes_per_launch": B_csr,
                "avg_launch_us": slow["us"],
                "timing": "per rank: mean of 20 cold launches (a 512 MB read before each), each "
                          "timed by the events of its own dispatch packet (hipExtLaunchKernel); "
                          "the slowest rank's",
                "warm_avg_launch_us": slow["warm_us"],
            },
            "per_rank_spmv": per_rank,
            "setup_s": {("distributed_build" if dist_setup else "replicated_build"):
                        round(setup_s, 3), "partition": round(part_s, 3),
                        "partition_phases_rank0": {k: round(v, 3)
                                                   for k, v in D.setup_times.items()},
                        **({"distributed_phases_rank0": S.times} if dist_setup else {})},
        }
    ph.enter("report")

    def teardown():
        nonlocal D
        ph.enter("teardown")
        _barrier(world)
        D = None
        if world > 1:
            dist.destroy_process_group()
        ph.done()

    return out, H, x0, teardown


def _load_rank_pmc(world, fmt, format_bytes):
    """PMC-measured HBM bytes of one rank's local fine SpMV (profiles/spmv_w{world}_pmc_{fmt}.json,
    written by tools/pmc_traffic.py on the same local operator), if its bytes match."""
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    path = os.path.join(root, "profiles", f"spmv_w{world}_pmc_{fmt}.json")
    try:
        with open(path) as fh:
            d = json.load(fh)
    except (OSError, ValueError):
        return None
    return d if d.get("algorithmic_bytes_per_launch") == format_bytes else None
