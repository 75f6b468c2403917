"""CPU: the host side of the distributed setup (mlamg/dsetup.py) — the setup transport (ranks as
threads, and torch.distributed gloo at world 2), the halo maps on globally indexed arrays
(forward, reverse-min, row fetch), the routing that forms R = P^T's owned rows, and the
Bellman-Ford exchange protocol, driven with a CPU restatement of the csrc/graph.hip sweep
kernels: at every world size the labels equal the world-1 run (the order-independent fixed
point), ties included. The device kernels themselves are covered in tests/test_gpu_dsetup.py."""
import os
import socket

import numpy as np
import pytest
import scipy.sparse as sp
import torch

from mlamg import dsetup, partition
from mlamg.partition import TCSR

INT32_MAX = 2 ** 31 - 1


def _grid(m):
    """2-D 5-point Laplacian on an m x m grid (scipy CSR, sorted indices)."""
    I = sp.identity(m)
    T = sp.diags([-1.0, 2.0, -1.0], [-1, 0, 1], shape=(m, m))
    return (sp.kron(I, T) + sp.kron(T, I)).tocsr()


def _gs(T, lo, n):
    """A global-shaped CPU CSR (rows outside [lo, lo + T.shape[0]) empty) as a TCSR."""
    lens = (T.crow[1:] - T.crow[:-1]).to(torch.int64)
    full = torch.zeros(n, dtype=torch.int64)
    full[lo:lo + T.shape[0]] = lens
    crow = torch.zeros(n + 1, dtype=torch.int64)
    crow[1:] = torch.cumsum(full, 0)
    return TCSR(crow, T.col.to(torch.int32), T.val, (n, T.shape[1]))


class CpuBF:
    """Row-sequential restatement of k_bf_init / k_bf_seeds / k_bf_sweep / k_bf_label /
    k_lab_finish (csrc/graph.hip): push relaxations in fp32, min-labels along tight edges."""

    def begin(self, C, seeds, w, dist, lab, is_seed):
        w[:C.nnz] = C.val.to(torch.float32)
        dist.fill_(float("inf"))
        lab.fill_(INT32_MAX)
        is_seed.zero_()
        s = seeds.to(torch.int64)
        dist[s] = 0.0
        lab[s] = s.to(torch.int32)
        is_seed[s] = 1

    def sweep(self, C, w, dist, changed):
        crow, col, wn, d = C.crow.numpy(), C.col.numpy(), w.numpy(), dist.numpy()
        for i in range(C.shape[0]):
            di = d[i]
            if not di < np.float32(np.inf):
                continue
            for k in range(crow[i], crow[i + 1]):
                j = col[k]
                cand = np.float32(di + wn[k])
                if cand < d[j]:
                    d[j] = cand
                    changed[0] = 1

    def label(self, C, w, dist, is_seed, lab, changed):
        crow, col, wn, d = C.crow.numpy(), C.col.numpy(), w.numpy(), dist.numpy()
        lb, sd = lab.numpy(), is_seed.numpy()
        for i in range(C.shape[0]):
            if not d[i] < np.float32(np.inf) or lb[i] == INT32_MAX:
                continue
            for k in range(crow[i], crow[i + 1]):
                j = col[k]
                if sd[j]:
                    continue
                if np.float32(d[i] + wn[k]) == d[j] and lb[i] < lb[j]:
                    lb[j] = lb[i]
                    changed[0] = 1

    def end(self, lab):
        lab[lab == INT32_MAX] = -1


def _labels(A, world, seeds):
    n = A.shape[0]
    ranges = partition.row_ranges(n, world)

    def rank_fn(comm):
        lo, hi = ranges[comm.rank]
        T = TCSR.from_scipy(A[lo:hi])
        hx = dsetup.GHalo(comm, dsetup._ghosts(T, lo, hi), ranges)
        lab, sweeps = dsetup.bellman_ford_distributed(_gs(T, lo, n), seeds, hx, comm,
                                                      kernels=CpuBF())
        return lab[lo:hi].clone(), sweeps

    out = dsetup.run_threads(world, rank_fn, device=torch.device("cpu"))
    return torch.cat([o[0] for o in out]).numpy(), [o[1] for o in out]


def test_thread_comm_collectives():
    def fn(comm):
        got = comm.allgather_obj(comm.rank * 10)
        sends = {q: torch.full((q + 1,), float(comm.rank), dtype=torch.float64)
                 for q in range(comm.world)}
        recvs = {q: (comm.rank + 1, torch.float64) for q in range(comm.world)}
        x = comm.exchange(sends, recvs)
        return got, {q: x[q].tolist() for q in x}

    out = dsetup.run_threads(3, fn, device=torch.device("cpu"))
    for r, (got, x) in enumerate(out):
        assert got == [0, 10, 20]
        assert x == {q: [float(q)] * (r + 1) for q in range(3)}


def test_thread_comm_error_reaches_caller():
    def fn(comm):
        if comm.rank == 1:
            raise KeyError("rank 1 failed")
        comm.allgather_obj(0)  # the others block here until the barrier is aborted

    with pytest.raises(KeyError):
        dsetup.run_threads(3, fn, device=torch.device("cpu"))


@pytest.mark.parametrize("world", [2, 3, 5])
def test_halo_forward_reverse_and_row_fetch(world):
    A = sp.random(90, 90, density=0.06, random_state=3, format="csr") + sp.identity(90)
    A = A.tocsr()
    A.sort_indices()
    n = A.shape[0]
    ranges = partition.row_ranges(n, world)
    v = np.random.RandomState(0).rand(n)

    def fn(comm):
        lo, hi = ranges[comm.rank]
        T = TCSR.from_scipy(A[lo:hi])
        g = dsetup._ghosts(T, lo, hi)
        hx = dsetup.GHalo(comm, g, ranges)
        arr = torch.full((n,), -1.0, dtype=torch.float64)
        arr[lo:hi] = torch.as_tensor(v[lo:hi])
        hx.forward(arr)
        fwd = arr[g].numpy().copy()
        # ghost copies lowered to 0.5 * value: every holder's copy reaches the owner as a min
        arr[g] = arr[g] * 0.5
        hx.reverse_min(arr)
        rows = hx.fetch_rows(T, lo)
        return g.numpy(), fwd, arr[lo:hi].numpy(), rows

    out = dsetup.run_threads(world, fn, device=torch.device("cpu"))
    held = np.zeros(n, bool)
    for r, (g, fwd, own, rows) in enumerate(out):
        lo, hi = ranges[r]
        assert np.array_equal(fwd, v[g])
        held[g] = True
        R = rows.to_scipy()
        ref = A[g]
        assert np.array_equal(R.indptr, ref.indptr) and np.array_equal(R.indices, ref.indices)
        assert np.array_equal(R.data, ref.data)
    for r, (_, _, own, _) in enumerate(out):
        lo, hi = ranges[r]
        expect = np.where(held[lo:hi], 0.5 * v[lo:hi], v[lo:hi])
        assert np.array_equal(own, expect)


@pytest.mark.parametrize("world", [1, 2, 4])
def test_route_transpose_forms_owned_rows_of_PT(world):
    rs = np.random.RandomState(5)
    n, nc = 120, 30
    seeds = np.sort(rs.choice(n, nc, replace=False))
    P = sp.random(n, nc, density=0.15, random_state=7, format="csr")
    P.sort_indices()
    ranges = partition.row_ranges(n, world)
    c_ranges = partition._seed_ranges(seeds, ranges, nc)
    RT = P.T.tocsr()
    RT.sort_indices()

    def fn(comm):
        lo, hi = ranges[comm.rank]
        T = TCSR.from_scipy(P[lo:hi])
        return dsetup._route_transpose(comm, T, lo, n, c_ranges).to_scipy()

    out = dsetup.run_threads(world, fn, device=torch.device("cpu"))
    for r, R in enumerate(out):
        clo, chi = c_ranges[r]
        ref = RT[clo:chi]
        assert R.shape == ref.shape
        assert np.array_equal(R.indptr, ref.indptr)
        assert np.array_equal(R.indices, ref.indices)
        assert np.array_equal(R.data, ref.data)


@pytest.mark.parametrize("world", [2, 3, 7])
def test_bellman_ford_protocol_matches_one_rank(world):
    """Unit weights on a grid: many shortest paths tie, so the labels depend on the min rule,
    not on an order — world 1 and world 2/3/7 must give the same labels bit for bit."""
    A = _grid(14)
    C = A.copy()
    C.data[:] = 1.0
    C.setdiag(0.0)
    C.eliminate_zeros()
    C.sort_indices()
    n = C.shape[0]
    seeds = torch.as_tensor(np.sort(np.random.RandomState(2).permutation(n)[:20]).astype(np.int32))
    lab1, _ = _labels(C, 1, seeds)
    labw, sweeps = _labels(C, world, seeds)
    assert (lab1 >= 0).all()
    assert np.array_equal(lab1, labw)
    assert len(set(sweeps)) == 1  # every rank ran the same number of exchange rounds


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gloo_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        comm = dsetup.TorchComm(device=torch.device("cpu"))
        A = _grid(10)
        C = A.copy()
        C.data[:] = 1.0
        C.setdiag(0.0)
        C.eliminate_zeros()
        C.sort_indices()
        n = C.shape[0]
        ranges = partition.row_ranges(n, world)
        lo, hi = ranges[rank]
        T = TCSR.from_scipy(C[lo:hi])
        hx = dsetup.GHalo(comm, dsetup._ghosts(T, lo, hi), ranges)
        seeds = torch.as_tensor(np.sort(np.random.RandomState(4).permutation(n)[:12])
                                .astype(np.int32))
        lab, _ = dsetup.bellman_ford_distributed(_gs(T, lo, n), seeds, hx, comm,
                                                 kernels=CpuBF())
        rows = hx.fetch_rows(T, lo).to_scipy()
        ok_rows = (np.array_equal(rows.indices, C[hx.ghosts.numpy()].indices))
        q.put((rank, lab[lo:hi].numpy().tolist(), bool(ok_rows)))
    finally:
        dist.destroy_process_group()


def test_torch_comm_gloo_world2():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict()
    for _ in range(2):
        r, lab, ok = q.get(timeout=240)
        got[r] = (lab, ok)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    A = _grid(10)
    C = A.copy()
    C.data[:] = 1.0
    C.setdiag(0.0)
    C.eliminate_zeros()
    C.sort_indices()
    n = C.shape[0]
    seeds = torch.as_tensor(np.sort(np.random.RandomState(4).permutation(n)[:12])
                            .astype(np.int32))
    lab1, _ = _labels(C, 1, seeds)
    assert got[0][1] and got[1][1]
    assert np.array_equal(np.array(got[0][0] + got[1][0]), lab1)
