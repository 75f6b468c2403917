"""CPU, world_size 2 and 3 over gloo: the row partition + halo maps of mlamg.partition (the host
logic the RCCL executor runs on) reproduce the single-process V-cycle bit for bit.

Each rank emulates csrc/comm.hip's distributed cycle step for step with the oracle's arithmetic
(scipy csr_matvec order) and torch.distributed (gloo) point-to-point messages in place of RCCL.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _halo(ext, halo, n_own, tag):
    """Exchange ghost values of ext (numpy, [owned | ghosts]) in place."""
    reqs = []
    off = 0
    bufs = []
    soff = 0
    for q, sc, rc in zip(halo.neighbors, halo.send_counts, halo.recv_counts):
        if sc:
            sb = torch.from_numpy(np.ascontiguousarray(ext[halo.send_idx[soff:soff + sc]]))
            bufs.append(sb)
            reqs.append(dist.isend(sb, dst=q, tag=tag))
        soff += sc
        if rc:
            rb = torch.empty(rc, dtype=torch.float64)
            bufs.append((rb, n_own + off))
            reqs.append(dist.irecv(rb, src=q, tag=tag))
        off += rc
    for r in reqs:
        r.wait()
    for b in bufs:
        if isinstance(b, tuple):
            rb, o = b
            ext[o:o + len(rb)] = rb.numpy()


def _allgatherv(bc, c_ranges, rank, world, tag):
    lo, hi = c_ranges[rank]
    reqs, recv = [], []
    mine = torch.from_numpy(np.ascontiguousarray(bc[lo:hi]))
    for q in range(world):
        if q == rank:
            continue
        if hi > lo:
            reqs.append(dist.isend(mine, dst=q, tag=tag))
        a, b = c_ranges[q]
        if b > a:
            t = torch.empty(b - a, dtype=torch.float64)
            recv.append((t, a))
            reqs.append(dist.irecv(t, src=q, tag=tag))
    for r in reqs:
        r.wait()
    for t, a in recv:
        bc[a:a + len(t)] = t.numpy()


def _problem(kind):
    from mlamg import problems
    if kind == "3d":
        return problems.poisson_3d_7pt(10)
    return problems.jump_2d(30, np.array([[0.3, 0.4, 1e-2], [0.7, 0.6, 1e2]]))


def _worker(rank, world, port, kind, ncyc, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import scipy.sparse as sp
        import scipy.sparse.linalg as spla
        from mlamg import partition
        from oracle import restated as orc

        A = _problem(kind)
        n = A.shape[0]
        levels, Ac = orc.build_hierarchy(A, alpha=0.1, seed=0, sort_seeds=True, max_coarse=40,
                                         omegas=[0.61, 0.63, 0.65, 0.67, 0.69])
        lu = spla.factorized(sp.csc_matrix(Ac))
        x0 = np.random.RandomState(0).randn(n)
        b = np.random.RandomState(1).randn(n)
        x_ref, h_ref = orc.vcycle_solve(levels, Ac, b, x0, ncyc, lu=lu)
        L0 = levels[0]
        p = partition.build(L0["A"], L0["P"], L0["seeds"], world, rank)
        lo, hi = p["lo"], p["hi"]
        n_own = hi - lo
        d = L0["Dw"].diagonal()[lo:hi]
        bo = b[lo:hi]
        hx, hr = p["halo_x"], p["halo_r"]
        x = np.zeros(n_own + hx.n_ghost)
        x[:n_own] = x0[lo:hi]
        r = np.zeros(n_own + hr.n_ghost)
        coarse = orc.make_cycle(levels[1:], lu)
        tag = 0

        def resid(v):
            return bo - orc.csr_matvec(p["A_loc"], v)

        _halo(x, hx, n_own, tag)
        r[:n_own] = resid(x)
        hist = []
        for _ in range(ncyc):
            x[:n_own] = x[:n_own] + d * r[:n_own]
            tag += 1
            _halo(x, hx, n_own, tag)
            r[:n_own] = resid(x)
            tag += 1
            _halo(r, hr, n_own, tag)
            bc = np.zeros(p["nc"])
            clo, chi = p["c_lo"], p["c_hi"]
            bc[clo:chi] = orc.csr_matvec(p["R_own"], r)
            tag += 1
            _allgatherv(bc, p["c_ranges"], rank, world, tag)
            xc = coarse(0, bc, None)
            x[:n_own] = x[:n_own] + orc.csr_matvec(p["P_loc"], xc)
            tag += 1
            _halo(x, hx, n_own, tag)
            t = np.zeros_like(x)
            t[:n_own] = x[:n_own] + d * resid(x)
            tag += 1
            _halo(t, hx, n_own, tag)
            r[:n_own] = resid(t)
            s = torch.tensor([float(np.dot(r[:n_own], r[:n_own]))], dtype=torch.float64)
            dist.all_reduce(s)
            hist.append(float(np.sqrt(s.item())))
            x[:n_own] = t[:n_own]
        same_x = bool(np.array_equal(x[:n_own], x_ref[lo:hi]))
        same_h = bool(np.allclose(hist, h_ref, rtol=1e-12, atol=0))
        q.put((rank, same_x, same_h, hx.n_ghost, hr.n_ghost, len(hx.neighbors)))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported through the queue
        import traceback
        q.put((rank, "error", traceback.format_exc()))


@pytest.mark.parametrize("world,kind", [(2, "3d"), (3, "3d"), (2, "jump")])
def test_partitioned_vcycle_bitwise(world, kind):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kind, 4, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
    for item in res:
        assert item[1] != "error", item[2]
        rank, same_x, same_h, gx, gr, nn = item
        assert same_x, f"rank {rank}: iterate differs from the single-process cycle"
        assert same_h, f"rank {rank}: residual history differs"
        assert gx > 0 and gr > 0 and nn >= 1


def test_row_ranges_and_owner():
    from mlamg import partition
    rr = partition.row_ranges(10, 3)
    assert rr == [(0, 4), (4, 7), (7, 10)]
    his = np.array([h for _, h in rr])
    assert list(partition.owner_of(np.array([0, 3, 4, 6, 7, 9]), his)) == [0, 0, 1, 1, 2, 2]


def test_partition_rejects_unsorted_seeds():
    import scipy.sparse as sp
    from mlamg import partition, problems
    A = problems.poisson_1d(12)
    P = sp.csr_matrix((np.ones(12), np.arange(12) // 3, np.arange(13)), shape=(12, 4))
    with pytest.raises(ValueError):
        partition.build(A, P, np.array([9, 0, 3, 6]), 2)
