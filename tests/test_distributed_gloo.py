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


def _worker(rank, world, port, kind, ncyc, K, q):
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
        K = min(K, len(levels))
        lu = spla.factorized(sp.csc_matrix(Ac))
        x0 = np.random.RandomState(0).randn(n)
        b = np.random.RandomState(1).randn(n)
        x_ref, h_ref = orc.vcycle_solve(levels, Ac, b, x0, ncyc, lu=lu)
        parts = partition.build_levels([levels[l]["A"] for l in range(K)],
                                       [levels[l]["P"] for l in range(K)],
                                       [levels[l]["seeds"] for l in range(K)], world, rank)
        dl = [levels[l]["Dw"].diagonal()[p["lo"]:p["hi"]] for l, p in enumerate(parts)]
        coarse = orc.make_cycle(levels[K:], lu)
        tag = [0]

        def halo(v, h, n_own):
            tag[0] += 1
            _halo(v, h, n_own, tag[0])

        def ext(l):
            p = parts[l]
            return np.zeros(p["hi"] - p["lo"] + max(p["halo_x"].n_ghost, p["halo_r"].n_ghost))

        # emulation of csrc/comm.hip: correct / dcycle_below / dcycle
        def correct(l, r):
            p = parts[l]
            m = p["hi"] - p["lo"]
            halo(r, p["halo_r"], m)
            if p["halo_p"] is not None:
                xn = below(l + 1, orc.csr_matvec(p["R_own"], r))
                hp = p["halo_p"]
                xp = np.zeros(hp.n_own + hp.n_ghost)
                xp[:hp.n_own] = xn
                halo(xp, hp, hp.n_own)
                return orc.csr_matvec(p["P_loc"], xp)
            bc = np.zeros(p["nc"])
            bc[p["c_lo"]:p["c_hi"]] = orc.csr_matvec(p["R_own"], r)
            tag[0] += 1
            _allgatherv(bc, p["c_ranges"], rank, world, tag[0])
            return orc.csr_matvec(p["P_loc"], coarse(0, bc, None))

        def prolong(l, x, r):
            # P_loc rows = owned + x-ghost rows: the ghosts are updated locally (no x halo)
            k = parts[l]["P_loc"].shape[0]
            x[:k] = x[:k] + correct(l, r)

        def below(l, bl):
            p = parts[l]
            m = p["hi"] - p["lo"]
            d = dl[l]
            x, r = ext(l), ext(l)
            x[:m] = d * bl
            halo(x, p["halo_x"], m)
            r[:m] = bl - orc.csr_matvec(p["A_loc"], x)
            prolong(l, x, r)
            return x[:m] + d * (bl - orc.csr_matvec(p["A_loc"], x))

        p0 = parts[0]
        lo, hi = p0["lo"], p0["hi"]
        n_own = hi - lo
        d = dl[0]
        bo = b[lo:hi]
        hx = p0["halo_x"]
        x, r = ext(0), ext(0)
        x[:n_own] = x0[lo:hi]

        def resid(v):
            return bo - orc.csr_matvec(p0["A_loc"], v)

        halo(x, hx, n_own)
        r[:n_own] = resid(x)
        hist = []
        for _ in range(ncyc):
            x[:n_own] = x[:n_own] + d * r[:n_own]
            halo(x, hx, n_own)
            r[:n_own] = resid(x)
            prolong(0, x, r)
            t = np.zeros_like(x)
            t[:n_own] = x[:n_own] + d * resid(x)
            halo(t, hx, n_own)
            r[:n_own] = resid(t)
            s = torch.tensor([float(np.dot(r[:n_own], r[:n_own]))], dtype=torch.float64)
            dist.all_reduce(s)
            hist.append(float(np.sqrt(s.item())))
            x[:n_own] = t[:n_own]
        same_x = bool(np.array_equal(x[:n_own], x_ref[lo:hi]))
        same_h = bool(np.allclose(hist, h_ref, rtol=1e-12, atol=0))
        gp = [pp["halo_p"].n_ghost for pp in parts[:-1]]
        q.put((rank, same_x, same_h, hx.n_ghost, p0["halo_r"].n_ghost, len(hx.neighbors), K,
               gp))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:  # pragma: no cover - reported through the queue
        import traceback
        q.put((rank, "error", traceback.format_exc()))


@pytest.mark.parametrize("world,kind,K", [(2, "3d", 1), (3, "3d", 1), (2, "jump", 1),
                                          (2, "3d", 2), (3, "3d", 9), (2, "jump", 9)])
def test_partitioned_vcycle_bitwise(world, kind, K):
    """K = number of finest levels row-partitioned (9 = all above the coarse solve)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kind, 4, K, q))
             for r in range(world)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
    for item in res:
        assert item[1] != "error", item[2]
        rank, same_x, same_h, gx, gr, nn, k_used, gp = item
        assert same_x, f"rank {rank}: iterate differs from the single-process cycle (K={k_used})"
        assert same_h, f"rank {rank}: residual history differs (K={k_used})"
        assert gx > 0 and gr > 0 and nn >= 1
        assert len(gp) == k_used - 1
        if K > 1:
            assert k_used >= 2


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
