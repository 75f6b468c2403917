"""GPU, one process: the distributed setup (mlamg/dsetup.py, SURVEY.md §8(e) "Setup") with the
ranks as host threads of this process on one device.

* With every level's lambda_max supplied (the single-GPU values), each rank's partition maps —
  local A / R / P operators, halos, coarse ranges — are array for array the maps
  partition.build_levels_torch cuts from the replicated single-GPU hierarchy, its labels,
  seeds and Jacobi weights equal the single-GPU level's, and the replicated tail equals the
  single-GPU levels below (bitwise), at worlds 1, 2, 3, 5 and 8; then the executor built from
  the setup (DistributedHierarchy.from_setup, loopback transport) runs the single-GPU V-cycle
  bit for bit.
* With the distributed Lanczos, lambda_max agrees with the single-GPU Lanczos to 1e-13 and the
  cycle to 1e-12 relative, the aggregates still bitwise.
* aggregation='reference' (level 0 by the reference's push-order sweep, replicated): the maps
  equal the single-GPU hierarchy built with coarse_order='sorted'."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def prob():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mlamg import problems
    from mlamg.hierarchy import Hierarchy
    A = problems.poisson_3d_7pt(36)
    H = Hierarchy.build(A, alpha=0.1, max_coarse=200)
    assert H.n_levels >= 3
    return A, H


def _setups(A, world, **kw):
    from mlamg import dsetup
    n = A.shape[0]

    def fn(comm):
        return dsetup.build_distributed(dsetup.split_rows(A, world, comm.rank), n, comm, **kw)

    return dsetup.run_threads(world, fn)


def _tcsr_equal(T, ref, what):
    import torch
    a = [T.crow.to(torch.int64).cpu(), T.col.to(torch.int64).cpu(), T.val.cpu()]
    b = [ref.crow.to(torch.int64).cpu(), ref.col.to(torch.int64).cpu(), ref.val.cpu()]
    assert T.shape == ref.shape, what
    for x, y, part in zip(a, b, ("crow", "col", "val")):
        assert torch.equal(x, y), f"{what}: {part} differs"


def _halo_equal(h, ref, what):
    if ref is None:
        assert h is None, what
        return
    assert np.array_equal(h.ghosts, ref.ghosts), what
    assert h.neighbors == ref.neighbors, what
    assert h.recv_counts == ref.recv_counts and h.send_counts == ref.send_counts, what
    assert np.array_equal(h.send_idx, ref.send_idx), what


def _replicated_maps(H, K, world, rank):
    from mlamg import partition

    def tc(M):
        crow, col, val = M.to_torch()
        return partition.TCSR(crow, col, val, M.shape)

    return partition.build_levels_torch([tc(H.levels[l].A) for l in range(K)],
                                        [tc(H.levels[l].P) for l in range(K)],
                                        [tc(H.levels[l].R) for l in range(K)],
                                        [H.levels[l].seeds for l in range(K)], world, rank)


def _check_against(H, Ss, world):
    import torch
    K = len(Ss[0].parts)
    for r, S in enumerate(Ss):
        assert len(S.parts) == K
        ref = _replicated_maps(H, K, world, r)
        for l, (d, e) in enumerate(zip(S.parts, ref)):
            tag = f"world {world} rank {r} level {l}"
            for key in ("lo", "hi", "n", "nc", "c_lo", "c_hi", "c_ranges", "ranges"):
                assert d[key] == e[key], f"{tag}: {key}"
            for key in ("A_loc", "R_own", "P_loc"):
                _tcsr_equal(d[key], e[key], f"{tag}: {key}")
            for key in ("halo_x", "halo_r", "halo_p"):
                _halo_equal(d[key], e[key], f"{tag}: {key}")
            L = H.levels[l]
            assert np.array_equal(S.seeds[l], L.seeds), tag
            lo, hi = d["lo"], d["hi"]
            assert torch.equal(S.labels[l][lo:hi].cpu(), L.labels[lo:hi].cpu()), tag
            assert torch.equal(S.dinv[l].cpu(), L.dinv[lo:hi].cpu()), tag
        # the replicated tail: H's levels K.. and its coarse operator, bitwise
        T = S.tail
        assert len(T.levels) == len(H.levels) - K
        for Lt, Lh in zip(T.levels, H.levels[K:]):
            for name in ("A", "P", "R"):
                a, b = getattr(Lt, name).to_scipy(), getattr(Lh, name).to_scipy()
                assert (np.array_equal(a.indptr, b.indptr) and np.array_equal(a.indices, b.indices)
                        and np.array_equal(a.data, b.data)), f"tail {name}"
        a, b = T.Ac.to_scipy(), H.Ac.to_scipy()
        assert np.array_equal(a.indptr, b.indptr) and np.array_equal(a.data, b.data)


@pytest.mark.parametrize("world,min_rows", [(1, 0), (2, 0), (3, 0), (5, 0), (8, 0), (3, 2000)])
def test_dsetup_maps_equal_replicated(prob, world, min_rows):
    A, H = prob
    Ss = _setups(A, world, alpha=0.1, max_coarse=200, min_rows=min_rows,
                 lams=[L.lam for L in H.levels])
    K = 1
    while K < len(H.levels) and H.levels[K].A.shape[0] >= min_rows:
        K += 1
    assert len(Ss[0].parts) == K
    _check_against(H, Ss, world)


def _cycle_from_setups(A, Ss, world, b, x0, ncyc=6):
    import torch
    from mlamg.distributed import DistributedHierarchy, LoopbackGroup
    group = LoopbackGroup(world)
    try:
        Ds = [DistributedHierarchy.from_setup(Ss[r], group.comms[r], overlap_min_rows=None)
              for r in range(world)]
        for D in Ds:
            D.set_cycle_graph(False)
            D.set_coarse_graph(False)
        bs = [torch.as_tensor(b[D.lo:D.hi]).cuda() for D in Ds]
        xs = [D.new_x(torch.as_tensor(x0[D.lo:D.hi])) for D in Ds]
        torch.cuda.synchronize()
        out, errs = [None] * world, []

        def work(r):
            try:
                torch.cuda.set_device(0)
                s = torch.cuda.Stream()
                with torch.cuda.stream(s):
                    h = Ds[r].cycle(bs[r], xs[r], ncyc)
                    s.synchronize()
                    out[r] = (xs[r][: Ds[r].n_own].cpu().numpy(), h)
            except Exception as e:  # surfaces in the main thread
                errs.append((r, e))

        th = [threading.Thread(target=work, args=(r,)) for r in range(world)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=300)
        assert not any(t.is_alive() for t in th), "a rank did not finish"
        assert not errs, errs
        return Ds, out
    finally:
        torch.cuda.synchronize()
        Ds = None
        group.close()


@pytest.mark.parametrize("world,min_rows", [(2, 0), (3, 2000), (8, 0)])
def test_executor_from_setup_bitwise(prob, world, min_rows):
    import torch
    A, H = prob
    n = A.shape[0]
    x0 = np.random.RandomState(0).randn(n)
    b = np.random.RandomState(1).randn(n)
    xd = torch.as_tensor(x0).cuda()
    h_ref = H.cycle(torch.as_tensor(b).cuda(), xd, 6, use_graph=False)
    x_ref = xd.cpu().numpy()
    Ss = _setups(A, world, alpha=0.1, max_coarse=200, min_rows=min_rows,
                 lams=[L.lam for L in H.levels])
    Ds, out = _cycle_from_setups(A, Ss, world, b, x0)
    for D, (x_own, h) in zip(Ds, out):
        assert np.array_equal(x_own, x_ref[D.lo:D.hi]), f"rank {D.comm.rank} of {world}"
        np.testing.assert_allclose(h, h_ref, rtol=1e-12, atol=0)


@pytest.mark.parametrize("world", [1, 3])
def test_distributed_lanczos_and_cycle(prob, world):
    import torch
    A, H = prob
    n = A.shape[0]
    Ss = _setups(A, world, alpha=0.1, max_coarse=200, min_rows=0)
    for S in Ss:
        assert S.lams == Ss[0].lams  # every rank reduces the same partials in the same order
        for l, lam in enumerate(S.lams):
            assert abs(lam - H.levels[l].lam) <= 1e-13 * abs(H.levels[l].lam)
            assert np.array_equal(S.seeds[l], H.levels[l].seeds)
            lo, hi = S.parts[l]["lo"], S.parts[l]["hi"]
            assert torch.equal(S.labels[l][lo:hi].cpu(), H.levels[l].labels[lo:hi].cpu())
    x0 = np.random.RandomState(0).randn(n)
    b = np.random.RandomState(1).randn(n)
    xd = torch.as_tensor(x0).cuda()
    h_ref = H.cycle(torch.as_tensor(b).cuda(), xd, 6, use_graph=False)
    x_ref = xd.cpu().numpy()
    Ds, out = _cycle_from_setups(A, Ss, world, b, x0)
    for D, (x_own, h) in zip(Ds, out):
        np.testing.assert_allclose(x_own, x_ref[D.lo:D.hi], rtol=1e-12,
                                   atol=1e-12 * np.abs(x_ref).max())
        np.testing.assert_allclose(h, h_ref, rtol=1e-12, atol=0)


@pytest.mark.parametrize("world", [2, 4])
def test_dsetup_reference_aggregation(world):
    import torch
    from mlamg import problems
    from mlamg.hierarchy import Hierarchy
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    A = problems.poisson_3d_7pt(30)
    H = Hierarchy.build(A, alpha=0.1, max_coarse=200, aggregation="reference",
                        coarse_order="sorted")
    Ss = _setups(A, world, alpha=0.1, max_coarse=200, min_rows=0, aggregation="reference",
                 A0_global=A, lams=[L.lam for L in H.levels])
    _check_against(H, Ss, world)


def test_dsetup_refuses_bad_input(prob):
    from mlamg import dsetup
    A, _ = prob
    n = A.shape[0]
    with pytest.raises(ValueError):
        dsetup.run_threads(1, lambda c: dsetup.build_distributed(
            dsetup.split_rows(A, 1, 0), n, c, aggregation="reference"))
    with pytest.raises(ValueError):
        dsetup.run_threads(2, lambda c: dsetup.build_distributed(
            dsetup.split_rows(A, 1, 0), n, c))  # rows of a world-1 split at world 2


def _mp_worker(rank, world, port, q):
    """One process of a gloo job on the shared GPU: the distributed setup over TorchComm (host
    copies through gloo), reporting digests of its maps."""
    import os
    import hashlib
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from mlamg import dsetup, problems
        from mlamg.hierarchy import Hierarchy
        A = problems.poisson_3d_7pt(24)
        n = A.shape[0]
        # the single-GPU lambda_max values, so that the maps compare bitwise (the distributed
        # Lanczos alone is held to 1e-13 below and in test_distributed_lanczos_and_cycle)
        lams = [L.lam for L in Hierarchy.build(A, alpha=0.1, max_coarse=100).levels]
        comm = dsetup.setup_comm(world)
        S = dsetup.build_distributed(dsetup.split_rows(A, world, rank), n, comm, alpha=0.1,
                                     max_coarse=100, min_rows=0, lams=lams)
        lam_d = [dsetup.lambda_max_distributed(
            dsetup._gs_csr(torch.arange(d["lo"], d["hi"], device="cuda"), A_own, d["n"],
                           d["n"]),
            dsetup.GHalo(comm, dsetup._ghosts(A_own, d["lo"], d["hi"]), d["ranges"]),
            d["lo"], d["hi"], comm)[0]
            for d, (A_own, _) in zip(S.parts, S.own_rows)]
        dig = []
        for d in S.parts:
            h = hashlib.sha256()
            for key in ("A_loc", "R_own", "P_loc"):
                T = d[key]
                for t in (T.crow.to(torch.int64), T.col.to(torch.int64), T.val):
                    h.update(t.cpu().numpy().tobytes())
            dig.append(h.hexdigest())
        q.put((rank, dig, lam_d, None))
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 — reported to the parent
        q.put((rank, None, None, repr(e)))


def test_dsetup_torch_comm_gloo_processes():
    """World 2 as two processes on the one GPU over torch.distributed (gloo): the same maps as
    the thread-transport run and the replicated build."""
    import hashlib
    import socket
    import torch
    import torch.multiprocessing as mp
    from mlamg import problems
    from mlamg.hierarchy import Hierarchy
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_mp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = {}
    for _ in range(2):
        r, dig, lams, err = q.get(timeout=240)
        assert err is None, f"rank {r}: {err}"
        got[r] = (dig, lams)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    A = problems.poisson_3d_7pt(24)
    H = Hierarchy.build(A, alpha=0.1, max_coarse=100)
    K = len(got[0][0])
    for r in range(2):
        ref = _replicated_maps(H, K, 2, r)
        for l, e in enumerate(ref):
            h = hashlib.sha256()
            for key in ("A_loc", "R_own", "P_loc"):
                T = e[key]
                for t in (T.crow.to(torch.int64), T.col.to(torch.int64), T.val):
                    h.update(t.cpu().numpy().tobytes())
            assert got[r][0][l] == h.hexdigest(), f"rank {r} level {l}"
        for l, lam in enumerate(got[r][1]):
            assert abs(lam - H.levels[l].lam) <= 1e-13 * abs(H.levels[l].lam)


def test_dsetup_c4_world8_bench_configuration():
    """The bench's C4 configuration (216^3, reference aggregation, max_coarse 2000, levels of
    >= 50,000 rows partitioned) at world 8: every rank's maps, labels and Jacobi weights are the
    replicated build's, bitwise (single-GPU lambda_max supplied); the distributed Lanczos gives
    the same lambda_max to 1e-13 on every partitioned level."""
    import torch
    from mlamg import problems
    from mlamg.hierarchy import Hierarchy
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    A = problems.poisson_3d_7pt(216)
    kw = dict(alpha=0.1, max_coarse=2000, aggregation="reference")
    H = Hierarchy.build(A, coarse_order="sorted", **kw)
    world = 8
    Ss = _setups(A, world, min_rows=50000, A0_global=A, lams=[L.lam for L in H.levels], **kw)
    K = len(Ss[0].parts)
    assert K == 3
    for r in (0, 3, 7):  # first, interior and last slab (the maps of all 8 cost ~2 s each)
        ref = _replicated_maps(H, K, world, r)
        for l, (d, e) in enumerate(zip(Ss[r].parts, ref)):
            tag = f"C4 world 8 rank {r} level {l}"
            for key in ("A_loc", "R_own", "P_loc"):
                _tcsr_equal(d[key], e[key], f"{tag}: {key}")
            for key in ("halo_x", "halo_r", "halo_p"):
                _halo_equal(d[key], e[key], f"{tag}: {key}")
            lo, hi = d["lo"], d["hi"]
            assert torch.equal(Ss[r].dinv[l].cpu(), H.levels[l].dinv[lo:hi].cpu()), tag
    del Ss
    torch.cuda.empty_cache()
    # the distributed Lanczos on the same operators, world 8
    from mlamg import dsetup

    def lam_fn(comm):
        S = dsetup.build_distributed(dsetup.split_rows(A, world, comm.rank), A.shape[0], comm,
                                     min_rows=50000, A0_global=A, **kw)
        return S.lams
    lams = dsetup.run_threads(world, lam_fn)
    for l in range(K):
        assert all(x[l] == lams[0][l] for x in lams)
        assert abs(lams[0][l] - H.levels[l].lam) <= 1e-13 * abs(H.levels[l].lam)
