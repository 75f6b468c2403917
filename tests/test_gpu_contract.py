"""GPU: the entry points under the boundary contract's names (csrc/contract.hip)
give the same results as the general API they wrap, called through ctypes exactly as a binding
written against the contract would."""
import ctypes

import numpy as np
import pytest
import scipy.sparse as sp

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ml():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mlamg.graph
    import mlamg.hierarchy
    import mlamg.problems
    import mlamg.sparse
    return mlamg


def test_mlamg_lloyd_matches_lloyd_cluster(ml):
    import torch
    from mlamg._lib import call, ptr, stream_ptr
    C = ml.problems.strength_invabs(ml.problems.poisson_2d_5pt(64))
    G = ml.sparse.DeviceCSR.from_scipy(C)
    seeds = np.sort(np.random.RandomState(0).permutation(C.shape[0])[:400]).astype(np.int32)
    s1 = torch.as_tensor(seeds).cuda()
    d, c1, s1, _ = ml.graph.lloyd_cluster_device(G, s1, maxiter=10)
    s2 = torch.as_tensor(seeds).cuda()
    c2 = torch.empty(C.shape[0], dtype=torch.int32, device="cuda")
    call("mlamg_lloyd", G.handle, ptr(s2), len(seeds), 10, ptr(c2), stream_ptr())
    assert torch.equal(c1, c2) and torch.equal(s1, s2)


def test_mlamg_vcycle_matches_hier_vcycle(ml):
    import torch
    from mlamg._lib import call, ptr, stream_ptr
    A = ml.problems.poisson_3d_7pt(24)
    H = ml.hierarchy.Hierarchy.build(A, alpha=0.1, max_coarse=100)
    n = A.shape[0]
    b = torch.as_tensor(np.random.RandomState(1).randn(n)).cuda()
    x0 = np.random.RandomState(2).randn(n)
    x1 = torch.as_tensor(x0).cuda()
    h1 = H.cycle(b, x1, 5)
    x2 = torch.as_tensor(x0).cuda()
    h2 = torch.zeros(5, dtype=torch.float64, device="cuda")
    call("mlamg_vcycle", H.handle, ptr(b), ptr(x2), 5, ptr(h2), stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(x1, x2)
    assert np.array_equal(h1, h2.cpu().numpy())


def test_comm_init_and_partitioned_operator(ml):
    import torch
    from mlamg import _lib
    from mlamg._lib import call, ptr, stream_ptr
    uid = ctypes.create_string_buffer(128)
    call("mlamg_comm_unique_id", uid)
    call("mlamg_comm_init", uid, 1, 0)
    try:
        assert _lib.lib.mlamg_comm_init(uid, 1, 0) == _lib.MLAMG_EINVAL  # one per process
        c = ctypes.c_void_p()
        call("mlamg_comm_default", ctypes.byref(c))
        assert c.value
        # single rank: no neighbours, no ghosts -> the operator is the plain matrix
        A = ml.problems.poisson_2d_5pt(32)
        ip = np.ascontiguousarray(A.indptr, np.int32)
        ij = np.ascontiguousarray(A.indices, np.int32)
        ax = np.ascontiguousarray(A.data, np.float64)
        h_csr, h_halo = ctypes.c_void_p(), ctypes.c_void_p()
        call("mlamg_csr_create_partitioned", A.shape[0], 0, A.nnz,
             ip.ctypes.data_as(ctypes.c_void_p), ij.ctypes.data_as(ctypes.c_void_p),
             ax.ctypes.data_as(ctypes.c_void_p), _lib.MLAMG_COPY_HOST, 0, None, None, None, None,
             ctypes.byref(h_csr), ctypes.byref(h_halo))
        x = torch.as_tensor(np.random.RandomState(3).randn(A.shape[0])).cuda()
        y = torch.empty_like(x)
        call("mlamg_halo_exchange", h_halo, ptr(x), stream_ptr())
        call("mlamg_spmv", h_csr, ptr(x), ptr(y), 1.0, 0.0, stream_ptr())
        assert np.array_equal(y.cpu().numpy(), A @ x.cpu().numpy())
        # ghost count must match the halo layout
        bad = ctypes.c_void_p(), ctypes.c_void_p()
        rc = _lib.lib.mlamg_csr_create_partitioned(
            A.shape[0], 5, A.nnz, ip.ctypes.data_as(ctypes.c_void_p),
            ij.ctypes.data_as(ctypes.c_void_p), ax.ctypes.data_as(ctypes.c_void_p),
            _lib.MLAMG_COPY_HOST, 0, None, None, None, None, ctypes.byref(bad[0]),
            ctypes.byref(bad[1]))
        assert rc == _lib.MLAMG_EINVAL
        _lib.lib.mlamg_halo_destroy(h_halo)
        _lib.lib.mlamg_csr_destroy(h_csr)
    finally:
        call("mlamg_comm_finalize")
    c = ctypes.c_void_p()
    assert _lib.lib.mlamg_comm_default(ctypes.byref(c)) == _lib.MLAMG_EINVAL


def test_dispatch_packet_timer(ml):
    """mlamg_timer_* (bench.py's roofline timing): an armed timer is consumed by the next
    SpMV-family launch, which still computes scipy's bits; elapsed_ms returns that kernel's time
    (positive, below the host-measured wall time of the call); reading a timer that no launch
    consumed is an error, and a timer armed then destroyed leaves later launches untimed."""
    import time

    import torch
    from mlamg._lib import MlamgError, call, ptr, stream_ptr
    A = ml.problems.poisson_3d_7pt(64)
    n = A.shape[0]
    x = np.random.RandomState(3).randn(n)
    Ad = ml.sparse.DeviceCSR.from_scipy(A).set_format("rowpat")
    xd = torch.as_tensor(x).cuda()
    yd = torch.empty_like(xd)
    tm = ctypes.c_void_p()
    call("mlamg_timer_create", ctypes.byref(tm))
    ms = ctypes.c_float()
    with pytest.raises(MlamgError):
        call("mlamg_timer_elapsed_ms", tm, ctypes.byref(ms))  # never armed
    torch.cuda.synchronize()
    for _ in range(3):
        t0 = time.perf_counter()
        call("mlamg_timer_arm", tm)
        call("mlamg_spmv", Ad.handle, ptr(xd), ptr(yd), 1.0, 0.0, stream_ptr())
        call("mlamg_timer_elapsed_ms", tm, ctypes.byref(ms))
        wall_ms = (time.perf_counter() - t0) * 1e3
        assert 0.0 < ms.value < wall_ms
        assert np.array_equal(yd.cpu().numpy(), A @ x)
    # disarm drops a timer no launch took
    call("mlamg_timer_arm", tm)
    call("mlamg_timer_disarm")
    call("mlamg_spmv", Ad.handle, ptr(xd), ptr(yd), 1.0, 0.0, stream_ptr())
    with pytest.raises(MlamgError):
        call("mlamg_timer_elapsed_ms", tm, ctypes.byref(ms))
    # a launch recorded into a stream capture never takes the timer
    g = torch.cuda.CUDAGraph()
    yd.zero_()
    torch.cuda.synchronize()
    call("mlamg_timer_arm", tm)
    with torch.cuda.graph(g):
        call("mlamg_spmv", Ad.handle, ptr(xd), ptr(yd), 1.0, 0.0, stream_ptr())
    with pytest.raises(MlamgError):
        call("mlamg_timer_elapsed_ms", tm, ctypes.byref(ms))
    call("mlamg_timer_disarm")
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(yd.cpu().numpy(), A @ x)
    call("mlamg_timer_arm", tm)
    call("mlamg_timer_destroy", tm)  # disarms: the next launch must not touch the freed events
    call("mlamg_spmv", Ad.handle, ptr(xd), ptr(yd), 1.0, 0.0, stream_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(yd.cpu().numpy(), A @ x)
