"""Device CSR handles and the scipy/torch conversions of ns/lib/sparse.py.

Reference: ns/lib/sparse.py:20-32 (to_torch_sparse: scipy -> torch COO with fp32 values),
ns/lib/sparse.py:8,35,51,78 (col_normalize_csr, get_diagonal, triu, tril: the reference's own
scipy / torch COO helpers, kept as they are so that aliasing ns.lib.sparse to this module
leaves its callers — ns/model/data.py:127, demos/1d_poisson.py:106 — working),
ns/lib/sparse.py:105-106 (scipy_to_torch / torch_to_scipy aliases), ns/lib/sparse_tensor.py:54-59
(to_scipy: torch COO -> scipy CSR). The V-cycle itself never goes through torch COO: matrices are
uploaded once as int32/fp64 CSR into a `DeviceCSR` (C handle `mlamg_csr`, include/mlamg.h).
"""
from __future__ import annotations

import ctypes

import numpy as np
import scipy.sparse as sp
import torch

from . import _lib
from ._lib import call, ptr, stream_ptr


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("mlamg: no HIP device visible (the MI355X path has no CPU fallback)")
    return torch.device("cuda", torch.cuda.current_device())


def canonical_rows(A):
    """Return a CSR whose rows have no duplicate columns.

    The kernels sum rows in their STORED order, exactly like scipy, so unsorted rows are kept
    as they are. Rows with duplicate column indices (never produced by the reference's
    generators) are merged with scipy's sum_duplicates on a copy, which also sorts them.
    """
    A = A.tocsr() if not sp.isspmatrix_csr(A) else A
    if A.has_canonical_format:
        return A
    B = A.copy()
    B.has_sorted_indices = False
    B.sort_indices()
    if B.nnz and B.nnz == A.nnz:
        rows = np.repeat(np.arange(B.shape[0]), np.diff(B.indptr))
        dup = (rows[1:] == rows[:-1]) & (B.indices[1:] == B.indices[:-1])
        if not dup.any():
            return A
    C = A.copy()
    C.sum_duplicates()
    return C


_INT32_MAX = 2**31 - 1


def _check_int32(shape, nnz):
    """The device handle stores int32 indptr/indices (scipy's type at these sizes): refuse an
    operator whose nonzero count or dimensions would wrap instead of uploading a corrupted one."""
    if nnz > _INT32_MAX or shape[0] >= _INT32_MAX or shape[1] > _INT32_MAX:
        raise ValueError(f"matrix of shape {tuple(shape)} with {nnz} nonzeros exceeds the int32 "
                         "index range of the device CSR handle")


class DeviceCSR:
    """An int32/fp64 CSR matrix resident on the GPU (owns a `mlamg_csr*`)."""

    __slots__ = ("handle", "shape", "nnz", "_keep", "_dinv_ref", "__weakref__")

    def __init__(self, handle, keep=()):
        self.handle = handle
        nr, nc, nz = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        call("mlamg_csr_shape", handle, ctypes.byref(nr), ctypes.byref(nc), ctypes.byref(nz))
        self.shape = (int(nr.value), int(nc.value))
        self.nnz = int(nz.value)
        self._keep = keep
        self._dinv_ref = None

    # ------------------------------------------------------------------ construction
    @classmethod
    def from_scipy(cls, A, check=True):
        A = sp.csr_matrix(A) if not sp.issparse(A) else A
        A = A.tocsr()
        if check:
            A = canonical_rows(A)
        _device()
        _check_int32(A.shape, A.nnz)
        indptr = np.ascontiguousarray(A.indptr, dtype=np.int32)
        indices = np.ascontiguousarray(A.indices, dtype=np.int32)
        data = np.ascontiguousarray(A.data, dtype=np.float64)
        h = ctypes.c_void_p()
        call("mlamg_csr_create", A.shape[0], A.shape[1], A.nnz,
             indptr.ctypes.data_as(ctypes.c_void_p), indices.ctypes.data_as(ctypes.c_void_p),
             data.ctypes.data_as(ctypes.c_void_p), _lib.MLAMG_COPY_HOST, ctypes.byref(h))
        return cls(h)

    @classmethod
    def from_torch(cls, crow, col, val, shape, wrap=False):
        """From device tensors (int32 crow/col, float64 val); wrap=True keeps them alive."""
        for t, dt in ((crow, torch.int32), (col, torch.int32), (val, torch.float64)):
            if t.dtype != dt or not t.is_cuda or not t.is_contiguous():
                raise TypeError("from_torch needs contiguous cuda int32/int32/float64 tensors")
        _check_int32(shape, val.numel())
        h = ctypes.c_void_p()
        where = _lib.MLAMG_WRAP_DEVICE if wrap else _lib.MLAMG_COPY_DEVICE
        call("mlamg_csr_create", shape[0], shape[1], val.numel(), ptr(crow), ptr(col), ptr(val),
             where, ctypes.byref(h))
        return cls(h, keep=(crow, col, val) if wrap else ())

    @classmethod
    def _adopt(cls, handle):
        return cls(handle)

    # ------------------------------------------------------------------ export
    def to_torch(self):
        """Device copies (crow int32, col int32, val float64) as torch tensors."""
        n = self.shape[0]
        dev = _device()
        crow = torch.empty(n + 1, dtype=torch.int32, device=dev)
        col = torch.empty(max(self.nnz, 1), dtype=torch.int32, device=dev)
        val = torch.empty(max(self.nnz, 1), dtype=torch.float64, device=dev)
        call("mlamg_csr_copy_device", self.handle, ptr(crow), ptr(col), ptr(val), stream_ptr())
        return crow, col[:self.nnz], val[:self.nnz]

    def to_scipy(self):
        n, m = self.shape
        indptr = np.empty(n + 1, dtype=np.int32)
        indices = np.empty(self.nnz, dtype=np.int32)
        data = np.empty(self.nnz, dtype=np.float64)
        call("mlamg_csr_download", self.handle, indptr.ctypes.data_as(ctypes.c_void_p),
             indices.ctypes.data_as(ctypes.c_void_p), data.ctypes.data_as(ctypes.c_void_p))
        return sp.csr_matrix((data, indices, indptr), shape=(n, m))

    def arrays(self):
        """Raw device pointers (indptr, indices, data)."""
        a, b, c = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        call("mlamg_csr_device_arrays", self.handle, ctypes.byref(a), ctypes.byref(b),
             ctypes.byref(c))
        return a.value, b.value, c.value

    # ------------------------------------------------------------------ ops
    def matvec(self, x, out=None, alpha=1.0, beta=0.0):
        if out is None:
            out = torch.zeros(self.shape[0], dtype=torch.float64, device=x.device)
        call("mlamg_spmv", self.handle, ptr(x), ptr(out), alpha, beta, stream_ptr())
        return out

    def transpose(self):
        h = ctypes.c_void_p()
        call("mlamg_transpose", self.handle, ctypes.byref(h), stream_ptr())
        return DeviceCSR(h)

    @property
    def T(self):
        return self.transpose()

    def __matmul__(self, other):
        if isinstance(other, DeviceCSR):
            h = ctypes.c_void_p()
            call("mlamg_spgemm", self.handle, other.handle, ctypes.byref(h), stream_ptr())
            return DeviceCSR(h)
        if isinstance(other, torch.Tensor):
            return self.matvec(other)
        return NotImplemented

    FORMATS = {"csr_stream": 0, "sell": 1, "vector": 2, "auto_exact": 3, "sorted": 4,
               "sell_dict": 5, "rowpat": 6, "long": 7}

    def set_format(self, fmt, vec_width=0):
        """SpMV kernel/storage: 'csr_stream' | 'sell' | 'sell_dict' | 'sorted' | 'rowpat' |
        'long' | 'auto_exact' (all scipy's order) or 'vector' (lane-strided order, see
        include/mlamg.h)."""
        call("mlamg_csr_set_format", self.handle, self.FORMATS[fmt], int(vec_width), stream_ptr())
        return self

    def get_format(self):
        f, vw, st = ctypes.c_int(), ctypes.c_int(), ctypes.c_int64()
        call("mlamg_csr_get_format", self.handle, ctypes.byref(f), ctypes.byref(vw),
             ctypes.byref(st))
        name = {v: k for k, v in self.FORMATS.items()}[f.value]
        return name, int(vw.value), int(st.value)

    def fingerprint(self):
        """64-bit fingerprint of the rows, columns and value bits (mlamg_csr_fingerprint)."""
        v = ctypes.c_uint64()
        call("mlamg_csr_fingerprint", self.handle, ctypes.byref(v), stream_ptr())
        return int(v.value)

    def format_bytes(self):
        """Algorithmic HBM bytes of one y = A@x in the active storage format."""
        b = ctypes.c_double()
        call("mlamg_csr_format_bytes", self.handle, ctypes.byref(b))
        return float(b.value)

    def attach_dinv(self, dinv):
        """Attach Jacobi weights to a 'rowpat' operator (include/mlamg.h mlamg_csr_attach_dinv):
        epilogues given this very tensor read its per-pattern values from the pattern table.
        Returns False (nothing attached) when A is not rowpat or dinv is not pattern-constant."""
        try:
            call("mlamg_csr_attach_dinv", self.handle, ptr(dinv) if dinv is not None else None,
                 stream_ptr())
        except _lib.MlamgError as e:
            if e.code != _lib.MLAMG_EUNSUPPORTED:
                raise
            self._dinv_ref = None
            return False
        self._dinv_ref = dinv  # keeps the attached vector alive
        return dinv is not None

    def diag_inv(self, omega=1.0):
        d = torch.empty(self.shape[0], dtype=torch.float64, device=_device())
        call("mlamg_diag_inv", self.handle, omega, ptr(d), stream_ptr())
        return d

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            try:
                _lib.lib.mlamg_csr_destroy(h)
            except Exception:  # interpreter shutdown
                pass
            self.handle = None

    def __repr__(self):
        return f"DeviceCSR(shape={self.shape}, nnz={self.nnz})"


def as_device(A):
    return A if isinstance(A, DeviceCSR) else DeviceCSR.from_scipy(A)


def galerkin(R, A, P):
    """A_c = (R@A)@P on the device (ns/lib/multigrid.py:165 `P.T@A@P`)."""
    h = ctypes.c_void_p()
    call("mlamg_galerkin", R.handle, A.handle, P.handle, ctypes.byref(h), stream_ptr())
    return DeviceCSR(h)


def to_device_vec(x, dtype=torch.float64):
    if isinstance(x, torch.Tensor):
        return x.to(device=_device(), dtype=dtype).contiguous()
    return torch.as_tensor(np.ascontiguousarray(x), dtype=dtype).to(_device())


# ---------------------------------------------------------------------- ns/lib/sparse.py mirror
def to_torch_sparse(A):
    """scipy -> torch COO with fp32 values, coalesced (ns/lib/sparse.py:20-32)."""
    A = A.tocoo()
    T = torch.sparse_coo_tensor(
        torch.as_tensor(np.vstack([A.row, A.col]).astype(np.int64)),
        torch.as_tensor(A.data.astype(np.float32)),
        A.shape,
    )
    return T.coalesce()


def to_scipy(T):
    """torch COO -> scipy CSR (ns/lib/sparse_tensor.py:54-59)."""
    T = T.coalesce() if not T.is_coalesced() else T
    idx = T.indices().cpu().numpy()
    return sp.coo_matrix((T.values().cpu().numpy(), (idx[0], idx[1])), shape=tuple(T.shape)).tocsr()


def col_normalize_csr(A_sp, ord=1):
    """ns/lib/sparse.py:8-17: divide every nonzero by its column's `ord`-norm (scipy CSR)."""
    import scipy.sparse.linalg as spla
    if not sp.isspmatrix_csr(A_sp):
        A_sp = A_sp.tocsr()
    norms = spla.norm(A_sp, axis=0, ord=ord)
    return sp.csr_matrix((A_sp.data / norms[A_sp.indices], A_sp.indices, A_sp.indptr), A_sp.shape)


def get_diagonal(A_T, as_vector=True):
    """ns/lib/sparse.py:35-48: diagonal entries of a torch sparse COO tensor (the stored ones, in
    storage order), as a vector or as a sparse COO tensor. Runs where A_T lives."""
    values = A_T.values()
    indices = A_T.indices()
    diag_entries = indices[0] == indices[1]
    if as_vector:
        return values[diag_entries]
    return torch.sparse_coo_tensor(indices[:, diag_entries], values[diag_entries],
                                   size=A_T.shape)


def triu(A_T, diag=0):
    """ns/lib/sparse.py:51-75: entries with col - row >= diag of a torch sparse COO tensor."""
    values = A_T.values()
    indices = A_T.indices()
    keep = (indices[1] - indices[0]) >= diag
    return torch.sparse_coo_tensor(indices[:, keep], values[keep], size=A_T.shape)


def tril(A_T, diag=0):
    """ns/lib/sparse.py:78-102: entries with row - col >= diag of a torch sparse COO tensor."""
    values = A_T.values()
    indices = A_T.indices()
    keep = (indices[0] - indices[1]) >= diag
    return torch.sparse_coo_tensor(indices[:, keep], values[keep], size=A_T.shape)


scipy_to_torch = to_torch_sparse
torch_to_scipy = to_scipy
