"""ctypes binding of libmlamg_hip.so (C-ABI declared in include/mlamg.h).

torch is imported first on purpose: torch ships its own libamdhip64.so.7, and loading it before
this library makes both share one HIP runtime (the .so resolves libamdhip64.so.7 by soname), so
device pointers and streams from torch are valid here.

There is no CPU fallback: if the library is missing, importing this module raises.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch  # noqa: F401  (must be loaded before the HIP library, see module doc)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MLAMG_LIB", os.path.join(_HERE, "libmlamg_hip.so"))

MLAMG_OK = 0
MLAMG_EINVAL = -1
MLAMG_EHIP = -2
MLAMG_ENCCL = -3
MLAMG_ENOMEM = -4
MLAMG_EUNSUPPORTED = -5

MLAMG_COPY_HOST = 0
MLAMG_COPY_DEVICE = 1
MLAMG_WRAP_DEVICE = 2

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"libmlamg_hip.so not found at {LIB_PATH}; build it with "
        "`python ml-amg_amd/build_native.py` (or __graft_entry__.build()). "
        "The MI355X path has no CPU fallback."
    )

lib = ctypes.CDLL(LIB_PATH)

c_i32 = ctypes.c_int32
c_i64 = ctypes.c_int64
c_u64 = ctypes.c_uint64
c_int = ctypes.c_int
c_dbl = ctypes.c_double
c_vp = ctypes.c_void_p
c_vpp = ctypes.POINTER(ctypes.c_void_p)
P_i32 = ctypes.POINTER(ctypes.c_int32)
P_i64 = ctypes.POINTER(ctypes.c_int64)
P_dbl = ctypes.POINTER(ctypes.c_double)
P_int = ctypes.POINTER(ctypes.c_int)

class Amg2vProblem(ctypes.Structure):
    """mlamg_amg2v_problem (include/mlamg.h)."""
    _fields_ = [("n", ctypes.c_int64), ("n_c", ctypes.c_int64),
                ("A_indptr", ctypes.c_void_p), ("A_indices", ctypes.c_void_p),
                ("A_data", ctypes.c_void_p), ("A_nnz", ctypes.c_int64),
                ("P_indptr", ctypes.c_void_p), ("P_indices", ctypes.c_void_p),
                ("P_data", ctypes.c_void_p), ("P_nnz", ctypes.c_int64),
                ("b", ctypes.c_void_p), ("x0", ctypes.c_void_p),
                ("x_out", ctypes.c_void_p), ("err_out", ctypes.c_void_p),
                ("iters_out", ctypes.c_int32), ("status_out", ctypes.c_int32)]


# the same record as a numpy dtype: a batch's problem list is filled column-wise
AMG2V_DTYPE = np.dtype([(name, {ctypes.c_int64: "<i8", ctypes.c_void_p: "<u8",
                                ctypes.c_int32: "<i4"}[t]) for name, t in Amg2vProblem._fields_])
assert AMG2V_DTYPE.itemsize == ctypes.sizeof(Amg2vProblem)


# name -> (restype, argtypes); every symbol of include/mlamg.h
SIGNATURES = {
    "mlamg_version": (c_int, []),
    "mlamg_last_error": (ctypes.c_char_p, []),
    "mlamg_set_device": (c_int, [c_int]),
    "mlamg_get_device": (c_int, [P_int]),
    "mlamg_stream_sync": (c_int, [c_vp]),
    "mlamg_timer_create": (c_int, [c_vpp]),
    "mlamg_timer_destroy": (c_int, [c_vp]),
    "mlamg_timer_arm": (c_int, [c_vp]),
    "mlamg_timer_disarm": (c_int, []),
    "mlamg_timer_elapsed_ms": (c_int, [c_vp, ctypes.POINTER(ctypes.c_float)]),
    "mlamg_csr_create": (c_int, [c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_int, c_vpp]),
    "mlamg_csr_destroy": (c_int, [c_vp]),
    "mlamg_csr_shape": (c_int, [c_vp, P_i64, P_i64, P_i64]),
    "mlamg_csr_device_arrays": (c_int, [c_vp, c_vpp, c_vpp, c_vpp]),
    "mlamg_csr_fingerprint": (c_int, [c_vp, ctypes.POINTER(ctypes.c_uint64), c_vp]),
    "mlamg_csr_download": (c_int, [c_vp, c_vp, c_vp, c_vp]),
    "mlamg_csr_copy_device": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mlamg_csr_set_format": (c_int, [c_vp, c_int, c_int, c_vp]),
    "mlamg_csr_get_format": (c_int, [c_vp, P_int, P_int, P_i64]),
    "mlamg_csr_format_bytes": (c_int, [c_vp, P_dbl]),
    "mlamg_csr_attach_dinv": (c_int, [c_vp, c_vp, c_vp]),
    "mlamg_lsqr": (c_int, [c_vp, c_vp, c_vp, c_vp, c_dbl, c_dbl, c_dbl, c_int, P_int, P_int,
                           c_vp]),
    "mlamg_remove_mean": (c_int, [c_vp, c_i64, c_vp]),
    "mlamg_spmv": (c_int, [c_vp, c_vp, c_vp, c_dbl, c_dbl, c_vp]),
    "mlamg_residual": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mlamg_jacobi": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp]),
    "mlamg_jacobi_explicit": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp]),
    "mlamg_restrict": (c_int, [c_vp, c_vp, c_vp, c_vp]),
    "mlamg_prolong_add": (c_int, [c_vp, c_vp, c_vp, c_vp]),
    "mlamg_diag_inv": (c_int, [c_vp, c_dbl, c_vp, c_vp]),
    "mlamg_norm2": (c_int, [c_vp, c_i64, c_vp, c_vp]),
    "mlamg_transpose": (c_int, [c_vp, c_vpp, c_vp]),
    "mlamg_spgemm": (c_int, [c_vp, c_vp, c_vpp, c_vp]),
    "mlamg_galerkin": (c_int, [c_vp, c_vp, c_vp, c_vpp, c_vp]),
    "mlamg_scratch_trim": (c_int, [ctypes.POINTER(ctypes.c_size_t)]),
    "mlamg_device_cache_trim": (c_int, [ctypes.POINTER(ctypes.c_size_t)]),
    "mlamg_device_cache_stats": (c_int, [ctypes.POINTER(ctypes.c_size_t),
                                         ctypes.POINTER(ctypes.c_int64),
                                         ctypes.POINTER(ctypes.c_int64)]),
    "mlamg_setup_phase_times": (c_int, [P_dbl, c_int, c_int]),
    "mlamg_sa_smoother": (c_int, [c_vp, c_dbl, c_vpp, c_vp]),
    "mlamg_csr_scale_rows": (c_int, [c_vp, c_vp, c_int, c_vpp, c_vp]),
    "mlamg_lambda_max_dinvA": (c_int, [c_vp, c_int, c_dbl, c_u64, P_dbl, P_int, c_vp]),
    "mlamg_strength": (c_int, [c_vp, c_int, c_vpp, c_vp]),
    "mlamg_evolution_strength": (c_int, [c_vp, c_dbl, c_dbl, c_int, c_vpp, c_vp]),
    "mlamg_gnn_linear": (c_int, [c_vp, c_i64, c_int, c_vp, c_vp, c_int, c_int, ctypes.c_float,
                                 c_vp, c_int, c_vp, c_vp]),
    "mlamg_gnn_gcn_norm": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp,
                                   c_vp]),
    "mlamg_gnn_propagate": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_vp, c_vp]),
    "mlamg_gnn_instance_norm": (c_int, [c_vp, c_i64, c_int, ctypes.c_float, c_vp, c_vp]),
    "mlamg_gnn_nnconv": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_vp, c_vp, c_vp, c_vp,
                                 c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_vp, c_vp, c_int,
                                 c_vp, c_int, c_vp, c_vp, c_vp]),
    "mlamg_gnn_edge_mlp": (c_int, [c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_i64, c_vp, c_vp,
                                   c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_vp, c_int,
                                   c_vp, c_vp]),
    "mlamg_gnn_topk": (c_int, [c_vp, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "mlamg_bellman_ford": (c_int, [c_vp, c_vp, c_i32, c_vp, c_vp, P_i32, c_vp]),
    "mlamg_bellman_ford_canon": (c_int, [c_vp, c_vp, c_i32, c_vp, c_vp, P_i32, c_vp]),
    "mlamg_bellman_ford_pyamg": (c_int, [c_vp, c_vp, c_i32, c_int, c_vp, c_vp, P_i32, c_vp]),
    "mlamg_bf_canon_begin": (c_int, [c_vp, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mlamg_bf_canon_sweep": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mlamg_bf_canon_label": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mlamg_bf_canon_end": (c_int, [c_vp, c_i64, c_vp]),
    "mlamg_aggregate_op": (c_int, [c_vp, c_i64, c_i64, c_vpp, c_vp]),
    "mlamg_labels_to_columns": (c_int, [c_vp, c_i64, c_vp, c_i32, c_vp, c_vp]),
    "mlamg_lloyd_cluster": (c_int, [c_vp, c_vp, c_i32, c_int, c_vp, c_vp, P_i32, c_vp]),
    "mlamg_lloyd_cluster_canon": (c_int, [c_vp, c_vp, c_i32, c_int, c_vp, c_vp, P_i32, c_vp]),
    "mlamg_gs_create": (c_int, [c_vp, c_vpp, c_vp]),
    "mlamg_gs_create_ex": (c_int, [c_vp, c_int, c_int, c_vpp, c_vp]),
    "mlamg_legacy_permutation": (c_int, [ctypes.c_uint32, c_i64, c_i64, c_vp, c_vp]),
    "mlamg_gmres_householder": (c_int, [c_vp, c_vp, c_vp, c_vp, c_dbl, c_int, c_int, P_int,
                                        P_int, c_vp, c_int, c_vp]),
    "mlamg_symmetric_strength": (c_int, [c_vp, c_dbl, c_vpp, c_vp]),
    "mlamg_standard_aggregation": (c_int, [c_vp, c_vp, c_vp, P_i64, P_i32, c_vp]),
    "mlamg_fit_candidates": (c_int, [c_vp, c_vp, c_dbl, c_vpp, c_vp, c_vp]),
    "mlamg_csr_sub": (c_int, [c_vp, c_vp, c_vpp, c_vp]),
    "mlamg_diag_pinv": (c_int, [c_vp, c_vp, c_vp]),
    "mlamg_dense_create_matrix": (c_int, [c_vp, c_i64, c_vpp, c_vp]),
    "mlamg_gs_destroy": (c_int, [c_vp]),
    "mlamg_gs_levels": (c_int, [c_vp, P_i32]),
    "mlamg_gs_sweep": (c_int, [c_vp, c_vp, c_vp, c_int, c_vp]),
    "mlamg_dense_create": (c_int, [c_vp, c_vpp, c_vp]),
    "mlamg_dense_info": (c_int, [c_vp, P_int, P_i64]),
    "mlamg_dense_destroy": (c_int, [c_vp]),
    "mlamg_dense_solve": (c_int, [c_vp, c_vp, c_vp, c_vp]),
    "mlamg_hier_create": (c_int, [c_vpp]),
    "mlamg_hier_destroy": (c_int, [c_vp]),
    "mlamg_hier_add_level": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mlamg_hier_set_coarse": (c_int, [c_vp, c_vp, c_vp]),
    "mlamg_amg2v_batch": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_dbl, c_int, c_dbl, c_int,
                                  c_vp]),
    "mlamg_amg2v_batch_limits": (c_int, [P_i64, P_i64, P_int]),
    "mlamg_hier_set_coarse_pcg": (c_int, [c_vp, c_vp, c_vp]),
    "mlamg_hier_set_coarse_gmres": (c_int, [c_vp, c_vp, c_vp, c_dbl, c_dbl, c_int, c_int]),
    "mlamg_hier_coarse_gmres_stats": (c_int, [c_vp, P_i32, P_i32, P_i32, P_i32, P_dbl]),
    "mlamg_pcg_create": (c_int, [c_vp, c_vp, c_dbl, c_int, c_vpp]),
    "mlamg_pcg_destroy": (c_int, [c_vp]),
    "mlamg_pcg_solve": (c_int, [c_vp, c_vp, c_vp, c_vp]),
    "mlamg_pcg_stats": (c_int, [c_vp, P_i32, P_i32, P_i32, P_dbl, c_vp]),
    "mlamg_pcg_breakdowns": (c_int, [c_vp, P_i32, c_vp]),
    "mlamg_gmres": (c_int, [c_vp, c_vp, c_vp, c_vp, c_dbl, c_int, c_int, c_int, P_int, P_int,
                            c_vp, c_int, c_vp]),
    "mlamg_csr_symmetric": (c_int, [c_vp, c_dbl, P_int, c_vp]),
    "mlamg_hier_set_smoothing": (c_int, [c_vp, c_int, c_int]),
    "mlamg_hier_set_done_check": (c_int, [c_vp, c_int]),
    "mlamg_hier_set_factored_prolong": (c_int, [c_vp, c_int, c_vp, c_vp, c_vp]),
    "mlamg_hier_set_level_smoother": (c_int, [c_vp, c_int, c_vp]),
    "mlamg_hier_set_norm": (c_int, [c_vp, c_int]),
    "mlamg_hier_vcycle": (c_int, [c_vp, c_vp, c_vp, c_int, c_dbl, c_vp, P_i32, c_int, c_vp]),
    "mlamg_hier_cycle_bytes": (c_int, [c_vp, P_dbl]),
    "mlamg_hier_cycle_format_bytes": (c_int, [c_vp, P_dbl]),
    "mlamg_comm_unique_id": (c_int, [c_vp]),
    "mlamg_comm_create": (c_int, [c_vp, c_int, c_int, c_vpp]),
    "mlamg_comm_destroy": (c_int, [c_vp]),
    "mlamg_comm_info": (c_int, [c_vp, P_int, P_int, P_int, P_int]),
    "mlamg_loop_group_create": (c_int, [c_int, c_vpp]),
    "mlamg_loop_group_destroy": (c_int, [c_vp]),
    "mlamg_comm_create_loopback": (c_int, [c_vp, c_int, c_vpp]),
    "mlamg_comm_create_null": (c_int, [c_int, c_int, c_vpp]),
    "mlamg_comm_allreduce_sum": (c_int, [c_vp, c_vp, c_i64, c_vp]),
    "mlamg_halo_create": (c_int, [c_vp, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_vpp]),
    "mlamg_halo_destroy": (c_int, [c_vp]),
    "mlamg_halo_exchange": (c_int, [c_vp, c_vp, c_vp]),
    "mlamg_dhier_create": (c_int, [c_vp, c_vp, c_i64, c_vp, c_vp, c_vpp]),
    "mlamg_dhier_add_level": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mlamg_dhier_destroy": (c_int, [c_vp]),
    "mlamg_dhier_set_coarse_graph": (c_int, [c_vp, c_int]),
    "mlamg_dhier_set_cycle_graph": (c_int, [c_vp, c_int]),
    "mlamg_dhier_set_split": (c_int, [c_vp, c_int, c_int, c_vp, c_vp, c_vp]),
    "mlamg_dhier_set_overlap": (c_int, [c_vp, c_int]),
    "mlamg_dhier_vcycle": (c_int, [c_vp, c_vp, c_vp, c_int, c_dbl, c_vp, P_i32, c_vp]),
    # boundary-contract spellings (csrc/contract.hip)
    "mlamg_lloyd": (c_int, [c_vp, c_vp, c_i32, c_int, c_vp, c_vp]),
    "mlamg_vcycle": (c_int, [c_vp, c_vp, c_vp, c_int, c_vp, c_vp]),
    "mlamg_comm_init": (c_int, [c_vp, c_int, c_int]),
    "mlamg_comm_default": (c_int, [c_vpp]),
    "mlamg_comm_finalize": (c_int, []),
    "mlamg_csr_create_partitioned": (c_int, [c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_int, c_i32,
                                             c_vp, c_vp, c_vp, c_vp, c_vpp, c_vpp]),
}

for _name, (_res, _args) in SIGNATURES.items():
    _f = getattr(lib, _name)
    _f.restype = _res
    _f.argtypes = _args


class MlamgError(RuntimeError):
    def __init__(self, code, where):
        msg = lib.mlamg_last_error()
        msg = msg.decode() if msg else ""
        super().__init__(f"{where} failed ({code}): {msg}")
        self.code = code


def check(rc, where=""):
    if rc != MLAMG_OK:
        raise MlamgError(rc, where)
    return rc


def call(name, *args):
    """Call a C-ABI entry point and raise MlamgError on a nonzero status."""
    return check(getattr(lib, name)(*args), name)


def stream_ptr(stream=None):
    """hipStream_t of the given (or current) torch stream."""
    if stream is None:
        stream = torch.cuda.current_stream()
    return ctypes.c_void_p(stream.cuda_stream)


def _tol_arg(tol):
    """Tolerance argument of the cycle entry points: None = no tolerance (-1.0: the C side arms
    its stop flag only for tol >= 0, so a requested tol = 0 stops on an exactly zero norm like
    the reference's `e <= tol`, ns/lib/multigrid.py:197)."""
    return -1.0 if tol is None else float(tol)


def ptr(t):
    """Device pointer of a torch tensor (None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())
