"""Mirror of ns/lib/sparse_tensor.py without torch_sparse (absent here; every caller imports the
module at top level: utils/common.py:15, utils/train_dataset.py:23, utils/evaluate_model.py:21,
utils/evaluate_dataset.py:38).

  to_scipy   :54-59  torch COO -> scipy CSR (what the callers use: evaluate_dataset.py:74,
                     evaluate_model.py:167, train_dataset.py:99)
  spspmm     :9-20   sparse @ sparse -> coalesced COO      (torch.sparse.mm here)
  spmm       :22-29  sparse @ dense                        (torch.sparse.mm here)
  spT        :31-38  transpose, coalesced
  diag       :40-52  diagonal as a float32 vector (ones where no entry is stored)

Only to_scipy is on the V-cycle path's boundary; the other four serve the reference's torch
training loss (ns/model/loss.py), out of scope, and run on torch's own sparse kernels — results
match torch_sparse's up to the summation order of its SpGEMM (parity unpinned: torch_sparse
absent).
"""
from __future__ import annotations

import torch

from .sparse import to_scipy  # noqa: F401


def spspmm(A, B):
    assert A.shape[1] == B.shape[0]
    return torch.sparse.mm(A.coalesce(), B.coalesce()).coalesce()


def spmm(A, B):
    assert A.shape[1] == B.shape[0]
    return torch.sparse.mm(A.coalesce(), B)


def spT(A):
    return A.coalesce().t().coalesce()


def diag(A):
    n = min(A.shape[0], A.shape[1])
    d = torch.ones(n)
    A = A.coalesce()
    idx, val = A.indices(), A.values()
    on = idx[0] == idx[1]
    d[idx[0][on].cpu()] = val[on].detach().cpu().to(d.dtype)
    return d
