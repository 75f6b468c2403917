// Setup kernels of pyamg.aggregation.smoothed_aggregation_solver with its default recipe, the
// multilevel solver the reference's PyAMG preconditioner builds (ns/preconditioner/PyAMG.py:94):
//   C = symmetric_strength_of_connection(A, theta=0)        pyamg/strength.py, amg_core
//   AggOp = standard_aggregation(C)                          pyamg/aggregation/aggregate.py
//   T, B_c = fit_candidates(AggOp, B)                        pyamg/aggregation/tentative.py
//   P = T - (omega / rho(D^-1 A)) D^-1 A T                   jacobi_prolongation_smoother
// (the symmetric block Gauss-Seidel candidate improvement and smoother: csrc/gs.hip; the products
// and the Galerkin operator: csrc/spgemm.hip). pyamg is absent here: the kernels restate its
// published algorithm (amg_core C++), parity unpinned; they are bitwise the oracle's
// restatement (oracle/oracle.c pyamg_*, oracle/restated.py pyamg_sa_*).
#include "common.hpp"

#include <algorithm>
#include <vector>

namespace mlamg {

static inline dim3 gsa(int64_t n) {
  return dim3((unsigned)std::max<int64_t>(1, (n + 255) / 256));
}

// ---------------------------------------------------------------- symmetric strength
// amg_core symmetric_strength_of_connection: diags[i] = |sum of row i's diagonal entries|; row i
// keeps its diagonal and every a_ij with a_ij^2 >= (theta^2 diags[i]) diags[j], in stored order;
// then pyamg takes |s_ij| and scales each row by 1 / (its largest entry) (scale_rows_by_largest_
// entry; a row whose largest entry is 0 is multiplied by 0).
__global__ void k_ss_diag(const int32_t* __restrict__ ip, const int32_t* __restrict__ ij,
                          const double* __restrict__ ax, int64_t n, double* __restrict__ dg) {
  const int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  double d = 0.0;
  for (int k = ip[i]; k < ip[i + 1]; ++k)
    if (ij[k] == (int32_t)i) d += ax[k];
  dg[i] = fabs(d);
}

__device__ __forceinline__ bool ss_keep(int64_t i, int32_t j, double a, double eps_i,
                                        const double* __restrict__ dg) {
  return j == (int32_t)i || a * a >= eps_i * dg[j];
}

__global__ void k_ss_count(const int32_t* __restrict__ ip, const int32_t* __restrict__ ij,
                           const double* __restrict__ ax, int64_t n, double theta,
                           const double* __restrict__ dg, int32_t* __restrict__ cnt) {
  const int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  const double eps_i = theta * theta * dg[i];
  int32_t c = 0;
  for (int k = ip[i]; k < ip[i + 1]; ++k) c += ss_keep(i, ij[k], ax[k], eps_i, dg);
  cnt[i] = c;
}

__global__ void k_ss_fill(const int32_t* __restrict__ ip, const int32_t* __restrict__ ij,
                          const double* __restrict__ ax, int64_t n, double theta,
                          const double* __restrict__ dg, const int32_t* __restrict__ sp,
                          int32_t* __restrict__ sj, double* __restrict__ sx) {
  const int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  const double eps_i = theta * theta * dg[i];
  double mx = 0.0;
  for (int k = ip[i]; k < ip[i + 1]; ++k)
    if (ss_keep(i, ij[k], ax[k], eps_i, dg)) mx = fmax(mx, fabs(ax[k]));
  const double inv = mx != 0.0 ? 1.0 / mx : 0.0;
  int32_t o = sp[i];
  for (int k = ip[i]; k < ip[i + 1]; ++k)
    if (ss_keep(i, ij[k], ax[k], eps_i, dg)) {
      sj[o] = ij[k];
      sx[o] = fabs(ax[k]) * inv;
      ++o;
    }
}

// ---------------------------------------------------------------- standard aggregation
// amg_core standard_aggregation, pass 1 (sequential in the row order): an unmarked row i with
// off-diagonal neighbours none of which is marked becomes a root and marks itself and every
// column of its row; a row with no off-diagonal entry is marked isolated. Whether row i is a
// root depends only on the decisions of rows r < i that could have marked i or one of its
// neighbours v (r = v, or v a column of row r: the transpose's row v), and on its neighbours
// j < i being isolated (their isolated mark blocks i). That makes pass 1 the lexicographically
// first independent set of that conflict relation, decided here in rounds: a row becomes a
// non-root as soon as one such r is a root, a root once all of them are decided non-roots. The
// smallest undecided row always decides, so rounds terminate; each thread walks a run of
// consecutive rows in order, so a chain of decisions inside a run resolves in one round, and a
// row that must wait re-reads only the row it waits on until that row is decided.
// rows per thread: long runs resolve chains of short-row operators in one round; an operator
// with long rows (coarse Galerkin levels: ~30 entries, ~900 markers per decision) gets short
// runs so that one round's work is spread over enough threads
static int sa_run_len(const mlamg_csr* C) {
  const double m = C->n_rows ? (double)C->nnz / (double)C->n_rows : 1.0;
  return (int)std::max(1.0, std::min(32.0, 512.0 / (m * m)));
}
enum : int8_t { kSaUndecided = 0, kSaRoot = 1, kSaNonRoot = 2 };

__global__ void k_sa_iso(const int32_t* __restrict__ ip, const int32_t* __restrict__ ij,
                         int64_t n, int8_t* __restrict__ iso) {
  const int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  int8_t f = 1;
  for (int k = ip[i]; k < ip[i + 1]; ++k)
    if (ij[k] != (int32_t)i) f = 0;
  iso[i] = f;
}

// the decision of row i, or kSaUndecided with *blocker = the smallest undecided row among its
// markers (decisions mostly arrive in row order, so it is usually the last one i waits for);
// `st` entries only ever go from undecided to final
__device__ int8_t sa_decide(int64_t i, const int32_t* __restrict__ ip,
                            const int32_t* __restrict__ ij, const int32_t* __restrict__ tp,
                            const int32_t* __restrict__ tj, const int8_t* __restrict__ iso,
                            const int8_t* st, int32_t* blocker) {
  if (iso[i]) return kSaNonRoot;
  for (int k = ip[i]; k < ip[i + 1]; ++k) {
    const int32_t j = ij[k];
    if (j < i && iso[j]) return kSaNonRoot;
  }
  int32_t blk = INT32_MAX;
  // markers of v: rows r < i with v a column of row r, and v itself; true: a root marks v
  auto check = [&](int32_t v) -> bool {
    if (v < i) {
      const int8_t s = st[v];
      if (s == kSaRoot) return true;
      if (s == kSaUndecided) blk = min(blk, v);
    }
    for (int q = tp[v]; q < tp[v + 1]; ++q) {
      const int32_t r = tj[q];
      if (r >= i || r == v) continue;
      const int8_t s = st[r];
      if (s == kSaRoot) return true;
      if (s == kSaUndecided) blk = min(blk, r);
    }
    return false;
  };
  if (check((int32_t)i)) return kSaNonRoot;
  for (int k = ip[i]; k < ip[i + 1]; ++k) {
    const int32_t j = ij[k];
    if (j != (int32_t)i && check(j)) return kSaNonRoot;
  }
  if (blk == INT32_MAX) return kSaRoot;
  *blocker = blk;
  return kSaUndecided;
}

// one round: a thread walks its run of rows in order (a chain of decisions inside the run
// resolves in one round); an undecided row remembers the row it waits on and is re-examined only
// once that row is decided (two byte reads per round until then). Reads of other threads'
// decisions may be stale within a launch — they can only read as undecided: a delay, never a
// wrong decision; the launch boundary makes every decision visible to the next round.
__global__ void k_sa_round(const int32_t* __restrict__ ip, const int32_t* __restrict__ ij,
                           const int32_t* __restrict__ tp, const int32_t* __restrict__ tj,
                           const int8_t* __restrict__ iso, int64_t n, int8_t* st,
                           int32_t* __restrict__ wait, int32_t* __restrict__ run_pos,
                           int run_len, int32_t* __restrict__ pending) {
  const int64_t r = blockIdx.x * 256ll + threadIdx.x;
  if (r * run_len >= n) return;
  const int64_t z = std::min<int64_t>((r + 1) * run_len, n);
  int64_t first = run_pos[r];
  if (first >= z) return;
  bool all = true;
  for (int64_t i = first; i < z; ++i) {
    if (st[i] != kSaUndecided) {
      if (all) first = i + 1;
      continue;
    }
    const int32_t w = wait[i];
    if (w >= 0 && st[w] == kSaUndecided) {
      all = false;
      continue;
    }
    int32_t blk = -1;
    const int8_t d = sa_decide(i, ip, ij, tp, tj, iso, st, &blk);
    if (d == kSaUndecided) {
      wait[i] = blk;
      all = false;
    } else {
      st[i] = d;
      if (all) first = i + 1;
    }
  }
  run_pos[r] = (int32_t)first;
  if (!all) atomicAdd(pending, 1);
}

__global__ void k_sa_runs_init(int64_t runs, int64_t n, int run_len,
                               int32_t* __restrict__ run_pos, int32_t* __restrict__ wait) {
  const int64_t r = blockIdx.x * 256ll + threadIdx.x;
  if (r < runs) run_pos[r] = (int32_t)(r * run_len);
  if (r < n) wait[r] = -1;
}

__global__ void k_sa_root_flag(const int8_t* __restrict__ st, int64_t n, int32_t* __restrict__ f) {
  const int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i < n) f[i] = st[i] == kSaRoot;
}

// pass 1 marks: root r (id from the scan) writes id + 1 to itself and its row's columns (no two
// roots mark the same row); Cpts[id] = r
__global__ void k_sa_mark(const int32_t* __restrict__ ip, const int32_t* __restrict__ ij,
                          const int8_t* __restrict__ st, const int32_t* __restrict__ id, int64_t n,
                          int32_t* __restrict__ x, int32_t* __restrict__ cpts) {
  const int64_t r = blockIdx.x * 256ll + threadIdx.x;
  if (r >= n || st[r] != kSaRoot) return;
  const int32_t v = id[r] + 1;
  x[r] = v;
  for (int k = ip[r]; k < ip[r + 1]; ++k) x[ij[k]] = v;
  if (cpts) cpts[id[r]] = (int32_t)r;
}

// isolated rows nobody marked: -n; then pass 2: an unmarked row joins the aggregate of its first
// (stored order) neighbour with a pass-1 mark (> 0), as -mark (negative marks are never > 0, so
// rows of pass 2 do not chain)
__global__ void k_sa_iso_mark(const int8_t* __restrict__ iso, int64_t n, int32_t* __restrict__ x) {
  const int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i < n && iso[i] && x[i] == 0) x[i] = -(int32_t)n;
}

__global__ void k_sa_pass2(const int32_t* __restrict__ ip, const int32_t* __restrict__ ij,
                           int64_t n, int32_t* x, int32_t* __restrict__ unmarked) {
  const int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n || x[i] != 0) return;
  for (int k = ip[i]; k < ip[i + 1]; ++k) {
    const int32_t xj = x[ij[k]];
    if (xj > 0) {
      x[i] = -xj;
      return;
    }
  }
  atomicMin(unmarked, (int32_t)i);
}

// pass 3 conversion of rows below `lim`: mark m > 0 -> m - 1, -n -> -1, other m < 0 -> -m - 1
__global__ void k_sa_convert(int64_t lim, int64_t n, int32_t* __restrict__ x) {
  const int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= lim) return;
  const int32_t v = x[i];
  if (v > 0) x[i] = v - 1;
  else if (v == -(int32_t)n) x[i] = -1;
  else if (v < 0) x[i] = -v - 1;
}

// the rest of pass 3 from the first row still unmarked after pass 2 (only non-symmetric patterns
// leave one): amg_core's loop literally, one thread, rows u0..n-1 in order
__global__ void k_sa_pass3_tail(const int32_t* __restrict__ ip, const int32_t* __restrict__ ij,
                                int64_t u0, int64_t n, int32_t* x, int32_t* cpts,
                                int32_t* next_agg) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  int32_t next = *next_agg;
  for (int64_t i = u0; i < n; ++i) {
    const int32_t v = x[i];
    if (v != 0) {
      if (v > 0) x[i] = v - 1;
      else if (v == -(int32_t)n) x[i] = -1;
      else x[i] = -v - 1;
      continue;
    }
    x[i] = next;
    if (cpts) cpts[next] = (int32_t)i;
    for (int k = ip[i]; k < ip[i + 1]; ++k)
      if (x[ij[k]] == 0) x[ij[k]] = next;
    ++next;
  }
  *next_agg = next;
}

// ---------------------------------------------------------------- fit_candidates (one candidate)
// amg_core fit_candidates_common with K1 = K2 = 1: per aggregate (AggOp column, rows ascending),
// norm = sqrt(sum B_i^2); scale = 1 / norm if norm > tol * norm else 0; R = norm (or 0);
// T_i = B_i * scale.
__global__ void k_fit_norm(const int32_t* __restrict__ tp, const int32_t* __restrict__ tj,
                           const double* __restrict__ B, int64_t k, double tol,
                           double* __restrict__ scale, double* __restrict__ Bc) {
  const int64_t j = blockIdx.x * 256ll + threadIdx.x;
  if (j >= k) return;
  double s = 0.0;
  for (int q = tp[j]; q < tp[j + 1]; ++q) {
    const double b = B[tj[q]];
    s += b * b;
  }
  const double nrm = sqrt(s);
  const double thr = tol * nrm;
  const bool ok = nrm > thr;
  scale[j] = ok ? 1.0 / nrm : 0.0;
  Bc[j] = ok ? nrm : 0.0;
}

__global__ void k_fit_vals(const int32_t* __restrict__ ip, const int32_t* __restrict__ ij,
                           int64_t n, const double* __restrict__ B,
                           const double* __restrict__ scale, double* __restrict__ tx) {
  const int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  for (int k = ip[i]; k < ip[i + 1]; ++k) tx[k] = B[i] * scale[ij[k]];
}

// ---------------------------------------------------------------- C = A - B
// scipy csr_binop_csr (canonical inputs): a - b where both rows hold the column, a - 0 and
// 0 - b where one does; results equal to 0 are not stored; columns ascending
template <bool FILL>
__global__ void k_csr_sub(const int32_t* __restrict__ ap, const int32_t* __restrict__ aj,
                          const double* __restrict__ ax, const int32_t* __restrict__ bp,
                          const int32_t* __restrict__ bj, const double* __restrict__ bx,
                          int64_t n, int32_t* __restrict__ cnt, const int32_t* __restrict__ cp,
                          int32_t* __restrict__ cj, double* __restrict__ cx) {
  const int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  int p = ap[i], pe = ap[i + 1], q = bp[i], qe = bp[i + 1];
  int32_t o = FILL ? cp[i] : 0;
  auto emit = [&](int32_t c, double v) {
    if (v != 0.0) {
      if (FILL) {
        cj[o] = c;
        cx[o] = v;
      }
      ++o;
    }
  };
  while (p < pe && q < qe) {
    const int32_t ca = aj[p], cb = bj[q];
    if (ca == cb) emit(ca, ax[p++] - bx[q++]);
    else if (ca < cb) emit(ca, ax[p++] - 0.0);
    else emit(cb, 0.0 - bx[q++]);
  }
  while (p < pe) {
    emit(aj[p], ax[p] - 0.0);
    ++p;
  }
  while (q < qe) {
    emit(bj[q], 0.0 - bx[q]);
    ++q;
  }
  if (!FILL) cnt[i] = o;
}

// get_diagonal(A, inv=True): 1 / (sum of the diagonal entries), 0 where that sum is 0
__global__ void k_diag_pinv(const int32_t* __restrict__ ip, const int32_t* __restrict__ ij,
                            const double* __restrict__ ax, int64_t n, double* __restrict__ d) {
  const int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  double s = 0.0;
  for (int k = ip[i]; k < ip[i + 1]; ++k)
    if (ij[k] == (int32_t)i) s += ax[k];
  d[i] = s != 0.0 ? 1.0 / s : 0.0;
}

// a copy of A with every row's columns in ascending order (A^T^T; values and duplicates kept)
static int sorted_copy(const mlamg_csr* A, mlamg_csr** out, hipStream_t s) {
  mlamg_csr* T = nullptr;
  MLAMG_TRY(transpose_impl(A, &T, s));
  const int rc = transpose_impl(T, out, s);
  csr_free(T);
  return rc;
}

// CSR of n rows from per-row counts (device): indptr by scan, arrays allocated
static int csr_from_counts(const int32_t* cnt, int64_t n_rows, int64_t n_cols, mlamg_csr** out,
                           hipStream_t s) {
  int32_t* ip = nullptr;
  MLAMG_HIP(hipMalloc(&ip, sizeof(int32_t) * (n_rows + 1)));
  int rc = exclusive_scan_i32(cnt, ip, n_rows, s);
  int32_t nnz = 0;
  if (rc == MLAMG_OK) {
    (void)hipMemcpyAsync(&nnz, ip + n_rows, sizeof(int32_t), hipMemcpyDeviceToHost, s);
    if (hipStreamSynchronize(s) != hipSuccess) rc = MLAMG_EHIP;
  }
  mlamg_csr* C = nullptr;
  if (rc == MLAMG_OK) rc = csr_alloc(n_rows, n_cols, nnz, &C);
  if (rc == MLAMG_OK &&
      hipMemcpyAsync(C->indptr, ip, sizeof(int32_t) * (n_rows + 1), hipMemcpyDeviceToDevice, s) !=
          hipSuccess)
    rc = MLAMG_EHIP;
  (void)hipStreamSynchronize(s);
  (void)hipFree(ip);
  if (rc != MLAMG_OK) {
    if (C) csr_free(C);
    return rc;
  }
  *out = C;
  return MLAMG_OK;
}

}  // namespace mlamg

using namespace mlamg;

extern "C" {

int mlamg_symmetric_strength(const mlamg_csr* A, double theta, mlamg_csr** out, void* stream) {
  MLAMG_REQUIRE(A && out, "NULL argument");
  MLAMG_REQUIRE(A->n_rows == A->n_cols, "square matrix required");
  MLAMG_REQUIRE(theta >= 0.0, "expected a positive theta");
  hipStream_t s = S(stream);
  const int64_t n = A->n_rows;
  double* dg = nullptr;
  int32_t* cnt = nullptr;
  MLAMG_HIP(hipMalloc(&dg, sizeof(double) * std::max<int64_t>(n, 1)));
  if (hipMalloc(&cnt, sizeof(int32_t) * std::max<int64_t>(n, 1)) != hipSuccess) {
    (void)hipFree(dg);
    set_error("symmetric_strength: hipMalloc failed");
    return MLAMG_ENOMEM;
  }
  if (n) {
    hipLaunchKernelGGL(k_ss_diag, gsa(n), dim3(256), 0, s, A->indptr, A->indices, A->data, n, dg);
    hipLaunchKernelGGL(k_ss_count, gsa(n), dim3(256), 0, s, A->indptr, A->indices, A->data, n,
                       theta, dg, cnt);
  }
  mlamg_csr* C = nullptr;
  int rc = csr_from_counts(cnt, n, n, &C, s);
  if (rc == MLAMG_OK && n)
    hipLaunchKernelGGL(k_ss_fill, gsa(n), dim3(256), 0, s, A->indptr, A->indices, A->data, n,
                       theta, dg, C->indptr, C->indices, C->data);
  if (rc == MLAMG_OK) rc = csr_finalize(C, s);
  (void)hipStreamSynchronize(s);
  (void)hipFree(dg);
  (void)hipFree(cnt);
  if (rc != MLAMG_OK) {
    if (C) csr_free(C);
    return rc;
  }
  *out = C;
  return MLAMG_OK;
}

int mlamg_standard_aggregation(const mlamg_csr* C, int32_t* agg, int32_t* cpts, int64_t* n_agg,
                               int32_t* rounds_host, void* stream) {
  MLAMG_REQUIRE(C && n_agg && (C->n_rows == 0 || agg), "NULL argument");
  MLAMG_REQUIRE(C->n_rows == C->n_cols, "square matrix required");
  hipStream_t s = S(stream);
  const int64_t n = C->n_rows;
  *n_agg = 0;
  if (rounds_host) *rounds_host = 0;
  if (n == 0) return MLAMG_OK;
  mlamg_csr* T = nullptr;
  MLAMG_TRY(transpose_impl(C, &T, s));
  const int run_len = sa_run_len(C);
  const int64_t runs = (n + run_len - 1) / run_len;
  constexpr int kBatch = 8;
  int8_t *st = nullptr, *iso = nullptr;
  int32_t *flag = nullptr, *id = nullptr, *ctr = nullptr, *run_pos = nullptr, *run_wait = nullptr;
  auto cleanup = [&]() {
    for (void* q : {(void*)st, (void*)iso, (void*)run_pos, (void*)run_wait, (void*)flag,
                    (void*)id, (void*)ctr})
      if (q) (void)hipFree(q);
    csr_free(T);
  };
  if (hipMalloc(&st, n) != hipSuccess || hipMalloc(&iso, n) != hipSuccess ||
      hipMalloc(&run_pos, sizeof(int32_t) * runs) != hipSuccess ||
      hipMalloc(&run_wait, sizeof(int32_t) * n) != hipSuccess ||
      hipMalloc(&flag, sizeof(int32_t) * n) != hipSuccess ||
      hipMalloc(&id, sizeof(int32_t) * (n + 1)) != hipSuccess ||
      hipMalloc(&ctr, sizeof(int32_t) * (kBatch + 2)) != hipSuccess) {
    cleanup();
    set_error("standard_aggregation: hipMalloc failed");
    return MLAMG_ENOMEM;
  }
  (void)hipMemsetAsync(st, 0, n, s);
  hipLaunchKernelGGL(k_sa_runs_init, gsa(n), dim3(256), 0, s, runs, n, run_len, run_pos,
                     run_wait);
  hipLaunchKernelGGL(k_sa_iso, gsa(n), dim3(256), 0, s, C->indptr, C->indices, n, iso);
  // pass 1 in rounds, kBatch launches between host checks; the smallest undecided row decides
  // every round, so n + 1 rounds always suffice
  int32_t rounds = 0;
  bool done = false;
  while (!done) {
    if (rounds > n + kBatch) {
      cleanup();
      set_error("standard_aggregation: pass 1 did not converge");
      return MLAMG_EINVAL;
    }
    (void)hipMemsetAsync(ctr, 0, sizeof(int32_t) * kBatch, s);
    for (int b = 0; b < kBatch; ++b)
      hipLaunchKernelGGL(k_sa_round, gsa(runs), dim3(256), 0, s, C->indptr, C->indices,
                         T->indptr, T->indices, iso, n, st, run_wait, run_pos, run_len,
                         ctr + b);
    int32_t h[kBatch];
    (void)hipMemcpyAsync(h, ctr, sizeof(h), hipMemcpyDeviceToHost, s);
    hipError_t e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
      cleanup();
      set_error(std::string("standard_aggregation: ") + hipGetErrorString(e));
      return MLAMG_EHIP;
    }
    for (int b = 0; b < kBatch && !done; ++b) {
      ++rounds;
      done = h[b] == 0;
    }
  }
  // root ids in row order, pass-1 marks, isolated marks, pass 2
  hipLaunchKernelGGL(k_sa_root_flag, gsa(n), dim3(256), 0, s, st, n, flag);
  int rc = exclusive_scan_i32(flag, id, n, s);
  int32_t n1 = 0;
  if (rc == MLAMG_OK) {
    (void)hipMemcpyAsync(&n1, id + n, sizeof(int32_t), hipMemcpyDeviceToHost, s);
    (void)hipMemsetAsync(agg, 0, sizeof(int32_t) * n, s);
    hipLaunchKernelGGL(k_sa_mark, gsa(n), dim3(256), 0, s, C->indptr, C->indices, st, id, n, agg,
                       cpts);
    hipLaunchKernelGGL(k_sa_iso_mark, gsa(n), dim3(256), 0, s, iso, n, agg);
    const int32_t big = (int32_t)n;
    (void)hipMemcpyAsync(ctr + kBatch, &big, sizeof(int32_t), hipMemcpyHostToDevice, s);
    hipLaunchKernelGGL(k_sa_pass2, gsa(n), dim3(256), 0, s, C->indptr, C->indices, n, agg,
                       ctr + kBatch);
    int32_t u0 = 0;
    (void)hipMemcpyAsync(&u0, ctr + kBatch, sizeof(int32_t), hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
    // pass 3: convert the rows before the first unmarked one in parallel, the rest literally
    hipLaunchKernelGGL(k_sa_convert, gsa(u0), dim3(256), 0, s, (int64_t)u0, n, agg);
    int32_t total = n1;
    if (u0 < n) {
      (void)hipMemcpyAsync(ctr + kBatch + 1, &n1, sizeof(int32_t), hipMemcpyHostToDevice, s);
      hipLaunchKernelGGL(k_sa_pass3_tail, dim3(1), dim3(64), 0, s, C->indptr, C->indices,
                         (int64_t)u0, n, agg, cpts, ctr + kBatch + 1);
      (void)hipMemcpyAsync(&total, ctr + kBatch + 1, sizeof(int32_t), hipMemcpyDeviceToHost, s);
    }
    hipError_t e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
      set_error(std::string("standard_aggregation: ") + hipGetErrorString(e));
      rc = MLAMG_EHIP;
    }
    *n_agg = total;
  }
  if (rounds_host) *rounds_host = rounds;
  cleanup();
  return rc;
}

int mlamg_fit_candidates(const mlamg_csr* AggOp, const double* B, double tol, mlamg_csr** T_out,
                         double* Bc, void* stream) {
  MLAMG_REQUIRE(AggOp && T_out && (AggOp->n_rows == 0 || B) && (AggOp->n_cols == 0 || Bc),
                "NULL argument");
  hipStream_t s = S(stream);
  const int64_t n = AggOp->n_rows, k = AggOp->n_cols;
  mlamg_csr* At = nullptr;
  MLAMG_TRY(transpose_impl(AggOp, &At, s));
  double* scale = nullptr;
  if (hipMalloc(&scale, sizeof(double) * std::max<int64_t>(k, 1)) != hipSuccess) {
    csr_free(At);
    set_error("fit_candidates: hipMalloc failed");
    return MLAMG_ENOMEM;
  }
  mlamg_csr* T = nullptr;
  int rc = csr_alloc(n, k, AggOp->nnz, &T);
  if (rc == MLAMG_OK) {
    (void)hipMemcpyAsync(T->indptr, AggOp->indptr, sizeof(int32_t) * (n + 1),
                         hipMemcpyDeviceToDevice, s);
    if (AggOp->nnz)
      (void)hipMemcpyAsync(T->indices, AggOp->indices, sizeof(int32_t) * AggOp->nnz,
                           hipMemcpyDeviceToDevice, s);
    if (k) hipLaunchKernelGGL(k_fit_norm, gsa(k), dim3(256), 0, s, At->indptr, At->indices, B, k,
                              tol, scale, Bc);
    if (n) hipLaunchKernelGGL(k_fit_vals, gsa(n), dim3(256), 0, s, AggOp->indptr,
                              AggOp->indices, n, B, scale, T->data);
    rc = csr_finalize(T, s);
  }
  (void)hipStreamSynchronize(s);
  (void)hipFree(scale);
  csr_free(At);
  if (rc != MLAMG_OK) {
    if (T) csr_free(T);
    return rc;
  }
  *T_out = T;
  return MLAMG_OK;
}

int mlamg_csr_sub(const mlamg_csr* A, const mlamg_csr* B, mlamg_csr** out, void* stream) {
  MLAMG_REQUIRE(A && B && out, "NULL argument");
  MLAMG_REQUIRE(A->n_rows == B->n_rows && A->n_cols == B->n_cols, "shape mismatch");
  hipStream_t s = S(stream);
  const int64_t n = A->n_rows;
  mlamg_csr *As = nullptr, *Bs = nullptr, *C = nullptr;
  int32_t* cnt = nullptr;
  int rc = sorted_copy(A, &As, s);
  if (rc == MLAMG_OK) rc = sorted_copy(B, &Bs, s);
  if (rc == MLAMG_OK && hipMalloc(&cnt, sizeof(int32_t) * std::max<int64_t>(n, 1)) != hipSuccess)
    rc = MLAMG_ENOMEM;
  if (rc == MLAMG_OK) {
    if (n)
      hipLaunchKernelGGL(k_csr_sub<false>, gsa(n), dim3(256), 0, s, As->indptr, As->indices,
                         As->data, Bs->indptr, Bs->indices, Bs->data, n, cnt, nullptr, nullptr,
                         nullptr);
    rc = csr_from_counts(cnt, n, A->n_cols, &C, s);
  }
  if (rc == MLAMG_OK) {
    if (n)
      hipLaunchKernelGGL(k_csr_sub<true>, gsa(n), dim3(256), 0, s, As->indptr, As->indices,
                         As->data, Bs->indptr, Bs->indices, Bs->data, n, nullptr, C->indptr,
                         C->indices, C->data);
    rc = csr_finalize(C, s);
  }
  (void)hipStreamSynchronize(s);
  if (cnt) (void)hipFree(cnt);
  if (As) csr_free(As);
  if (Bs) csr_free(Bs);
  if (rc != MLAMG_OK) {
    if (C) csr_free(C);
    if (rc == MLAMG_ENOMEM) set_error("csr_sub: hipMalloc failed");
    return rc;
  }
  *out = C;
  return MLAMG_OK;
}

int mlamg_diag_pinv(const mlamg_csr* A, double* dinv, void* stream) {
  MLAMG_REQUIRE(A && (A->n_rows == 0 || dinv), "NULL argument");
  if (A->n_rows)
    hipLaunchKernelGGL(k_diag_pinv, gsa(A->n_rows), dim3(256), 0, S(stream), A->indptr,
                       A->indices, A->data, A->n_rows, dinv);
  MLAMG_HIP(hipGetLastError());
  return MLAMG_OK;
}

}  // extern "C"
