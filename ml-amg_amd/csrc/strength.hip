// Evolution strength of connection — the default measure of the reference's evaluation and
// training loops: utils/common.py:26-31 `strength_measure_funcs['olson'](A)` =
// pyamg.strength.evolution_strength_of_connection(A) + 1/|A| (also 'evolution' =
// evolution(A) + 0.1 * unit(A)), called per grid at utils/common.py:53,
// utils/evaluate_dataset.py:76,84, utils/train_one_sample.py:61, demos/train_edge_removal.py:63.
//
// pyamg is not in the reference tree (an unpinned pip dependency), so this is a
// restatement of pyamg 4.x/5.x `evolution_strength_of_connection` at the reference's arguments
// (B = ones, epsilon = 4, k = 2, proj_type 'l2', symmetrize_measure=True, CSR input):
//   Dinv = 1/diag(A) (1 where the diagonal is 0);  U = I - (1/rho) Dinv A   (scipy binop: exact
//   zeros dropped);  T = U^T;  S = T^2 restricted to the pattern of A (amg_core
//   incomplete_mat_mult_csr: a sorted merge per entry, products summed in ascending k), zeros
//   dropped;  the B = ones shortcut per entry (i, j): ratio = S_ii / S_ij, weak if the angle
//   S_ii * S_ij < 0 or |ratio| < 1e-4, else |1 - ratio|, zeros dropped, values below sqrt(eps)
//   -> 1e-4;  amg_core apply_distance_filter (row minimum off-diagonal m: entries >= 4 m
//   dropped; a diagonal entry -> 1);  0.5 (E + E^T);  + (I - diag) (diagonal -> 1);  1/x;  each
//   row scaled by the reciprocal of its largest |entry| (amg_core maximum_row_value +
//   scale_rows). rho = rho(Dinv A): pyamg estimates it by restarted Arnoldi from a seeded random
//   vector; the caller passes the value (the Python mirror uses the device Lanczos lambda_max).
//
// Device layout: A in CSR with ascending column indices and no explicit zeros (what pyamg
// sorts/eliminates to); every step is a thread-per-row kernel over short rows (count, scan,
// fill where the pattern changes), each entry formed with the reference's roundings
// (-ffp-contract=off: separate multiply and add, as scipy sparsetools / amg_core).
#include "common.hpp"

#include <cmath>
#include <limits>

namespace mlamg {
namespace {

constexpr int kT = 256;

inline unsigned grid_for(int64_t n) { return (unsigned)std::max<int64_t>(1, (n + kT - 1) / kT); }

// U = I - c * (Dinv A) row by row (Dinv_i = 1/a_ii, 1 when 0), a diagonal inserted when A has
// none; entries equal to zero dropped. Pass 0 counts, pass 1 fills.
template <int PASS>
__global__ void k_evo_u(const int32_t* __restrict__ ip, const int32_t* __restrict__ ij,
                        const double* __restrict__ ax, int64_t n, double c,
                        int32_t* __restrict__ cnt, const int32_t* __restrict__ up,
                        int32_t* __restrict__ uj, double* __restrict__ ux) {
  const int64_t i = blockIdx.x * (int64_t)kT + threadIdx.x;
  if (i >= n) return;
  const int32_t lo = ip[i], hi = ip[i + 1];
  double d = 0.0;  // scipy diagonal(): the sum of the (canonical: single) diagonal entries
  for (int32_t k = lo; k < hi; ++k)
    if (ij[k] == i) d += ax[k];
  const double dinv = d != 0.0 ? 1.0 / d : 1.0;
  int32_t o = PASS ? up[i] : 0;
  bool diag_done = false;
  auto emit = [&](int32_t col, double v) {
    if (v != 0.0) {
      if (PASS) {
        uj[o] = col;
        ux[o] = v;
      }
      ++o;
    }
  };
  for (int32_t k = lo; k < hi; ++k) {
    const int32_t j = ij[k];
    if (!diag_done && j > i) {  // I only
      emit((int32_t)i, 1.0);
      diag_done = true;
    }
    const double x = (ax[k] * dinv) * c;
    if (j == i) {
      emit(j, 1.0 - x);
      diag_done = true;
    } else {
      emit(j, 0.0 - x);
    }
  }
  if (!diag_done) emit((int32_t)i, 1.0);
  if (!PASS) cnt[i] = o;
}

// S_ij = sum_k T_ik T_kj on the pattern of A (T row i, U row j = column j of T; both sorted),
// then the B = ones shortcut and the distance filter of row i; keep[k] marks surviving entries
// of A's pattern, sx holds their values, cnt[i] counts them.
__global__ void k_evo_s(const int32_t* __restrict__ ip, const int32_t* __restrict__ ij,
                        const double* __restrict__ ax, int64_t n,
                        const int32_t* __restrict__ tp, const int32_t* __restrict__ tj,
                        const double* __restrict__ tx, const int32_t* __restrict__ up,
                        const int32_t* __restrict__ uj, const double* __restrict__ ux,
                        double epsilon, double* __restrict__ sx, int32_t* __restrict__ keep,
                        int32_t* __restrict__ cnt) {
  const int64_t i = blockIdx.x * (int64_t)kT + threadIdx.x;
  if (i >= n) return;
  const int32_t lo = ip[i], hi = ip[i + 1];
  // incomplete_mat_mult_csr
  for (int32_t q = lo; q < hi; ++q) {
    const int32_t j = ij[q];
    int32_t a = tp[i], ae = tp[i + 1], b = up[j], be = up[j + 1];
    double sum = 0.0;
    while (a < ae && b < be) {
      const int32_t ca = tj[a], cb = uj[b];
      if (ca == cb) {
        sum += tx[a] * ux[b];
        ++a;
        ++b;
      } else if (ca < cb) {
        ++a;
      } else {
        ++b;
      }
    }
    sx[q] = sum;
    // the mask is A after eliminate_zeros(); Atilde.eliminate_zeros() after the product
    keep[q] = sum != 0.0 && ax[q] != 0.0;
  }
  double dii = 0.0;  // Atilde.diagonal() after elimination
  for (int32_t q = lo; q < hi; ++q)
    if (keep[q] && ij[q] == i) dii += sx[q];
  const double tiny = 1.4901161193847656e-08;  // np.sqrt(np.finfo(float).eps)
  for (int32_t q = lo; q < hi; ++q) {
    if (!keep[q]) continue;
    const double data = sx[q];
    const double zt = dii;                       // scale_rows(ones, DAtilde / B) * B_j, B = 1
    const bool angle = (zt * data + 0.0 * 0.0) < 0.0;  // real part of z_tilde * conj(z)
    const double ratio = zt / data;
    const bool weak = fabs(ratio) < 1e-4;
    double v = fabs(1.0 - ratio);
    if (weak || angle) v = 0.0;
    keep[q] = v != 0.0;                          // eliminate_zeros()
    if (keep[q] && v < tiny) v = 1e-4;
    sx[q] = v;
  }
  // apply_distance_filter
  double mn = std::numeric_limits<double>::max();
  for (int32_t q = lo; q < hi; ++q)
    if (keep[q] && ij[q] != i) mn = fmin(mn, sx[q]);
  const double thr = epsilon * mn;
  int32_t c = 0;
  for (int32_t q = lo; q < hi; ++q) {
    if (!keep[q]) continue;
    if (ij[q] == i) {
      sx[q] = 1.0;
    } else if (sx[q] >= thr) {
      sx[q] = 0.0;
      keep[q] = 0;  // eliminate_zeros()
    }
    c += keep[q];
  }
  cnt[i] = c;
}

// rows whose column indices are not strictly ascending
__global__ void k_unsorted_rows(const int32_t* __restrict__ ip, const int32_t* __restrict__ ij,
                                int64_t n, int32_t* __restrict__ bad) {
  const int64_t i = blockIdx.x * (int64_t)kT + threadIdx.x;
  if (i >= n) return;
  for (int32_t q = ip[i] + 1; q < ip[i + 1]; ++q)
    if (ij[q] <= ij[q - 1]) {
      atomicAdd(bad, 1);
      return;
    }
}

// compaction of the kept entries (row order preserved: still sorted)
__global__ void k_compact(const int32_t* __restrict__ ip, const int32_t* __restrict__ ij,
                          int64_t n, const double* __restrict__ sx,
                          const int32_t* __restrict__ keep, const int32_t* __restrict__ ep,
                          int32_t* __restrict__ ej, double* __restrict__ ex) {
  const int64_t i = blockIdx.x * (int64_t)kT + threadIdx.x;
  if (i >= n) return;
  int32_t o = ep[i];
  for (int32_t q = ip[i]; q < ip[i + 1]; ++q)
    if (keep[q]) {
      ej[o] = ij[q];
      ex[o] = sx[q];
      ++o;
    }
}

// Row i of the result: union of E_i, (E^T)_i, the diagonal and (mode > 0) A_i, all sorted.
//   v = 0.5 * (e + et)   (csr_binop_csr: a one-sided entry is e + 0 / 0 + et; zero sums dropped)
//   v = v + (1 - d_ii) at the diagonal (d_ii: diagonal of 0.5 (E + E^T), 0 if absent)
//   v = 1 / v;  v *= 1 / max_row |v|
//   mode 1: v + 1.0 * 0.1 on A's pattern ('evolution'), mode 2: v + 1 / |a| ('olson')
// Pass 0 counts, pass 1 fills.
template <int PASS>
__global__ void k_evo_final(const int32_t* __restrict__ ep, const int32_t* __restrict__ ej,
                            const double* __restrict__ ex, const int32_t* __restrict__ fp,
                            const int32_t* __restrict__ fj, const double* __restrict__ fx,
                            const int32_t* __restrict__ ip, const int32_t* __restrict__ ij,
                            const double* __restrict__ ax, int64_t n, int mode,
                            int32_t* __restrict__ cnt, const int32_t* __restrict__ cp,
                            int32_t* __restrict__ cj, double* __restrict__ cx) {
  const int64_t i = blockIdx.x * (int64_t)kT + threadIdx.x;
  if (i >= n) return;
  const int32_t INF = INT32_MAX;
  // walk 1: the symmetrized + identity row, to find d_ii and the row maximum of 1/v
  auto sym_walk = [&](auto&& visit) {
    int32_t a = ep[i], ae = ep[i + 1], b = fp[i], be = fp[i + 1];
    bool diag = false;
    while (a < ae || b < be || !diag) {
      const int32_t ca = a < ae ? ej[a] : INF, cb = b < be ? fj[b] : INF;
      int32_t col = ca < cb ? ca : cb;
      if (!diag && (int64_t)i <= col) {
        if ((int64_t)i < col) {  // the identity entry alone
          visit((int32_t)i, 0.0, false, true);
          diag = true;
          continue;
        }
        diag = true;  // col == i: merged below
      }
      if (col == INF) break;
      double s;
      if (ca == cb) {
        s = ex[a] + fx[b];
        ++a;
        ++b;
      } else if (ca < cb) {
        s = ex[a] + 0.0;
        ++a;
      } else {
        s = 0.0 + fx[b];
        ++b;
      }
      visit(col, s, s != 0.0, col == (int32_t)i);
    }
  };
  double dii = 0.0;
  sym_walk([&](int32_t col, double s, bool present, bool isdiag) {
    if (isdiag && present) dii += 0.5 * s;
  });
  const double idv = 1.0 - dii;  // Id.data -= Atilde.diagonal()
  auto value = [&](int32_t col, double s, bool present, bool isdiag, bool& keep) {
    double v = present ? 0.5 * s : 0.0;
    if (isdiag) v = v + idv;
    keep = v != 0.0;
    return 1.0 / v;
  };
  double mx = -std::numeric_limits<double>::max();
  bool any = false;
  sym_walk([&](int32_t col, double s, bool present, bool isdiag) {
    bool k;
    const double w = value(col, s, present, isdiag, k);
    if (k) {
      mx = fmax(mx, fabs(w));
      any = true;
    }
  });
  const double scale = (any && mx != 0.0) ? 1.0 / mx : mx;
  // walk 2: emit, merged with A's pattern
  int32_t o = PASS ? cp[i] : 0;
  int32_t q = ip[i];
  const int32_t qe = ip[i + 1];
  auto emit = [&](int32_t col, double v) {
    if (v != 0.0) {
      if (PASS) {
        cj[o] = col;
        cx[o] = v;
      }
      ++o;
    }
  };
  auto add_of = [&](int32_t k) { return mode == 1 ? 1.0 * 0.1 : 1.0 / fabs(ax[k]); };
  sym_walk([&](int32_t col, double s, bool present, bool isdiag) {
    bool k;
    double w = value(col, s, present, isdiag, k);
    if (!k) return;
    w = w * scale;
    if (mode == 0) {
      emit(col, w);
      return;
    }
    while (q < qe && ij[q] < col) {  // A-only entries before this one
      emit(ij[q], 0.0 + add_of(q));
      ++q;
    }
    if (q < qe && ij[q] == col) {
      emit(col, w + add_of(q));
      ++q;
    } else {
      emit(col, w + 0.0);
    }
  });
  if (mode != 0)
    for (; q < qe; ++q) emit(ij[q], 0.0 + add_of(q));
  if (!PASS) cnt[i] = o;
}

struct Tmp {
  std::vector<void*> p;
  ~Tmp() {
    for (void* q : p) (void)hipFree(q);
  }
  template <class T>
  T* get(size_t count) {
    void* q = nullptr;
    if (hipMalloc(&q, sizeof(T) * std::max<size_t>(count, 1)) != hipSuccess) return nullptr;
    p.push_back(q);
    return static_cast<T*>(q);
  }
};

}  // namespace
}  // namespace mlamg

using namespace mlamg;

extern "C" {

int mlamg_evolution_strength(const mlamg_csr* A, double rho, double epsilon, int mode,
                             mlamg_csr** out, void* stream) {
  MLAMG_REQUIRE(A && out, "NULL argument");
  MLAMG_REQUIRE(A->n_rows == A->n_cols, "square matrix required");
  MLAMG_REQUIRE(rho > 0.0 && std::isfinite(rho), "rho must be positive and finite");
  MLAMG_REQUIRE(epsilon >= 1.0, "expected epsilon >= 1.0 (pyamg: epsilon > 1)");
  MLAMG_REQUIRE(mode >= 0 && mode <= 2, "mode must be 0 (evolution), 1 (+0.1 unit), 2 (olson)");
  hipStream_t s = S(stream);
  const int64_t n = A->n_rows, nnz = A->nnz;
  Tmp tmp;
  {  // pyamg sorts A's indices first; the merges here assume it
    int32_t* bad = tmp.get<int32_t>(1);
    MLAMG_REQUIRE(bad, "device allocation failed");
    MLAMG_HIP(hipMemsetAsync(bad, 0, sizeof(int32_t), s));
    hipLaunchKernelGGL(k_unsorted_rows, dim3(grid_for(n)), dim3(kT), 0, s, A->indptr, A->indices,
                       n, bad);
    int32_t nbad = 0;
    MLAMG_HIP(hipMemcpyAsync(&nbad, bad, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    MLAMG_HIP(hipStreamSynchronize(s));
    MLAMG_REQUIRE(nbad == 0, "evolution strength: rows of A must have ascending, distinct column "
                             "indices (sort_indices / sum_duplicates first)");
  }
  // U = I - (1/rho) Dinv A
  int32_t* cnt = tmp.get<int32_t>(n + 1);
  int32_t* upp = tmp.get<int32_t>(n + 1);
  MLAMG_REQUIRE(cnt && upp, "device allocation failed");
  const double c = 1.0 / rho;
  hipLaunchKernelGGL(k_evo_u<0>, dim3(grid_for(n)), dim3(kT), 0, s, A->indptr, A->indices,
                     A->data, n, c, cnt, nullptr, nullptr, nullptr);
  MLAMG_TRY(exclusive_scan_i32(cnt, upp, n, s));
  int32_t nnz_u = 0;
  MLAMG_HIP(hipMemcpyAsync(&nnz_u, upp + n, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  MLAMG_HIP(hipStreamSynchronize(s));
  mlamg_csr* U = nullptr;
  MLAMG_TRY(csr_alloc(n, n, nnz_u, &U));
  struct Guard {
    mlamg_csr* m;
    ~Guard() {
      if (m) csr_free(m);
    }
  } gu{U};
  MLAMG_HIP(hipMemcpyAsync(U->indptr, upp, sizeof(int32_t) * (n + 1), hipMemcpyDeviceToDevice, s));
  hipLaunchKernelGGL(k_evo_u<1>, dim3(grid_for(n)), dim3(kT), 0, s, A->indptr, A->indices,
                     A->data, n, c, nullptr, U->indptr, U->indices, U->data);
  MLAMG_TRY(csr_finalize(U, s));
  // T = U^T (sorted rows)
  mlamg_csr* T = nullptr;
  MLAMG_TRY(mlamg_transpose(U, &T, stream));
  Guard gt{T};
  // S on A's pattern, the shortcut and the distance filter
  double* sx = tmp.get<double>(nnz);
  int32_t* keep = tmp.get<int32_t>(nnz);
  int32_t* epp = tmp.get<int32_t>(n + 1);
  MLAMG_REQUIRE(sx && keep && epp, "device allocation failed");
  hipLaunchKernelGGL(k_evo_s, dim3(grid_for(n)), dim3(kT), 0, s, A->indptr, A->indices, A->data, n,
                     T->indptr, T->indices, T->data, U->indptr, U->indices, U->data, epsilon,
                     sx, keep, cnt);
  MLAMG_TRY(exclusive_scan_i32(cnt, epp, n, s));
  int32_t nnz_e = 0;
  MLAMG_HIP(hipMemcpyAsync(&nnz_e, epp + n, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  MLAMG_HIP(hipStreamSynchronize(s));
  mlamg_csr* E = nullptr;
  MLAMG_TRY(csr_alloc(n, n, nnz_e, &E));
  Guard ge{E};
  MLAMG_HIP(hipMemcpyAsync(E->indptr, epp, sizeof(int32_t) * (n + 1), hipMemcpyDeviceToDevice, s));
  hipLaunchKernelGGL(k_compact, dim3(grid_for(n)), dim3(kT), 0, s, A->indptr, A->indices, n, sx,
                     keep, E->indptr, E->indices, E->data);
  MLAMG_TRY(csr_finalize(E, s));
  mlamg_csr* F = nullptr;  // E^T
  MLAMG_TRY(mlamg_transpose(E, &F, stream));
  Guard gf{F};
  // symmetrize, identity, invert, row scaling, + the measure's second term
  int32_t* cpp = tmp.get<int32_t>(n + 1);
  MLAMG_REQUIRE(cpp, "device allocation failed");
  hipLaunchKernelGGL(k_evo_final<0>, dim3(grid_for(n)), dim3(kT), 0, s, E->indptr, E->indices,
                     E->data, F->indptr, F->indices, F->data, A->indptr, A->indices, A->data, n,
                     mode, cnt, nullptr, nullptr, nullptr);
  MLAMG_TRY(exclusive_scan_i32(cnt, cpp, n, s));
  int32_t nnz_c = 0;
  MLAMG_HIP(hipMemcpyAsync(&nnz_c, cpp + n, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  MLAMG_HIP(hipStreamSynchronize(s));
  mlamg_csr* Cm = nullptr;
  MLAMG_TRY(csr_alloc(n, n, nnz_c, &Cm));
  MLAMG_HIP(hipMemcpyAsync(Cm->indptr, cpp, sizeof(int32_t) * (n + 1), hipMemcpyDeviceToDevice, s));
  hipLaunchKernelGGL(k_evo_final<1>, dim3(grid_for(n)), dim3(kT), 0, s, E->indptr, E->indices,
                     E->data, F->indptr, F->indices, F->data, A->indptr, A->indices, A->data, n,
                     mode, nullptr, Cm->indptr, Cm->indices, Cm->data);
  int rc = csr_finalize(Cm, s);
  if (rc != MLAMG_OK) {
    csr_free(Cm);
    return rc;
  }
  *out = Cm;
  return MLAMG_OK;
}

}  // extern "C"
