// Coarsest-level direct solve. Replaces spla.factorized / splu (ns/lib/multigrid.py:168,
// ns/preconditioner/MLAMG.py:122): the coarse operator (n_c up to a few thousand) is expanded
// to a dense row-major matrix and inverted once at setup; each V-cycle's coarse solve is then one
// dense GEMV (n_c^2 * 8 bytes, HBM/L2-bound) instead of two sequential triangular solves.
//
// Inverse: a symmetric operator (every Galerkin P^T A P of the reference's SPD A) is inverted
// through its inverse Cholesky factor X = L^-1, built in place by right-looking blocked
// elimination of [A | I] (lower triangle) over the whole GPU — per 32-column panel one panel launch (every
// workgroup factorises the 32 x 32 diagonal block in LDS and solves its share of the rows below
// (L21 = A21 L11^-T) and of the panel's rows of X (Z = L11^-1 [X_top | I])) and one trailing
// launch (16 x 16 tiles on the fp64 matrix cores, v_mfma_f64_16x16x4_f64) — then A^-1 = X^T X
// (an MFMA tile per 16 x 16 block): n^3/3 + n^3/3 multiply-adds in 2 n/32 + 1 launches. A
// non-positive pivot (not SPD in floating point) or an unsymmetric operator takes Gauss-Jordan
// elimination with partial pivoting (one pivot launch + one elimination launch per column),
// which also reports an exactly singular operator like spla.factorized fails.
#include "common.hpp"

#include <cmath>
#include <cstdlib>

namespace mlamg {

__global__ void k_densify(const int32_t* __restrict__ ip, const int32_t* __restrict__ ij,
                          const double* __restrict__ ax, int64_t n, double* __restrict__ M) {
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  for (int k = ip[i]; k < ip[i + 1]; ++k) M[i * n + ij[k]] += ax[k];
}

// One workgroup per step k: argmax_{i >= k} |M[i][k]| (first index on ties), swap rows k and
// the pivot row, save column k, scale row k by 1/pivot (pivot slot -> 1/pivot); phases separated
// by workgroup barriers, one launch.
__global__ __launch_bounds__(1024) void k_gj_row(double* __restrict__ M, int64_t n, int64_t k,
                                                 int32_t* __restrict__ piv,
                                                 double* __restrict__ colk,
                                                 int32_t* __restrict__ fail) {
  __shared__ double bv[1024];
  __shared__ int32_t bi[1024];
  double best = -1.0;
  int32_t bidx = INT32_MAX;
  for (int64_t i = k + threadIdx.x; i < n; i += 1024) {
    const double v = fabs(M[i * n + k]);
    if (v > best) {
      best = v;
      bidx = (int32_t)i;
    }
  }
  bv[threadIdx.x] = best;
  bi[threadIdx.x] = bidx;
  __syncthreads();
  for (int s = 512; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      const double ov = bv[threadIdx.x + s];
      const int32_t oi = bi[threadIdx.x + s];
      if (ov > bv[threadIdx.x] || (ov == bv[threadIdx.x] && oi < bi[threadIdx.x])) {
        bv[threadIdx.x] = ov;
        bi[threadIdx.x] = oi;
      }
    }
    __syncthreads();
  }
  const int32_t p = (bv[0] > 0.0) ? bi[0] : -1;
  if (threadIdx.x == 0) piv[k] = p;
  if (p < 0) {
    if (threadIdx.x == 0) *fail = 1;
    return;
  }
  if (p != k)
    for (int64_t j = threadIdx.x; j < n; j += 1024) {
      const double t = M[k * n + j];
      M[k * n + j] = M[(int64_t)p * n + j];
      M[(int64_t)p * n + j] = t;
    }
  __syncthreads();
  const double inv = 1.0 / M[k * n + k];
  for (int64_t j = threadIdx.x; j < n; j += 1024) colk[j] = M[j * n + k];
  __syncthreads();
  for (int64_t j = threadIdx.x; j < n; j += 1024)
    M[k * n + j] = (j == k) ? inv : M[k * n + j] * inv;
}

// undo the row interchanges as column interchanges, last to first: one thread per row applies
// the whole sequence to its own row (one launch instead of one per interchange)
__global__ void k_unpivot_cols(double* __restrict__ M, int64_t n, const int32_t* __restrict__ piv) {
  const int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  double* r = M + i * n;
  for (int64_t k = n - 1; k >= 0; --k) {
    const int64_t q = piv[k];
    if (q != k) {
      const double t = r[k];
      r[k] = r[q];
      r[q] = t;
    }
  }
}

// eliminate column k from every other row: M[i][j] -= colk[i]*M[k][j]; M[i][k] = -colk[i]*inv
__global__ void k_eliminate(double* __restrict__ M, int64_t n, int64_t k,
                            const int32_t* __restrict__ piv, const double* __restrict__ colk) {
  if (piv[k] < 0) return;
  const int64_t j = blockIdx.x * 256ll + threadIdx.x;
  const int64_t i = blockIdx.y;
  if (j >= n || i == k) return;
  const double f = colk[i];
  if (f == 0.0) return;
  M[i * n + j] = (j == k) ? -f * M[k * n + k] : M[i * n + j] - f * M[k * n + j];
}

// x = M b, one wave per row, fixed-order reduction
__global__ __launch_bounds__(256) void k_gemv(const double* __restrict__ M, int64_t n,
                                              const double* __restrict__ b,
                                              double* __restrict__ x, const int32_t* done) {
  if (done && *done) return;
  const int64_t row = blockIdx.x * 4ll + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  const double* r = M + row * n;
  double s = 0.0;
  // same order as a plain lane-strided loop, with 8 row/b loads of a lane in flight at once (the
  // loop is otherwise a chain of dependent memory round trips: ~10 us for n = 1008); the tail
  // is one more predicated batch (a past-the-end slot adds 0 * 0), not a dependent loop
  for (int64_t j = lane; j < n; j += 8 * 64) {
    double m[8], v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t k = j + u * 64;
      m[u] = k < n ? r[k] : 0.0;
      v[u] = k < n ? b[k] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) s += m[u] * v[u];
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (lane == 0) x[row] = s;
}

// One of the two triangular passes of A^-1 b = X^T (X b) with X = L^-1 kept in M's lower triangle
// and X^T in its strict upper one (method 2): row i of M over columns [0, i] (UP false: y = X b)
// or [i, n) (UP true: x = X^T y, since (X^T)_ij = X_ji = M_ij for j > i). Same wave-per-row
// batches as k_gemv; together the two passes read M once.
template <bool UP>
__global__ __launch_bounds__(256) void k_gemv_tri(const double* __restrict__ M, int64_t n,
                                                  const double* __restrict__ b,
                                                  double* __restrict__ x, const int32_t* done) {
  if (done && *done) return;
  const int64_t row = blockIdx.x * 4ll + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  const double* r = M + row * n;
  const int64_t j0 = UP ? row : 0, j1 = UP ? n : row + 1;
  double s = 0.0;
  for (int64_t j = j0 + lane; j < j1; j += 8 * 64) {
    double m[8], v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t k = j + u * 64;
      m[u] = k < j1 ? r[k] : 0.0;
      v[u] = k < j1 ? b[k] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) s += m[u] * v[u];
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (lane == 0) x[row] = s;
}

// M's strict upper triangle <- the transpose of its strict lower one, 32 x 32 tiles through LDS
// (a workgroup per lower tile: coalesced reads along rows, coalesced writes along rows)
__global__ __launch_bounds__(256) void k_sym_upper(double* __restrict__ M, int64_t n) {
  __shared__ double t[32][33];
  const int64_t bi = blockIdx.y, bj = blockIdx.x;
  if (bj > bi) return;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int r = ty; r < 32; r += 8) {
    const int64_t i = bi * 32 + r, j = bj * 32 + tx;
    t[r][tx] = (i < n && j < n && j < i) ? M[i * n + j] : 0.0;
  }
  __syncthreads();
  for (int c = ty; c < 32; c += 8) {
    const int64_t i = bj * 32 + c, j = bi * 32 + tx;  // (i, j) = transposed (j, i), j > i
    if (i < n && j < n && j > i) M[i * n + j] = t[tx][c];
  }
}

// ------------------------------------------------------------ inverse Cholesky factor
#ifndef MLAMG_DENSE_NB  // panel width (A/B builds; 64: n 11449 factor 109 -> 88 ms, but 26 -> 28 ms
                        // at 7396 and slower fused singles / batches, so 32)
#define MLAMG_DENSE_NB 32
#endif
constexpr int kNB = MLAMG_DENSE_NB;
static_assert(kNB == 32 || kNB == 64, "panel width: 32 or 64 (lane-per-row diagonal factor)");
typedef double d4v __attribute__((ext_vector_type(4)));

// a lane's double, read by the whole wave (two 32-bit lane reads: no LDS round trip)
__device__ __forceinline__ double read_lane(double v, int l) {
  const int2 h = __builtin_bit_cast(int2, v);
  return __builtin_bit_cast(double, make_int2(__builtin_amdgcn_readlane(h.x, l),
                                              __builtin_amdgcn_readlane(h.y, l)));
}

// wave 0 of a workgroup: the diagonal block of panel k0 (lower part of M) factorised L11
// (right-looking), each lane holding its row of the block in registers and reading the other
// rows' column-t entries by lane reads; L11 into Dg (ld kNB + 1), 1/diag(L11) into rd. Returns
// false on a non-positive pivot (same in every lane). Per element the same operations in the
// same order as a right-looking sweep over an LDS copy (l_rt = a_rt * (1 / sqrt(a_tt)),
// a_rc -= l_rt l_ct), without its two wave barriers and LDS round trips per step.
__device__ bool panel_factor(const double* __restrict__ M, int64_t n, int64_t k0, int bw,
                             double* Dg, double* rd) {
  constexpr int ds = kNB + 1;
  const int lane = threadIdx.x & 63;
  const bool own = lane < bw;
  double a[kNB];
#pragma unroll
  for (int c = 0; c < kNB; ++c) a[c] = (own && c <= lane) ? M[(k0 + lane) * n + k0 + c] : 0.0;
  bool ok = true;
  // fully unrolled (a[] stays in registers): steps past bw or after a failed pivot do nothing
#pragma unroll
  for (int t = 0; t < kNB; ++t) {
    const double dtt = read_lane(a[t], t);
    const bool live = ok && t < bw;
    if (live && !(dtt > 0.0)) ok = false;
    if (live && ok) {
      // column t: l_rt = a_rt / sqrt(a_tt), one reciprocal per step
      const double sq = sqrt(dtt), isq = 1.0 / sq;
      if (lane == t) a[t] = sq;
      else if (lane > t && own) a[t] = a[t] * isq;
      if (lane == 0) rd[t] = isq;
      // trailing block: a_rc -= l_rt l_ct, t < c <= r
#pragma unroll
      for (int c = t + 1; c < kNB; ++c) {
        const double lct = read_lane(a[t], c);
        if (c <= lane && own && c < bw) a[c] = a[c] - a[t] * lct;
      }
    }
  }
  if (!ok) return false;
#pragma unroll
  for (int c = 0; c < kNB; ++c)
    if (lane < kNB) Dg[lane * ds + c] = (own && c <= lane) ? a[c] : 0.0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  return true;
}

// Panel k0: block b of the grid takes rows below the panel (L21 = A21 L11^-T into Lp, row-major
// (n - k1) x kNB) and columns < k1 of the panel's rows (Z = L11^-1 [X_top | I], written into M's
// rows k0..k1-1: the final rows of X), a row / column per thread with its values in registers.
__device__ __forceinline__ void chol_panel_body(double* __restrict__ M, int64_t n, int64_t k0,
                                                double* __restrict__ Lp,
                                                double* __restrict__ Zd,
                                                int32_t* __restrict__ fail) {
  __shared__ double Dg[kNB * (kNB + 1)];
  __shared__ double rd[kNB];
  __shared__ int ok_s;
  if (*fail) return;
  const int bw = (int)min<int64_t>(kNB, n - k0);
  const int64_t k1 = k0 + bw;
#ifndef MLAMG_DENSE_LAB  // timing builds only (tools/dense_lab.py): 1 = no row part, 2 = no factor
#define MLAMG_DENSE_LAB 0
#endif
  if (threadIdx.x < 64) {
    const bool ok = MLAMG_DENSE_LAB == 2 ? true : panel_factor(M, n, k0, bw, Dg, rd);
    if (threadIdx.x == 0) ok_s = ok ? 1 : 0;
  }
  __syncthreads();
  if (!ok_s) {
    if (blockIdx.x == 0 && threadIdx.x == 0) *fail = 1;
    return;
  }
  constexpr int ds = kNB + 1;
  const int64_t nrows = n - k1;  // rows below: bw == kNB whenever there are any
  const int64_t item = MLAMG_DENSE_LAB == 1 ? INT64_MAX / 2 : (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (item < nrows) {
    const int64_t i = k1 + item;
    double a[kNB];
#pragma unroll
    for (int t = 0; t < kNB; ++t) a[t] = M[i * n + k0 + t];
#pragma unroll
    for (int t = 0; t < kNB; ++t) {
      double l = a[t];
#pragma unroll
      for (int q = 0; q < t; ++q) l = fma(-a[q], Dg[t * ds + q], l);
      a[t] = l * rd[t];
      Lp[item * kNB + t] = a[t];
    }
  } else if (item < nrows + k1) {
    const int64_t j = item - nrows;  // a column of [X_top | I]
    double z[kNB];
#pragma unroll
    for (int t = 0; t < kNB; ++t)
      z[t] = t >= bw ? 0.0 : (j < k0 ? M[(k0 + t) * n + j] : (j - k0 == t ? 1.0 : 0.0));
#pragma unroll
    for (int t = 0; t < kNB; ++t) {
      if (t < bw) {
        double v = z[t];
#pragma unroll
        for (int q = 0; q < t; ++q) v = fma(-Dg[t * ds + q], z[q], v);
        z[t] = v * rd[t];
        // the diagonal block's columns (L11^-1) go to Zd: other workgroups of this launch are
        // still reading the block from M; the update launch copies them in
        if (j < k0)
          M[(k0 + t) * n + j] = z[t];
        else
          Zd[t * kNB + (j - k0)] = z[t];
      }
    }
  }
}

// Trailing update of panel k0, a wave per 32 x 32 tile (2 x 2 MFMA blocks: per k step two A and
// two B operand loads feed four MFMAs) of rows [k1, n) x columns [0, i]:
//   M[i, j] <- (j in [k0, k1) ? 0 : M[i, j]) - sum_t L21[i][t] W[t][j],
//   W = the panel's rows of X (j < k1) or L21^T (j >= k1).
// Row blocks of 32 from k1 (a multiple of 32 whenever rows remain); row block rb spans column
// tiles 0 .. k1/32 + rb.
constexpr int kUpd = 32;
__device__ __forceinline__ void chol_update_body(double* __restrict__ M, int64_t n, int64_t k0,
                                                 const double* __restrict__ Lp,
                                                 const double* __restrict__ Zd,
                                                 const int32_t* __restrict__ fail) {
  if (*fail) return;
  const int64_t k1 = min<int64_t>(k0 + kNB, n);
  if (blockIdx.x == 0)  // L11^-1 into M's diagonal block (no tile of this launch reads it there)
    for (int q = threadIdx.x; q < kNB * kNB; q += 256) {
      const int t = q / kNB, c = q % kNB;
      if (k0 + t < n && c <= t) M[(k0 + t) * n + k0 + c] = Zd[q];
    }
  if (k1 >= n) return;
  const int64_t a32 = k1 / kUpd, nrb = (n - k1 + kUpd - 1) / kUpd;
  auto C = [&](int64_t rb) { return rb * (a32 + 1) + rb * (rb - 1) / 2; };
  const int64_t T = C(nrb);
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= T) return;
  const int lane = threadIdx.x & 63, lr = lane & 15, lk = lane >> 4;
  const double bq = (double)a32 + 0.5;
  int64_t rb = (int64_t)(-bq + sqrt(bq * bq + 2.0 * (double)q));
  while (rb > 0 && C(rb) > q) --rb;
  while (C(rb + 1) <= q) ++rb;
  const int64_t i0 = k1 + kUpd * rb, j0 = kUpd * (q - C(rb));
  const int64_t last = n - k1 - 1;
  d4v acc[2][2];
  const double* arow[2];
  const double* brow[2];
  bool from_x[2];
  int64_t jz[2];
#pragma unroll
  for (int tj = 0; tj < 2; ++tj) {
    const int64_t jc = j0 + 16 * tj + lr;
    const bool zero = jc >= k0 && jc < k1;
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t i = i0 + 16 * ti + lk + 4 * r;
        acc[ti][tj][r] = (!zero && i < n && jc < n) ? M[i * n + jc] : 0.0;
      }
    from_x[tj] = jc < k1;
    brow[tj] = Lp + min(max(jc - k1, (int64_t)0), last) * kNB;
    jz[tj] = min(jc, k1 - 1);
  }
#pragma unroll
  for (int ti = 0; ti < 2; ++ti) arow[ti] = Lp + min(i0 + 16 * ti + lr - k1, last) * kNB;
#pragma unroll
  for (int kk = 0; kk < kNB; kk += 4) {
    const int k = kk + lk;
    double av[2], bv[2];
#pragma unroll
    for (int ti = 0; ti < 2; ++ti) av[ti] = -arow[ti][k];
#pragma unroll
    for (int tj = 0; tj < 2; ++tj)
      bv[tj] = from_x[tj] ? (jz[tj] >= k0 ? Zd[k * kNB + (jz[tj] - k0)] : M[(k0 + k) * n + jz[tj]])
                          : brow[tj][k];
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int tj = 0; tj < 2; ++tj)
        acc[ti][tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[ti], bv[tj], acc[ti][tj], 0, 0, 0);
  }
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int tj = 0; tj < 2; ++tj) {
      const int64_t jc = j0 + 16 * tj + lr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t i = i0 + 16 * ti + lk + 4 * r;
        if (i < n && jc < n) M[i * n + jc] = acc[ti][tj][r];
      }
    }
}

// A^-1 = X^T X from X = L^-1 (lower triangle of X; its upper triangle is not read): a wave per
// 16 x 16 tile, C_ij = sum over k >= max(i, j) of X_ki X_kj.
__device__ __forceinline__ void xtx_body(const double* __restrict__ X, int64_t n,
                                         double* __restrict__ Cm) {
  const int64_t nb = (n + 15) / 16;
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= nb * nb) return;
  const int lane = threadIdx.x & 63, lr = lane & 15, lk = lane >> 4;
  const int64_t i0 = 16 * (q / nb), j0 = 16 * (q % nb);
  const int64_t ia = i0 + lr, jb = j0 + lr;  // this lane's A row (i) and B column (j)
  d4v acc = {0.0, 0.0, 0.0, 0.0};
  for (int64_t kb = (max(i0, j0) / 4) * 4; kb < n; kb += 4) {
    const int64_t k = kb + lk;
    const double av = (k < n && ia < n && k >= ia) ? X[k * n + ia] : 0.0;
    const double bv = (k < n && jb < n && k >= jb) ? X[k * n + jb] : 0.0;
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t i = i0 + lk + 4 * r;
    if (i < n && jb < n) Cm[i * n + jb] = acc[r];
  }
}

// A symmetric up to rounding, checked on the device: |a_ij - a_ji| <= 1e-12 max(|a_ii|, |a_jj|)
// (a Galerkin P^T A P of a symmetric A is symmetric up to its SpGEMM's summation order; a
// genuinely unsymmetric operator differs by far more). bad[0] counts violations.
__device__ __forceinline__ void asym_body(const double* __restrict__ M, int64_t n,
                                          int32_t* __restrict__ bad) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= n * n) return;
  const int64_t i = q / n, j = q - i * n;
  if (j >= i) return;
  const double d = fmax(fabs(M[i * n + i]), fabs(M[j * n + j]));
  if (!(fabs(M[i * n + j] - M[j * n + i]) <= 1e-12 * d)) atomicAdd(bad, 1);
}

__global__ __launch_bounds__(256) void k_chol_panel(double* __restrict__ M, int64_t n, int64_t k0,
                                                    double* __restrict__ Lp,
                                                    double* __restrict__ Zd,
                                                    int32_t* __restrict__ fail) {
  chol_panel_body(M, n, k0, Lp, Zd, fail);
}
__global__ __launch_bounds__(256) void k_chol_update(double* __restrict__ M, int64_t n,
                                                     int64_t k0, const double* __restrict__ Lp,
                                                     const double* __restrict__ Zd,
                                                     const int32_t* __restrict__ fail) {
  chol_update_body(M, n, k0, Lp, Zd, fail);
}
__global__ __launch_bounds__(256) void k_xtx(const double* __restrict__ X, int64_t n,
                                             double* __restrict__ Cm) {
  xtx_body(X, n, Cm);
}
__global__ void k_asym(const double* __restrict__ M, int64_t n, int32_t* __restrict__ bad) {
  asym_body(M, n, bad);
}

// Many operators at once (the phased batch of batch.hip): job blockIdx.y, each launch sized for
// the largest job; blocks beyond a job's work return. flag[0] = failed pivot, flag[1] = asymmetry
// count: either stops the job's remaining launches.
__global__ __launch_bounds__(256) void k_chol_panel_b(const DenseJob* __restrict__ jobs,
                                                      int64_t k0) {
  const DenseJob J = jobs[blockIdx.y];
  if (k0 >= J.n || (int64_t)blockIdx.x * 256 >= J.n || J.flag[1]) return;
  chol_panel_body(J.M, J.n, k0, J.Lp, J.Zd, J.flag);
}
__global__ __launch_bounds__(256) void k_chol_update_b(const DenseJob* __restrict__ jobs,
                                                       int64_t k0) {
  const DenseJob J = jobs[blockIdx.y];
  if (k0 >= J.n || J.flag[1]) return;
  chol_update_body(J.M, J.n, k0, J.Lp, J.Zd, J.flag);
}
__global__ __launch_bounds__(256) void k_xtx_b(const DenseJob* __restrict__ jobs) {
  const DenseJob J = jobs[blockIdx.y];
  if (J.flag[0] || J.flag[1]) return;
  xtx_body(J.M, J.n, J.inv);
}
__global__ void k_asym_b(const DenseJob* __restrict__ jobs) {
  const DenseJob J = jobs[blockIdx.y];
  asym_body(J.M, J.n, J.flag + 1);
}

int dense_chol_inverse_batch(const DenseJob* jobs_host, int count, bool* spd, hipStream_t s) {
  if (count <= 0) return MLAMG_OK;
  int64_t max_n = 0, lp = 0;
  for (int j = 0; j < count; ++j) {
    max_n = std::max(max_n, jobs_host[j].n);
    lp += ((std::max<int64_t>(jobs_host[j].n, 1) + kNB) * kNB + kNB * kNB + 31) & ~int64_t(31);
  }
  // job table | flags (2 per job) | Lp + Zd per job
  const size_t tab = ((sizeof(DenseJob) * count + 255) & ~size_t(255));
  const size_t fl = ((sizeof(int32_t) * 2 * count + 255) & ~size_t(255));
  char* base = static_cast<char*>(scratch(tab + fl + sizeof(double) * lp, 12));
  MLAMG_REQUIRE(base, "dense batch: scratch allocation failed");
  std::vector<DenseJob> jobs(jobs_host, jobs_host + count);
  int32_t* flags = reinterpret_cast<int32_t*>(base + tab);
  double* work = reinterpret_cast<double*>(base + tab + fl);
  for (int j = 0; j < count; ++j) {
    jobs[j].flag = flags + 2 * j;
    jobs[j].Lp = work;
    jobs[j].Zd = work + (std::max<int64_t>(jobs[j].n, 1) + kNB) * kNB;
    work += ((std::max<int64_t>(jobs[j].n, 1) + kNB) * kNB + kNB * kNB + 31) & ~int64_t(31);
  }
  MLAMG_HIP(hipMemcpyAsync(base, jobs.data(), sizeof(DenseJob) * count, hipMemcpyHostToDevice,
                           s));
  MLAMG_HIP(hipMemsetAsync(flags, 0, sizeof(int32_t) * 2 * count, s));
  const DenseJob* dj = reinterpret_cast<const DenseJob*>(base);
  const unsigned cy = (unsigned)count;
  hipLaunchKernelGGL(k_asym_b, dim3((unsigned)((max_n * max_n + 255) / 256), cy), dim3(256), 0, s,
                     dj);
  for (int64_t k0 = 0; k0 < max_n; k0 += kNB) {
    hipLaunchKernelGGL(k_chol_panel_b, dim3((unsigned)((max_n + 255) / 256), cy), dim3(256), 0, s,
                       dj, k0);
    int64_t T = 1;
    for (int j = 0; j < count; ++j) {
      const int64_t n = jobs[j].n, k1 = std::min<int64_t>(k0 + kNB, n);
      if (k0 >= n || k1 >= n) continue;
      const int64_t a32 = k1 / kUpd, nrb = (n - k1 + kUpd - 1) / kUpd;
      T = std::max<int64_t>(T, nrb * (a32 + 1) + nrb * (nrb - 1) / 2);
    }
    hipLaunchKernelGGL(k_chol_update_b, dim3((unsigned)((T + 3) / 4), cy), dim3(256), 0, s, dj,
                       k0);
  }
  const int64_t nb = (max_n + 15) / 16;
  hipLaunchKernelGGL(k_xtx_b, dim3((unsigned)((nb * nb + 3) / 4), cy), dim3(256), 0, s, dj);
  MLAMG_HIP(hipGetLastError());
  std::vector<int32_t> h(2 * (size_t)count);
  MLAMG_HIP(hipMemcpyAsync(h.data(), flags, sizeof(int32_t) * 2 * count, hipMemcpyDeviceToHost,
                           s));
  MLAMG_HIP(hipStreamSynchronize(s));
  for (int j = 0; j < count; ++j) spd[j] = h[2 * j] == 0 && h[2 * j + 1] == 0;
  return MLAMG_OK;
}

// the inverse Cholesky path; *spd false when A is not symmetric to rounding or not SPD in
// floating point (M destroyed, inv untouched garbage). inv null: no X^T X product; M keeps
// X = L^-1 in its lower triangle and X^T in its strict upper one (method 2)
int dense_chol_inverse(double* M, int64_t n, double* inv, bool* spd, hipStream_t s) {
  *spd = false;
  // L21 panel + the diagonal block's L11^-1 + flags from a cached scratch slot (no per-call
  // hipMalloc / hipFree: the fused single-call path factors once per amg_2_v call)
  const size_t lp_doubles = (size_t)(std::max<int64_t>(n, 1) + kNB) * kNB + kNB * kNB;
  double* Lp = static_cast<double*>(scratch(sizeof(double) * lp_doubles + 256, 13));
  if (!Lp) {
    set_error("dense_create: scratch allocation failed");
    return MLAMG_ENOMEM;
  }
  int32_t* flag = reinterpret_cast<int32_t*>(Lp + lp_doubles);
  (void)hipMemsetAsync(flag, 0, sizeof(int32_t) * 2, s);
  hipLaunchKernelGGL(k_asym, dim3((unsigned)((n * n + 255) / 256)), dim3(256), 0, s, M, n,
                     flag + 1);
  int32_t h[2] = {0, 0};
  hipError_t e = hipMemcpyAsync(h, flag, sizeof(h), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e == hipSuccess && h[1] == 0) {
    double* Zd = Lp + std::max<int64_t>(n, 1) * kNB;  // kNB x kNB
    for (int64_t k0 = 0; k0 < n; k0 += kNB) {
      const int64_t k1 = std::min<int64_t>(k0 + kNB, n);
      const int64_t items = (n - k1) + k1;
      hipLaunchKernelGGL(k_chol_panel, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, s, M,
                         n, k0, Lp, Zd, flag);
      int64_t T = 0;
      if (k1 < n) {
        const int64_t a32 = k1 / kUpd, nrb = (n - k1 + kUpd - 1) / kUpd;
        T = nrb * (a32 + 1) + nrb * (nrb - 1) / 2;
      }
      hipLaunchKernelGGL(k_chol_update, dim3((unsigned)std::max<int64_t>(1, (T + 3) / 4)),
                         dim3(256), 0, s, M, n, k0, Lp, Zd, flag);
    }
    e = hipMemcpyAsync(h, flag, sizeof(int32_t), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e == hipSuccess && h[0] == 0) {
      if (inv) {
        const int64_t nb = (n + 15) / 16;
        hipLaunchKernelGGL(k_xtx, dim3((unsigned)((nb * nb + 3) / 4)), dim3(256), 0, s, M, n,
                           inv);
      } else {  // keep X and mirror it: the two triangular passes of method 2
        const unsigned nt = (unsigned)((n + 31) / 32);
        hipLaunchKernelGGL(k_sym_upper, dim3(nt, nt), dim3(256), 0, s, M, n);
      }
      e = hipStreamSynchronize(s);
      *spd = e == hipSuccess;
    }
  }
  if (e != hipSuccess) {
    set_error(std::string("dense_create: ") + hipGetErrorString(e));
    return MLAMG_EHIP;
  }
  return MLAMG_OK;
}

int dense_solve_impl(const mlamg_dense* D, const double* b, double* x, const int32_t* done,
                     hipStream_t s) {
  if (D->n == 0) return MLAMG_OK;
  if (D->method == 2) {
    hipLaunchKernelGGL(k_gemv_tri<false>, dim3((D->n + 3) / 4), dim3(256), 0, s, D->inv, D->n, b,
                       D->y, done);
    hipLaunchKernelGGL(k_gemv_tri<true>, dim3((D->n + 3) / 4), dim3(256), 0, s, D->inv, D->n,
                       D->y, x, done);
  } else {
    hipLaunchKernelGGL(k_gemv, dim3((D->n + 3) / 4), dim3(256), 0, s, D->inv, D->n, b, x, done);
  }
  MLAMG_HIP(hipGetLastError());
  return MLAMG_OK;
}

}  // namespace mlamg

using namespace mlamg;

extern "C" {

// operators of at least this many rows keep the factor (method 2); MLAMG_DENSE_TRI_MIN overrides
static int64_t dense_tri_min() {
  const char* e = std::getenv("MLAMG_DENSE_TRI_MIN");
  return e ? std::atoll(e) : 2048;
}

int mlamg_dense_create(const mlamg_csr* A, mlamg_dense** out, void* stream) {
  MLAMG_REQUIRE(A && out, "NULL argument");
  MLAMG_REQUIRE(A->n_rows == A->n_cols, "square matrix required");
  MLAMG_REQUIRE(A->n_rows <= 32768, "coarse matrix too large for the dense solver");
  hipStream_t s = S(stream);
  const int64_t n = A->n_rows;
  auto* D = new mlamg_dense();
  D->n = n;
  int32_t* piv = nullptr;
  double* colk = nullptr;
  int32_t* fail = nullptr;
  auto cleanup = [&]() {
    if (piv) (void)hipFree(piv);
    if (colk) (void)hipFree(colk);
    if (fail) (void)hipFree(fail);
  };
  if (hipMalloc(&D->inv, sizeof(double) * std::max<int64_t>(n * n, 1)) != hipSuccess ||
      hipMalloc(&piv, sizeof(int32_t) * std::max<int64_t>(n, 1)) != hipSuccess ||
      hipMalloc(&colk, sizeof(double) * std::max<int64_t>(n, 1)) != hipSuccess ||
      hipMalloc(&fail, sizeof(int32_t)) != hipSuccess) {
    cleanup();
    if (D->inv) (void)hipFree(D->inv);
    delete D;
    set_error("dense_create: hipMalloc failed");
    return MLAMG_ENOMEM;
  }
  if (n >= dense_tri_min() && !std::getenv("MLAMG_DENSE_GJ") &&
      hipMalloc(&D->y, sizeof(double) * n) == hipSuccess) {
    // large operators: the inverse Cholesky factor in place, applied as two triangular passes
    // (no O(n^3) X^T X product; the same n^2 doubles read per solve)
    (void)hipMemsetAsync(D->inv, 0, sizeof(double) * n * n, s);
    hipLaunchKernelGGL(k_densify, dim3((n + 255) / 256), dim3(256), 0, s, A->indptr, A->indices,
                       A->data, n, D->inv);
    bool spd = false;
    const int rc = dense_chol_inverse(D->inv, n, nullptr, &spd, s);
    if (rc != MLAMG_OK) {
      cleanup();
      (void)hipFree(D->inv);
      (void)hipFree(D->y);
      delete D;
      return rc;
    }
    if (spd) {
      cleanup();
      D->method = 2;
      *out = D;
      return MLAMG_OK;
    }
    (void)hipFree(D->y);  // not SPD: Gauss-Jordan below (the matrix is densified again)
    D->y = nullptr;
  } else if (n >= 64 && !std::getenv("MLAMG_DENSE_GJ")) {
    // inverse Cholesky factor in a scratch copy, the inverse into D->inv
    double* M = nullptr;
    if (hipMalloc(&M, sizeof(double) * n * n) == hipSuccess) {
      (void)hipMemsetAsync(M, 0, sizeof(double) * n * n, s);
      hipLaunchKernelGGL(k_densify, dim3((n + 255) / 256), dim3(256), 0, s, A->indptr,
                         A->indices, A->data, n, M);
      bool spd = false;
      const int rc = dense_chol_inverse(M, n, D->inv, &spd, s);
      (void)hipFree(M);
      if (rc != MLAMG_OK) {
        cleanup();
        (void)hipFree(D->inv);
        delete D;
        return rc;
      }
      if (spd) {
        cleanup();
        D->method = 1;
        *out = D;
        return MLAMG_OK;
      }
    }
  }
  (void)hipMemsetAsync(D->inv, 0, sizeof(double) * n * n, s);
  (void)hipMemsetAsync(fail, 0, sizeof(int32_t), s);
  if (n) hipLaunchKernelGGL(k_densify, dim3((n + 255) / 256), dim3(256), 0, s, A->indptr,
                            A->indices, A->data, n, D->inv);
  const unsigned gcols = (unsigned)((n + 255) / 256);
  for (int64_t k = 0; k < n; ++k) {
    hipLaunchKernelGGL(k_gj_row, dim3(1), dim3(1024), 0, s, D->inv, n, k, piv, colk, fail);
    hipLaunchKernelGGL(k_eliminate, dim3(gcols, (unsigned)n), dim3(256), 0, s, D->inv, n, k, piv,
                       colk);
  }
  int32_t hfail = 0;
  (void)hipMemcpyAsync(&hfail, fail, sizeof(int32_t), hipMemcpyDeviceToHost, s);
  hipError_t e = hipStreamSynchronize(s);
  if (e != hipSuccess || hfail) {
    cleanup();
    (void)hipFree(D->inv);
    delete D;
    if (e != hipSuccess) {
      set_error(std::string("dense_create: ") + hipGetErrorString(e));
      return MLAMG_EHIP;
    }
    set_error("dense_create: matrix is exactly singular");
    return MLAMG_EINVAL;
  }
  // undo the row interchanges as column interchanges, last to first
  hipLaunchKernelGGL(k_unpivot_cols, dim3(gcols), dim3(256), 0, s, D->inv, n, piv);
  e = hipStreamSynchronize(s);
  cleanup();
  if (e != hipSuccess) {
    (void)hipFree(D->inv);
    delete D;
    set_error(std::string("dense_create: ") + hipGetErrorString(e));
    return MLAMG_EHIP;
  }
  *out = D;
  return MLAMG_OK;
}

int mlamg_dense_create_matrix(const double* M_host, int64_t n, mlamg_dense** out, void* stream) {
  MLAMG_REQUIRE(out && (n == 0 || M_host), "NULL argument");
  MLAMG_REQUIRE(n >= 0 && n <= 32768, "matrix too large for the dense solver");
  hipStream_t s = S(stream);
  auto* D = new mlamg_dense();
  D->n = n;
  if (hipMalloc(&D->inv, sizeof(double) * std::max<int64_t>(n * n, 1)) != hipSuccess) {
    delete D;
    set_error("dense_create_matrix: hipMalloc failed");
    return MLAMG_ENOMEM;
  }
  hipError_t e = hipSuccess;
  if (n) e = hipMemcpyAsync(D->inv, M_host, sizeof(double) * n * n, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    (void)hipFree(D->inv);
    delete D;
    set_error(std::string("dense_create_matrix: ") + hipGetErrorString(e));
    return MLAMG_EHIP;
  }
  D->method = 0;  // applied as x = M b (k_gemv)
  *out = D;
  return MLAMG_OK;
}

int mlamg_dense_info(const mlamg_dense* D, int* method, int64_t* n) {
  MLAMG_REQUIRE(D, "NULL argument");
  if (method) *method = D->method;
  if (n) *n = D->n;
  return MLAMG_OK;
}

int mlamg_dense_destroy(mlamg_dense* D) {
  if (D) {
    if (D->inv) (void)hipFree(D->inv);
    if (D->y) (void)hipFree(D->y);
    delete D;
  }
  return MLAMG_OK;
}

int mlamg_dense_solve(const mlamg_dense* D, const double* b, double* x, void* stream) {
  MLAMG_REQUIRE(D && (D->n == 0 || (b && x)), "NULL argument");
  MLAMG_REQUIRE(b != x, "b and x must differ");
  return dense_solve_impl(D, b, x, nullptr, S(stream));
}

}  // extern "C"
