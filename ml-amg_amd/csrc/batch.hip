// The reference's own call pattern, one launch per batch: `amg_2_v(A, P, b, x, ...)`
// (ns/lib/multigrid.py:111-210) on small grids, called once per grid by the training and
// evaluation loops (utils/common.py:77,106, utils/evaluate_dataset.py:96,
// utils/train_dataset.py:114) and farmed out over processes (ns/parallel/pool.py). Launching
// the V-cycle kernels of a 1k-16k-row problem one by one leaves the GPU idle between launches,
// so here ONE workgroup runs one whole problem — Galerkin product, coarse inverse, every cycle
// and the tolerance test — and one launch runs a whole batch, one workgroup per problem.
//
// Per problem (workgroup of 1024 threads, x resident in LDS during the cycles):
//   A_H = P^T A P, dense n_c x n_c                 (multigrid.py:165)
//   A_H^-1 by blocked Gauss-Jordan with partial pivoting: panels of b columns factorised in
//     LDS, the row interchanges then the rank-b update applied to the other columns, columns
//     un-interchanged at the end (replaces spla.factorized, :168; singular -> status 1, the
//     reference's `except: return x, 1., err, 0`)
//   cycles (:172-199): pre-smoothing (pyamg forward Gauss-Seidel over a level schedule, bitwise
//     the sequential sweep; or the MLAMG weighted-Jacobi form x += w D^-1 (b - A x)),
//     r = b - A x, r_H = P^T r (ascending fine row per coarse row: scipy csc_matvec's order),
//     e_H = A_H^-1 r_H (wave per row, lane-strided + butterfly: the order of dense.hip k_gemv),
//     x += P e_H, post-smoothing, err[i] = ||b - A x||_2 or ||x||_2, stop at err[i] <= tol.
// Smoothing, residual, restriction and prolongation are bitwise the reference's sparse ops;
// the Galerkin product and the coarse inverse differ from scipy/SuperLU by rounding only
// (fp64 tolerance, like every dense-coarse path of this library).
//
// Structure-only preparation (level schedule of the Gauss-Seidel sweep, the transposed
// sparsity of P, a level-ordered packed copy of A's rows) is done on the host from the CSR
// index arrays the caller hands over; every floating-point operation runs in the kernel.
#include "common.hpp"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace mlamg {
namespace {

constexpr int kBT = 1024;
constexpr int kBWaves = kBT / 64;
constexpr int64_t kBMaxN = 16384;   // fine rows: x lives in LDS during the cycles
constexpr int64_t kBMaxNc = 2048;   // coarse rows: dense inverse, LDS panels of >= 8 columns
constexpr int kBMaxK = 32;          // off-diagonal entries per row (packed sweep layout)
constexpr int kBMaxPanel = 32;
constexpr size_t kBLdsBytes = 156 * 1024;

struct BDesc {
  int32_t n, nc, smoother, nu_pre, nu_post, norm_mode, max_iter, K, nlev, panel;
  int32_t n_chunks, cap, timing, pad_;
  double tol, omega;
  // byte offsets into the arena
  int64_t A_ip, A_ij, A_val, P_ip, P_ij, P_val, PT_ptr, PT_row, PT_src;
  int64_t lev_ptr, chunk_lev, pk_row, pk_col, pk_val, pk_diag, b_lvl, b, x0;
  int64_t AH, r, rc, e, dinv;
  int64_t x_out, err_out, stat_out;
};

template <class T>
__device__ __forceinline__ T* at(char* base, int64_t off) {
  return reinterpret_cast<T*>(base + off);
}

__device__ __forceinline__ double bw_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// fixed-order workgroup sum (wave butterflies, then the 16 wave totals left to right)
__device__ double block_sum(double v, double* red) {
  v = bw_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double t = 0.0;
#pragma unroll
  for (int w = 0; w < kBWaves; ++w) t += red[w];
  __syncthreads();
  return t;
}

// workgroup argmax of |v| over rows, ties to the smallest row (the sequential scan's choice)
__device__ void block_argmax(double v, int idx, double* redv, int* redi, double* outv,
                             int* outi) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const double ov = __shfl_xor(v, off, 64);
    const int oi = __shfl_xor(idx, off, 64);
    if (ov > v || (ov == v && oi < idx)) {
      v = ov;
      idx = oi;
    }
  }
  if ((threadIdx.x & 63) == 0) {
    redv[threadIdx.x >> 6] = v;
    redi[threadIdx.x >> 6] = idx;
  }
  __syncthreads();
  double bv = redv[0];
  int bi = redi[0];
  for (int w = 1; w < kBWaves; ++w)
    if (redv[w] > bv || (redv[w] == bv && redi[w] < bi)) {
      bv = redv[w];
      bi = redi[w];
    }
  *outv = bv;
  *outi = bi;
  __syncthreads();
}

// rows [i0, i1) of column j: M[i][j] = (i in the panel rows ? 0 : M[i][j]) + sum_t pan[i][t] B[t],
// t ascending; 8 rows per step so that 8 loads of the column are in flight at once
__device__ __forceinline__ void panel_update(double* AH, const double* pan, const double* B,
                                             int nc, int pb, int bw, int k0, int j, int i0,
                                             int i1) {
  constexpr int U = 8;
  int i = i0;
  for (; i + U <= i1; i += U) {
    double m[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int ii = i + u;
      m[u] = (ii >= k0 && ii < k0 + bw) ? 0.0 : AH[(int64_t)ii * nc + j];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const double* pr = pan + (i + u) * pb;
      double acc = m[u];
#pragma unroll
      for (int t = 0; t < kBMaxPanel; ++t)
        if (t < bw) acc += pr[t] * B[t];
      AH[(int64_t)(i + u) * nc + j] = acc;
    }
  }
  for (; i < i1; ++i) {
    double acc = (i >= k0 && i < k0 + bw) ? 0.0 : AH[(int64_t)i * nc + j];
    const double* pr = pan + i * pb;
#pragma unroll
    for (int t = 0; t < kBMaxPanel; ++t)
      if (t < bw) acc += pr[t] * B[t];
    AH[(int64_t)i * nc + j] = acc;
  }
}

__global__ __launch_bounds__(kBT) void k_amg2v_batch(const BDesc* __restrict__ descs,
                                                     char* __restrict__ arena) {
  extern __shared__ double lds[];
  __shared__ double redv[kBWaves];
  __shared__ int redi[kBWaves];
  const BDesc D = descs[blockIdx.x];
  const int tid = threadIdx.x;
  const int n = D.n, nc = D.nc;
  const int32_t* __restrict__ aip = at<int32_t>(arena, D.A_ip);
  const int32_t* __restrict__ aij = at<int32_t>(arena, D.A_ij);
  const double* __restrict__ aval = at<double>(arena, D.A_val);
  const int32_t* __restrict__ pip = at<int32_t>(arena, D.P_ip);
  const int32_t* __restrict__ pij = at<int32_t>(arena, D.P_ij);
  const double* __restrict__ pval = at<double>(arena, D.P_val);
  const int32_t* __restrict__ ptp = at<int32_t>(arena, D.PT_ptr);
  const int32_t* __restrict__ ptr_ = at<int32_t>(arena, D.PT_row);
  const int32_t* __restrict__ pts = at<int32_t>(arena, D.PT_src);
  const double* __restrict__ b = at<double>(arena, D.b);
  double* AH = at<double>(arena, D.AH);
  double* r = at<double>(arena, D.r);
  double* rc = at<double>(arena, D.rc);
  double* e = at<double>(arena, D.e);
  double* x_out = at<double>(arena, D.x_out);
  double* err = at<double>(arena, D.err_out);
  int32_t* stat = at<int32_t>(arena, D.stat_out);

  // phase wall times (100 MHz clock) when requested: [galerkin, inverse, smoothing, rest]
  int64_t* tstat = at<int64_t>(arena, D.stat_out + 8);
  int64_t t_mark = D.timing ? wall_clock64() : 0;
  auto stamp = [&](int slot) {
    if (D.timing && tid == 0) {
      const int64_t t = wall_clock64();
      tstat[slot] += t - t_mark;
      t_mark = t;
    }
  };
  if (D.timing && tid == 0)
    for (int q = 0; q < 4; ++q) tstat[q] = 0;

  // ---------------------------------------------------------------- A_H = P^T A P (dense)
  for (int64_t q = tid; q < (int64_t)nc * nc; q += kBT) AH[q] = 0.0;
  __syncthreads();
  for (int j = tid; j < nc; j += kBT) {
    double* row = AH + (int64_t)j * nc;
    for (int t = ptp[j]; t < ptp[j + 1]; ++t) {
      const int i = ptr_[t];
      const double p = pval[pts[t]];
      for (int k = aip[i]; k < aip[i + 1]; ++k) {
        const int c = aij[k];
        const double pa = p * aval[k];
        for (int m = pip[c]; m < pip[c + 1]; ++m) row[pij[m]] += pa * pval[m];
      }
    }
  }
  __syncthreads();

  stamp(0);
  // ---------------------------------------------------------------- A_H^-1, blocked Gauss-Jordan
  const int pb = D.panel;
  double* pan = lds;                                          // nc x pb, row-major
  double* colk = lds + (int64_t)nc * pb;                      // nc
  int32_t* piv = reinterpret_cast<int32_t*>(colk + nc);       // nc
  int status = 0;
  for (int k0 = 0; k0 < nc && status == 0; k0 += pb) {
    const int bw = min(pb, nc - k0);
    for (int q = tid; q < nc * bw; q += kBT) {
      const int i = q / bw, t = q - i * bw;
      pan[i * pb + t] = AH[(int64_t)i * nc + k0 + t];
    }
    __syncthreads();
    for (int t = 0; t < bw; ++t) {
      const int k = k0 + t;
      double v = -1.0;
      int vi = INT32_MAX;
      for (int i = k + tid; i < nc; i += kBT) {
        const double a = fabs(pan[i * pb + t]);
        if (a > v) {
          v = a;
          vi = i;
        }
      }
      double bv;
      int p;
      block_argmax(v, vi, redv, redi, &bv, &p);
      if (!(bv > 0.0)) {  // exactly singular (uniform across the workgroup)
        status = 1;
        break;
      }
      if (tid == 0) piv[k] = p;
      if (p != k)
        for (int s = tid; s < bw; s += kBT) {
          const double tmp = pan[k * pb + s];
          pan[k * pb + s] = pan[p * pb + s];
          pan[p * pb + s] = tmp;
        }
      __syncthreads();
      const double inv = 1.0 / pan[k * pb + t];
      for (int i = tid; i < nc; i += kBT) colk[i] = pan[i * pb + t];
      __syncthreads();
      for (int s = tid; s < bw; s += kBT)
        pan[k * pb + s] = (s == t) ? inv : pan[k * pb + s] * inv;
      __syncthreads();
      for (int q = tid; q < nc * bw; q += kBT) {
        const int i = q / bw, s = q - i * bw;
        if (i == k) continue;
        const double f = colk[i];
        if (f == 0.0) continue;
        pan[i * pb + s] = (s == t) ? -f * pan[k * pb + t] : pan[i * pb + s] - f * pan[k * pb + s];
      }
      __syncthreads();
    }
    if (status) break;
    // the panel's row interchanges on the other columns, then M <- T M on them, where T is the
    // identity with its panel columns replaced by the factorised panel: rows of the panel
    // become sum_t pan[i][t] * B[t], the others gain that sum (B = the panel rows, swapped)
    const int ncol = nc - bw;
    for (int jj = tid; jj < ncol; jj += kBT) {
      const int j = jj < k0 ? jj : jj + bw;
      for (int t = 0; t < bw; ++t) {
        const int k = k0 + t, p = piv[k];
        if (p != k) {
          const double tmp = AH[(int64_t)k * nc + j];
          AH[(int64_t)k * nc + j] = AH[(int64_t)p * nc + j];
          AH[(int64_t)p * nc + j] = tmp;
        }
      }
    }
    __syncthreads();
    if (ncol >= kBT) {  // a thread per column (several each): loads B, then updates it alone
      for (int jj = tid; jj < ncol; jj += kBT) {
        const int j = jj < k0 ? jj : jj + bw;
        double B[kBMaxPanel];
#pragma unroll
        for (int t = 0; t < kBMaxPanel; ++t)
          B[t] = t < bw ? AH[(int64_t)(k0 + t) * nc + j] : 0.0;
        panel_update(AH, pan, B, nc, pb, bw, k0, j, 0, nc);
      }
    } else if (ncol > 0) {  // fewer columns than threads: each column split into row ranges
      const int parts = max(1, min(kBT / ncol, nc));
      const int chunk = (nc + parts - 1) / parts;
      const int jj = tid % ncol, part = tid / ncol;
      const bool active = part < parts;
      const int j = jj < k0 ? jj : jj + bw;
      double B[kBMaxPanel];
#pragma unroll
      for (int t = 0; t < kBMaxPanel; ++t)
        B[t] = (active && t < bw) ? AH[(int64_t)(k0 + t) * nc + j] : 0.0;
      __syncthreads();
      if (active) {
        const int i0 = part * chunk, i1 = min(nc, i0 + chunk);
        panel_update(AH, pan, B, nc, pb, bw, k0, j, i0, i1);
      }
    }
    for (int q = tid; q < nc * bw; q += kBT) {
      const int i = q / bw, t = q - i * bw;
      AH[(int64_t)i * nc + k0 + t] = pan[i * pb + t];
    }
    __syncthreads();
  }
  if (status == 0) {
    // undo the row interchanges as column interchanges, last to first (thread per row)
    for (int i = tid; i < nc; i += kBT) {
      double* rw = AH + (int64_t)i * nc;
      for (int k = nc - 1; k >= 0; --k) {
        const int q = piv[k];
        if (q != k) {
          const double tmp = rw[k];
          rw[k] = rw[q];
          rw[q] = tmp;
        }
      }
    }
  }
  __syncthreads();
  stamp(1);

  // ---------------------------------------------------------------- cycles
  double* xs = lds;  // the panel space is free now
  const double* __restrict__ x0 = at<double>(arena, D.x0);
  for (int i = tid; i < n; i += kBT) xs[i] = x0[i];
  __syncthreads();
  if (status != 0) {  // multigrid.py:167-170: x returned untouched, no iteration
    for (int i = tid; i < n; i += kBT) x_out[i] = xs[i];
    if (tid == 0) {
      stat[0] = 0;
      stat[1] = status;
    }
    return;
  }
  double* dinv = at<double>(arena, D.dinv);
  if (D.smoother == 1) {  // (1/a_ii) * w, a_ii = sum of stored diagonal entries (csr_diagonal)
    for (int i = tid; i < n; i += kBT) {
      double d = 0.0;
      for (int k = aip[i]; k < aip[i + 1]; ++k)
        if (aij[k] == i) d += aval[k];
      dinv[i] = (1.0 / d) * D.omega;
    }
    __syncthreads();
  }
  const int32_t* __restrict__ lptr = at<int32_t>(arena, D.lev_ptr);
  const int32_t* __restrict__ clev = at<int32_t>(arena, D.chunk_lev);
  const int32_t* __restrict__ pkr = at<int32_t>(arena, D.pk_row);
  const int32_t* __restrict__ pkc = at<int32_t>(arena, D.pk_col);
  const double* __restrict__ pkv = at<double>(arena, D.pk_val);
  const double* __restrict__ pkd = at<double>(arena, D.pk_diag);
  const double* __restrict__ bl = at<double>(arena, D.b_lvl);
  const int K = D.K;
  // LDS staging area after x (GS): a chunk of consecutive levels' packed rows, copied in with
  // all loads in flight at once, so a level's critical path is LDS gathers + barrier only
  const int cap = D.cap;
  double* sv = xs + n;                                      // cap*K values
  double* sd = sv + (int64_t)cap * K;                       // cap diagonals
  double* sb = sd + cap;                                    // cap right-hand sides
  int32_t* sc = reinterpret_cast<int32_t*>(sb + cap);       // cap*K columns
  int32_t* sr = sc + (int64_t)cap * K;                      // cap rows
  int32_t* slp = sr + cap;                                  // level starts of the chunk

  auto smooth = [&](int nu) {
    for (int it = 0; it < nu; ++it) {
      if (D.smoother == 0) {
        // pyamg gauss_seidel: rsum over the off-diagonals in stored order, diag = the last
        // stored diagonal entry, x_i = (b_i - rsum) / diag unless diag == 0
        for (int ch = 0; ch < D.n_chunks; ++ch) {
          const int l0 = clev[ch], l1 = clev[ch + 1];
          const int P0 = lptr[l0], cnt = lptr[l1] - P0;
          if (cnt <= cap) {
            for (int q = tid; q < cnt * K; q += kBT) {
              sc[q] = pkc[(int64_t)P0 * K + q];
              sv[q] = pkv[(int64_t)P0 * K + q];
            }
            for (int q = tid; q < cnt; q += kBT) {
              sd[q] = pkd[P0 + q];
              sb[q] = bl[P0 + q];
              sr[q] = pkr[P0 + q];
            }
            for (int q = tid; q <= l1 - l0; q += kBT) slp[q] = lptr[l0 + q] - P0;
            __syncthreads();
            for (int l = 0; l < l1 - l0; ++l) {
              const int a = slp[l], z = slp[l + 1];
              for (int p = a + tid; p < z; p += kBT) {
                double rsum = 0.0;
                for (int s2 = 0; s2 < K; ++s2) {
                  const int c = sc[p * K + s2];
                  if (c < 0) break;
                  rsum += sv[p * K + s2] * xs[c];
                }
                const double dg = sd[p];
                if (dg != 0.0) xs[sr[p]] = (sb[p] - rsum) / dg;
              }
              __syncthreads();
            }
          } else {  // one level wider than the staging area: straight from the arena
            for (int l = l0; l < l1; ++l) {
              const int a = lptr[l], z = lptr[l + 1];
              for (int p = a + tid; p < z; p += kBT) {
                const int32_t* cc = pkc + (int64_t)p * K;
                const double* vv = pkv + (int64_t)p * K;
                double rsum = 0.0;
                for (int s2 = 0; s2 < K; ++s2) {
                  const int c = cc[s2];
                  if (c < 0) break;
                  rsum += vv[s2] * xs[c];
                }
                const double dg = pkd[p];
                if (dg != 0.0) xs[pkr[p]] = (bl[p] - rsum) / dg;
              }
              __syncthreads();
            }
          }
        }
      } else {
        for (int i = tid; i < n; i += kBT) {
          double y = 0.0;
          for (int k = aip[i]; k < aip[i + 1]; ++k) y += aval[k] * xs[aij[k]];
          r[i] = b[i] - y;
        }
        __syncthreads();
        for (int i = tid; i < n; i += kBT) xs[i] = xs[i] + dinv[i] * r[i];
        __syncthreads();
      }
    }
  };

  auto smooth_timed = [&](int nu) {
    stamp(3);
    smooth(nu);
    stamp(2);
  };
  int iters = 0;
  for (int itn = 0; itn < D.max_iter; ++itn) {
    smooth_timed(D.nu_pre);
    for (int i = tid; i < n; i += kBT) {
      double y = 0.0;
      for (int k = aip[i]; k < aip[i + 1]; ++k) y += aval[k] * xs[aij[k]];
      r[i] = b[i] - y;
    }
    __syncthreads();
    for (int j = tid; j < nc; j += kBT) {
      double s = 0.0;
      for (int t = ptp[j]; t < ptp[j + 1]; ++t) s += pval[pts[t]] * r[ptr_[t]];
      rc[j] = s;
    }
    __syncthreads();
    {
      const int w = tid >> 6, lane = tid & 63;
      for (int j = w; j < nc; j += kBWaves) {
        const double* rw = AH + (int64_t)j * nc;
        double s = 0.0;
        int l = lane;
        for (; l + 7 * 64 < nc; l += 8 * 64) {
          double m[8], v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            m[u] = rw[l + u * 64];
            v[u] = rc[l + u * 64];
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) s += m[u] * v[u];
        }
        for (; l < nc; l += 64) s += rw[l] * rc[l];
        s = bw_sum(s);
        if (lane == 0) e[j] = s;
      }
    }
    __syncthreads();
    for (int i = tid; i < n; i += kBT) {
      double y = 0.0;
      for (int k = pip[i]; k < pip[i + 1]; ++k) y += pval[k] * e[pij[k]];
      xs[i] = xs[i] + y;
    }
    __syncthreads();
    smooth_timed(D.nu_post);
    double part = 0.0;
    if (D.norm_mode == 0) {
      for (int i = tid; i < n; i += kBT) {
        double y = 0.0;
        for (int k = aip[i]; k < aip[i + 1]; ++k) y += aval[k] * xs[aij[k]];
        const double ri = b[i] - y;
        part += ri * ri;
      }
    } else {
      for (int i = tid; i < n; i += kBT) part += xs[i] * xs[i];
    }
    const double nrm = sqrt(block_sum(part, redv));
    if (tid == 0) err[itn] = nrm;
    iters = itn + 1;
    if (D.tol >= 0.0 && nrm <= D.tol) break;
  }
  for (int i = tid; i < n; i += kBT) x_out[i] = xs[i];
  stamp(3);
  if (tid == 0) {
    stat[0] = iters;
    stat[1] = 0;
  }
}

struct Layout {
  size_t off = 0;
  int64_t take(size_t bytes) {
    const int64_t o = (int64_t)off;
    off += (std::max<size_t>(bytes, 1) + 255) & ~size_t(255);
    return o;
  }
};

struct HostPinned {
  void* p = nullptr;
  size_t cap = 0;
  ~HostPinned() {
    if (p) (void)hipHostFree(p);
  }
};
thread_local HostPinned g_batch_host;

bool valid_csr(int64_t rows, int64_t cols, int64_t nnz, const int32_t* ip, const int32_t* ij) {
  if (!ip || (nnz > 0 && !ij) || ip[0] != 0 || ip[rows] != nnz) return false;
  for (int64_t i = 0; i < rows; ++i)
    if (ip[i + 1] < ip[i]) return false;
  for (int64_t k = 0; k < nnz; ++k)
    if (ij[k] < 0 || ij[k] >= cols) return false;
  return true;
}

}  // namespace
}  // namespace mlamg

using namespace mlamg;

extern "C" {

int mlamg_amg2v_batch_limits(int64_t* max_rows, int64_t* max_coarse, int* max_row_entries) {
  if (max_rows) *max_rows = kBMaxN;
  if (max_coarse) *max_coarse = kBMaxNc;
  if (max_row_entries) *max_row_entries = kBMaxK;
  return MLAMG_OK;
}

int mlamg_amg2v_batch(mlamg_amg2v_problem* probs, int count, int smoother, int nu_pre,
                      int nu_post, double jacobi_weight, int norm_mode, double tol,
                      int max_iter, void* stream) {
  MLAMG_REQUIRE(count >= 0 && (count == 0 || probs), "invalid problem list");
  MLAMG_REQUIRE(smoother == 0 || smoother == 1, "smoother must be 0 (Gauss-Seidel) or 1 (Jacobi)");
  MLAMG_REQUIRE(norm_mode == 0 || norm_mode == 1, "norm_mode must be 0 (residual) or 1 (x)");
  MLAMG_REQUIRE(nu_pre >= 0 && nu_post >= 0 && max_iter >= 0, "negative count");
  if (count == 0) return MLAMG_OK;
  hipStream_t s = S(stream);
  // ---- host: validation, structure analysis, layout
  struct Plan {
    std::vector<int32_t> ptp, ptr, pts, lev, pkr, pkc, clev;
    std::vector<double> pkv, pkd;
    int K = 0, nlev = 0, panel = 8, cap = 0;
  };
  static const bool timing = std::getenv("MLAMG_BATCH_TIMING") != nullptr;
  std::vector<Plan> plans(count);
  std::vector<BDesc> desc(count);
  Layout lay;
  const int64_t desc_off = lay.take(sizeof(BDesc) * count);
  size_t lds_bytes = 0;
  for (int q = 0; q < count; ++q) {
    mlamg_amg2v_problem& P = probs[q];
    const int64_t n = P.n, nc = P.n_c;
    MLAMG_REQUIRE(n >= 1 && n <= kBMaxN, "problem rows out of range for the batched solver");
    MLAMG_REQUIRE(nc >= 1 && nc <= kBMaxNc && nc <= n, "coarse size out of range");
    MLAMG_REQUIRE(valid_csr(n, n, P.A_nnz, P.A_indptr, P.A_indices) && P.A_data,
                  "A is not a valid n x n CSR");
    MLAMG_REQUIRE(valid_csr(n, nc, P.P_nnz, P.P_indptr, P.P_indices) && P.P_data,
                  "P is not a valid n x n_c CSR");
    MLAMG_REQUIRE(P.b && P.x0 && P.x_out && (max_iter == 0 || P.err_out), "NULL vector");
    Plan& L = plans[q];
    // P^T structure: entries of coarse column j in ascending fine row
    L.ptp.assign(nc + 1, 0);
    for (int64_t k = 0; k < P.P_nnz; ++k) L.ptp[P.P_indices[k] + 1]++;
    for (int64_t j = 0; j < nc; ++j) L.ptp[j + 1] += L.ptp[j];
    L.ptr.resize(P.P_nnz);
    L.pts.resize(P.P_nnz);
    {
      std::vector<int32_t> fill(L.ptp.begin(), L.ptp.end() - 1);
      for (int64_t i = 0; i < n; ++i)
        for (int32_t k = P.P_indptr[i]; k < P.P_indptr[i + 1]; ++k) {
          const int32_t j = P.P_indices[k];
          L.ptr[fill[j]] = (int32_t)i;
          L.pts[fill[j]++] = k;
        }
    }
    if (smoother == 0) {
      // level schedule of the forward sweep (gs.hip): level(i) = 1 + max level(j) over j < i
      // coupled in either direction; rows ascending within a level
      std::vector<int32_t> level(n, 0), req(n, 0);
      int maxoff = 0;
      for (int64_t i = 0; i < n; ++i) {
        int32_t lv = req[i];
        int off = 0;
        for (int32_t k = P.A_indptr[i]; k < P.A_indptr[i + 1]; ++k) {
          const int32_t j = P.A_indices[k];
          if (j < i) lv = std::max(lv, level[j] + 1);
          if (j != i) ++off;
        }
        level[i] = lv;
        maxoff = std::max(maxoff, off);
        for (int32_t k = P.A_indptr[i]; k < P.A_indptr[i + 1]; ++k) {
          const int32_t j = P.A_indices[k];
          if (j > i) req[j] = std::max(req[j], lv + 1);
        }
        L.nlev = std::max(L.nlev, lv + 1);
      }
      if (maxoff > kBMaxK) {
        set_error("amg2v_batch: a row of A has more than 32 off-diagonal entries");
        return MLAMG_EUNSUPPORTED;
      }
      L.K = std::max(maxoff, 1);
      L.lev.assign(L.nlev + 1, 0);
      for (int64_t i = 0; i < n; ++i) L.lev[level[i] + 1]++;
      for (int l = 0; l < L.nlev; ++l) L.lev[l + 1] += L.lev[l];
      L.pkr.resize(n);
      L.pkc.assign((size_t)n * L.K, -1);
      L.pkv.assign((size_t)n * L.K, 0.0);
      L.pkd.assign(n, 0.0);
      std::vector<int32_t> fill(L.lev.begin(), L.lev.end() - 1);
      for (int64_t i = 0; i < n; ++i) {
        const int32_t p = fill[level[i]]++;
        L.pkr[p] = (int32_t)i;
        int s2 = 0;
        for (int32_t k = P.A_indptr[i]; k < P.A_indptr[i + 1]; ++k) {
          if (P.A_indices[k] == i) {
            L.pkd[p] = P.A_data[k];  // the last stored diagonal entry, as the sweep takes it
          } else {
            L.pkc[(size_t)p * L.K + s2] = P.A_indices[k];
            L.pkv[(size_t)p * L.K + s2] = P.A_data[k];
            ++s2;
          }
        }
      }
    }
    // GS staging chunks: runs of consecutive levels with <= cap rows, cap from the LDS left
    // after x (a wider level is swept straight from the arena)
    if (smoother == 0) {
      const size_t per_pos = 12 * (size_t)L.K + 24;
      const size_t room = kBLdsBytes > (size_t)n * 8 + 64 ? kBLdsBytes - (size_t)n * 8 - 64 : 0;
      L.cap = (int)std::min<size_t>(4096, room / per_pos);
      L.clev.push_back(0);
      int l = 0;
      while (l < L.nlev) {
        const int start = l;
        int cnt = 0;
        while (l < L.nlev && (l == start || cnt + (L.lev[l + 1] - L.lev[l]) <= L.cap)) {
          cnt += L.lev[l + 1] - L.lev[l];
          ++l;
        }
        L.clev.push_back(l);
      }
    }
    // panel width: the widest power of two <= 32 whose n_c x b panel (+ column, pivots) fits
    int pb = kBMaxPanel;
    while (pb > 8 && (size_t)nc * (pb + 1) * 8 + (size_t)nc * 4 > kBLdsBytes) pb >>= 1;
    MLAMG_REQUIRE((size_t)nc * (pb + 1) * 8 + (size_t)nc * 4 <= kBLdsBytes, "coarse too large");
    L.panel = pb;
    lds_bytes = std::max(lds_bytes, std::max((size_t)nc * (pb + 1) * 8 + (size_t)nc * 4,
                                             (size_t)n * 8 + (size_t)L.cap * (12 * L.K + 24) + 8));
    BDesc& D = desc[q];
    D.n = (int32_t)n;
    D.nc = (int32_t)nc;
    D.smoother = smoother;
    D.nu_pre = nu_pre;
    D.nu_post = nu_post;
    D.norm_mode = norm_mode;
    D.max_iter = max_iter;
    D.K = L.K;
    D.nlev = L.nlev;
    D.panel = pb;
    D.n_chunks = L.clev.empty() ? 0 : (int32_t)L.clev.size() - 1;
    D.cap = L.cap;
    D.timing = timing ? 1 : 0;
    D.tol = tol;
    D.omega = jacobi_weight;
    D.A_ip = lay.take(4 * (n + 1));
    D.A_ij = lay.take(4 * P.A_nnz);
    D.A_val = lay.take(8 * P.A_nnz);
    D.P_ip = lay.take(4 * (n + 1));
    D.P_ij = lay.take(4 * P.P_nnz);
    D.P_val = lay.take(8 * P.P_nnz);
    D.PT_ptr = lay.take(4 * (nc + 1));
    D.PT_row = lay.take(4 * P.P_nnz);
    D.PT_src = lay.take(4 * P.P_nnz);
    D.lev_ptr = lay.take(4 * (L.lev.size()));
    D.chunk_lev = lay.take(4 * (L.clev.size()));
    D.pk_row = lay.take(4 * L.pkr.size());
    D.pk_col = lay.take(4 * L.pkc.size());
    D.pk_val = lay.take(8 * L.pkv.size());
    D.pk_diag = lay.take(8 * L.pkd.size());
    D.b_lvl = lay.take(8 * L.pkr.size());
    D.b = lay.take(8 * n);
    D.x0 = lay.take(8 * n);
  }
  const size_t in_bytes = lay.off;
  for (int q = 0; q < count; ++q) {
    BDesc& D = desc[q];
    D.AH = lay.take((size_t)8 * D.nc * D.nc);
    D.r = lay.take(8 * (size_t)D.n);
    D.rc = lay.take(8 * (size_t)D.nc);
    D.e = lay.take(8 * (size_t)D.nc);
    D.dinv = lay.take(8 * (size_t)D.n);
  }
  const size_t out_begin = lay.off;
  for (int q = 0; q < count; ++q) {
    BDesc& D = desc[q];
    D.x_out = lay.take(8 * (size_t)D.n);
    D.err_out = lay.take(8 * (size_t)std::max(max_iter, 1));
    D.stat_out = lay.take(8 + 8 * 4);
  }
  const size_t total = lay.off;
  // ---- pack the inputs into pinned host memory, one copy in
  HostPinned& H = g_batch_host;
  const size_t host_need = std::max(in_bytes, total - out_begin);
  if (H.cap < host_need) {
    if (H.p) (void)hipHostFree(H.p);
    H.p = nullptr;
    H.cap = 0;
    MLAMG_HIP(hipHostMalloc(&H.p, host_need, hipHostMallocDefault));
    H.cap = host_need;
  }
  char* hb = static_cast<char*>(H.p);
  std::memcpy(hb + desc_off, desc.data(), sizeof(BDesc) * count);
  for (int q = 0; q < count; ++q) {
    const mlamg_amg2v_problem& P = probs[q];
    const BDesc& D = desc[q];
    const Plan& L = plans[q];
    const int64_t n = P.n;
    std::memcpy(hb + D.A_ip, P.A_indptr, 4 * (n + 1));
    std::memcpy(hb + D.A_ij, P.A_indices, 4 * P.A_nnz);
    std::memcpy(hb + D.A_val, P.A_data, 8 * P.A_nnz);
    std::memcpy(hb + D.P_ip, P.P_indptr, 4 * (n + 1));
    std::memcpy(hb + D.P_ij, P.P_indices, 4 * P.P_nnz);
    std::memcpy(hb + D.P_val, P.P_data, 8 * P.P_nnz);
    std::memcpy(hb + D.PT_ptr, L.ptp.data(), 4 * L.ptp.size());
    std::memcpy(hb + D.PT_row, L.ptr.data(), 4 * L.ptr.size());
    std::memcpy(hb + D.PT_src, L.pts.data(), 4 * L.pts.size());
    if (!L.lev.empty()) std::memcpy(hb + D.lev_ptr, L.lev.data(), 4 * L.lev.size());
    if (!L.clev.empty()) std::memcpy(hb + D.chunk_lev, L.clev.data(), 4 * L.clev.size());
    if (!L.pkr.empty()) {
      std::memcpy(hb + D.pk_row, L.pkr.data(), 4 * L.pkr.size());
      std::memcpy(hb + D.pk_col, L.pkc.data(), 4 * L.pkc.size());
      std::memcpy(hb + D.pk_val, L.pkv.data(), 8 * L.pkv.size());
      std::memcpy(hb + D.pk_diag, L.pkd.data(), 8 * L.pkd.size());
      double* blv = reinterpret_cast<double*>(hb + D.b_lvl);
      for (size_t p = 0; p < L.pkr.size(); ++p) blv[p] = P.b[L.pkr[p]];
    }
    std::memcpy(hb + D.b, P.b, 8 * n);
    std::memcpy(hb + D.x0, P.x0, 8 * n);
  }
  char* arena = static_cast<char*>(scratch(total, 11));
  MLAMG_REQUIRE(arena, "device arena allocation failed");
  MLAMG_HIP(hipMemcpyAsync(arena, hb, in_bytes, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_amg2v_batch, dim3((unsigned)count), dim3(kBT), lds_bytes, s,
                     reinterpret_cast<const BDesc*>(arena + desc_off), arena);
  MLAMG_HIP(hipGetLastError());
  // the host staging buffer is reused for the outputs: the copy-in above completed before the
  // kernel (same stream), and the copy-out below is ordered after it
  MLAMG_HIP(hipMemcpyAsync(hb, arena + out_begin, total - out_begin, hipMemcpyDeviceToHost, s));
  MLAMG_HIP(hipStreamSynchronize(s));
  for (int q = 0; q < count; ++q) {
    mlamg_amg2v_problem& P = probs[q];
    const BDesc& D = desc[q];
    const int32_t* st = reinterpret_cast<const int32_t*>(hb + (D.stat_out - out_begin));
    P.iters_out = st[0];
    P.status_out = st[1];
    if (timing) {
      const int64_t* ts = reinterpret_cast<const int64_t*>(st + 2);
      std::fprintf(stderr,
                   "[amg2v_batch] problem %d n=%lld n_c=%lld iters=%d: galerkin %.3f ms, inverse "
                   "%.3f ms, smoothing %.3f ms, rest of cycles %.3f ms\n",
                   q, (long long)P.n, (long long)P.n_c, st[0], ts[0] * 1e-5, ts[1] * 1e-5,
                   ts[2] * 1e-5, ts[3] * 1e-5);
    }
    std::memcpy(P.x_out, hb + (D.x_out - out_begin), 8 * (size_t)P.n);
    if (max_iter > 0) std::memcpy(P.err_out, hb + (D.err_out - out_begin), 8 * (size_t)st[0]);
  }
  return MLAMG_OK;
}

}  // extern "C"
