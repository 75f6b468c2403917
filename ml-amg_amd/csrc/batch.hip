// The reference's own call pattern, one launch per batch: `amg_2_v(A, P, b, x, ...)`
// (ns/lib/multigrid.py:111-210) on small grids, called once per grid by the training and
// evaluation loops (utils/common.py:77,106, utils/evaluate_dataset.py:96,
// utils/train_dataset.py:114) and farmed out over processes (ns/parallel/pool.py). Launching
// the V-cycle kernels of a 1k-16k-row problem one by one leaves the GPU idle between launches,
// so here ONE workgroup runs one whole problem — Galerkin product, coarse inverse, every cycle
// and the tolerance test — and one launch runs a whole batch, one workgroup per problem.
//
// Per problem (workgroup of 1024 threads; x, and r when it fits, resident in LDS):
//   A_H = P^T A P, dense n_c x n_c                 (multigrid.py:165)
//   A_H^-1 by blocked Gauss-Jordan with partial pivoting: panels of b columns factorised in
//     LDS (the next pivot search fused into each elimination step: 2 barriers per column), the
//     panel's net row permutation then the rank-b update applied to the other columns, columns
//     un-interchanged by one gather pass (replaces spla.factorized, :168; singular -> status 1,
//     the reference's `except: return x, 1., err, 0`)
//   cycles (:172-199): pre-smoothing (pyamg forward Gauss-Seidel over a level schedule, bitwise
//     the sequential sweep; or the MLAMG weighted-Jacobi form x += w D^-1 (b - A x)),
//     r = b - A x, r_H = P^T r (ascending fine row per coarse row: scipy csc_matvec's order),
//     e_H = A_H^-1 r_H (wave per row, lane-strided + butterfly: the order of dense.hip k_gemv),
//     x += P e_H, post-smoothing, err[i] = ||b - A x||_2 or ||x||_2, stop at err[i] <= tol.
// Smoothing, residual, restriction and prolongation are bitwise the reference's sparse ops;
// the Galerkin product and the coarse inverse differ from scipy/SuperLU by rounding only
// (fp64 tolerance, like every dense-coarse path of this library).
//
// A single workgroup is bound by dependent memory round trips and barriers, not bandwidth, so
// every matrix the cycles read is pre-packed into fixed-width slot-major rows (all loads of a
// phase independent: one round trip per phase), the sweep's rows are staged into LDS a chunk of
// levels at a time, and the pivot search of Gauss-Jordan step k+1 rides on step k's barrier.
// Structure-only preparation (level schedule, transposed sparsity of P, packing) is done on the
// host from the CSR index arrays the caller hands over; every floating-point operation runs in
// the kernel.
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
constexpr int64_t kBMaxNc = 2048;   // coarse rows: dense inverse, LDS panels of >= 4 columns
constexpr int kBMaxK = 32;          // off-diagonal entries per row of A
constexpr int kBMaxKP = 32;         // entries per row of P
constexpr int kBMaxKT = 256;        // entries per row of P^T
constexpr int kBMaxPanel = 16;
constexpr size_t kBLdsBytes = 156 * 1024;

struct BDesc {
  int32_t n, nc, smoother, nu_pre, nu_post, norm_mode, max_iter;
  int32_t K, KA, KP, KT, nlev, panel, n_chunks, cap, timing;
  double tol, omega;
  // byte offsets into the arena; packed arrays are slot-major: a[s * rows + row]
  int64_t ak_col, ak_val;                  // A rows, stored order incl. diagonal (KA slots)
  int64_t pp_col, pp_val;                  // P rows (KP slots)
  int64_t pt_row, pt_val;                  // P^T rows: fine rows ascending (KT slots)
  int64_t lev_ptr, chunk_lev, pk_row, pk_col, pk_val, pk_diag, b_lvl;  // sweep, level order
  int64_t b, x0;
  int64_t AH, AI, rg, dinv;                // Galerkin / un-pivoted inverse / r when not in
                                           // LDS / weighted-Jacobi weights
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

// wave argmax of (v, idx), ties to the smaller idx; lane 0 of each wave posts it
__device__ __forceinline__ void wave_argmax_post(double v, int idx, double* redv, int* redi) {
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
}

// after a barrier: the workgroup's argmax from the posted wave results (every thread)
__device__ __forceinline__ void argmax_result(const double* redv, const int* redi, double* bv,
                                              int* bi) {
  double v = redv[0];
  int i = redi[0];
#pragma unroll
  for (int w = 1; w < kBWaves; ++w)
    if (redv[w] > v || (redv[w] == v && redi[w] < i)) {
      v = redv[w];
      i = redi[w];
    }
  *bv = v;
  *bi = i;
}

// sum_k v[k] * src[c[k]] over the slots of one packed row, slot order, from 0.0 (csr_matvec's
// order); col -1 pads end the row. The slots are read 8 at a time with every load of a group
// issued before any is used (a `break` on the pad would make each slot a full round trip).
__device__ __forceinline__ double packed_dot(const int32_t* __restrict__ col,
                                             const double* __restrict__ val, int stride,
                                             int row, int width, const double* src) {
  constexpr int G = 4;
  double y = 0.0;
  for (int k0 = 0; k0 < width; k0 += G) {
    int c[G];
    double v[G], g[G];
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const bool in = k0 + u < width;
      const int at = (k0 + u) * stride + row;  // < 2^31: widths <= 256, rows <= 16384
      c[u] = in ? col[at] : -1;
      v[u] = in ? val[at] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < G; ++u) g[u] = src[c[u] >= 0 ? c[u] : 0];
#pragma unroll
    for (int u = 0; u < G; ++u)
      if (c[u] >= 0) y += v[u] * g[u];
    if (c[G - 1] < 0) break;
  }
  return y;
}

// rows [i0, i1) of column j: M[i][j] = (i in the panel rows ? 0 : M[i][j]) + sum_t pan[i][t] B[t]
// (t ascending, fused multiply-adds: the inverse is a dense-coarse substitute for SuperLU, held
// to a tolerance, not to scipy's roundings), logical row i stored at physical row phys[i].
// 4 rows at a time with independent accumulators; the next 4 rows' loads issued before the
// current 4 are stored.
__device__ __forceinline__ void panel_update(double* AH, const double* pan, int ps,
                                             const int32_t* phys, const double* B, int nc,
                                             int bw, int k0, int j, int i0, int i1) {
  constexpr int U = 4;
  auto load4 = [&](int i, double* m, int* pr) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int ii = min(i + u, i1 - 1);
      pr[u] = phys[ii];
      const double a = AH[(int64_t)pr[u] * nc + j];
      m[u] = (ii >= k0 && ii < k0 + bw) ? 0.0 : a;
    }
  };
  double cur[U], nxt[U];
  int pc[U], pn[U];
  load4(i0, cur, pc);
  for (int i = i0; i < i1; i += U) {
    if (i + U < i1) load4(i + U, nxt, pn);
    const double* p0 = pan + min(i, i1 - 1) * ps;
    const double* p1 = pan + min(i + 1, i1 - 1) * ps;
    const double* p2 = pan + min(i + 2, i1 - 1) * ps;
    const double* p3 = pan + min(i + 3, i1 - 1) * ps;
#pragma unroll
    for (int t = 0; t < kBMaxPanel; ++t) {
      if (t < bw) {
        const double bt = B[t];
        cur[0] = fma(p0[t], bt, cur[0]);
        cur[1] = fma(p1[t], bt, cur[1]);
        cur[2] = fma(p2[t], bt, cur[2]);
        cur[3] = fma(p3[t], bt, cur[3]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u < i1) AH[(int64_t)pc[u] * nc + j] = cur[u];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      cur[u] = nxt[u];
      pc[u] = pn[u];
    }
  }
}

// one workgroup per problem: Galerkin product and coarse inverse
__global__ __launch_bounds__(kBT) void k_amg2v_setup(const BDesc* __restrict__ descs,
                                                     char* __restrict__ arena) {
  extern __shared__ double lds[];
  __shared__ double redv[kBWaves];
  __shared__ int redi[kBWaves];
  const BDesc D = descs[blockIdx.x];
  const int tid = threadIdx.x;
  const int n = D.n, nc = D.nc;
  const double* __restrict__ b = at<double>(arena, D.b);
  double* AH = at<double>(arena, D.AH);
  double* AI = at<double>(arena, D.AI);
  double* x_out = at<double>(arena, D.x_out);
  double* err = at<double>(arena, D.err_out);
  int32_t* stat = at<int32_t>(arena, D.stat_out);
  const int KA = D.KA, KP = D.KP, KT = D.KT;
  const int32_t* __restrict__ akc = at<int32_t>(arena, D.ak_col);
  const double* __restrict__ akv = at<double>(arena, D.ak_val);
  const int32_t* __restrict__ ppc = at<int32_t>(arena, D.pp_col);
  const double* __restrict__ ppv = at<double>(arena, D.pp_val);
  const int32_t* __restrict__ ptc = at<int32_t>(arena, D.pt_row);
  const double* __restrict__ ptv = at<double>(arena, D.pt_val);

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
    for (int q = 0; q < 6; ++q) tstat[q] = 0;

  // ---------------------------------------------------------------- A_H = P^T A P (dense)
  for (int64_t q = tid; q < (int64_t)nc * nc; q += kBT) AH[q] = 0.0;
  __syncthreads();
  for (int j = tid; j < nc; j += kBT) {
    double* row = AH + (int64_t)j * nc;
    for (int t = 0; t < KT; ++t) {
      const int i = ptc[(int64_t)t * nc + j];
      if (i < 0) break;
      const double p = ptv[(int64_t)t * nc + j];
      for (int k = 0; k < KA; ++k) {
        const int c = akc[(int64_t)k * n + i];
        if (c < 0) break;
        const double pa = p * akv[(int64_t)k * n + i];
        for (int m = 0; m < KP; ++m) {
          const int cc = ppc[(int64_t)m * n + c];
          if (cc < 0) break;
          row[cc] += pa * ppv[(int64_t)m * n + c];
        }
      }
    }
  }
  __syncthreads();
  stamp(0);

  // ---------------------------------------------------------------- A_H^-1, blocked Gauss-Jordan
  const int pb = D.panel;           // power of two, 4..16
  const int ps = pb + 1;            // padded LDS row stride (conflict-free column reads)
  int lgpb = 0;
  while ((1 << lgpb) < pb) ++lgpb;
  // Row interchanges are virtual: logical row i lives in physical row phys[i] of AH, so an
  // interchange is a swap of two phys entries; the panel in LDS is indexed by logical row.
  double* pan = lds;                                      // nc x ps
  double* prow = pan + (int64_t)nc * ps;                  // pb
  double* krow = prow + pb;                               // pb
  int32_t* piv = reinterpret_cast<int32_t*>(krow + pb);   // nc
  int32_t* phys = piv + nc;                               // nc
  int32_t* sig = phys + nc;                               // nc
  for (int i = tid; i < nc; i += kBT) phys[i] = i;
  __syncthreads();
  int status = 0;
  const int my_s = tid & (pb - 1), my_r0 = tid >> lgpb, rstep = kBT >> lgpb;
  for (int k0 = 0; k0 < nc && status == 0; k0 += pb) {
    const int bw = min(pb, nc - k0);
    for (int i = my_r0; i < nc; i += rstep)
      if (my_s < bw) pan[i * ps + my_s] = AH[(int64_t)phys[i] * nc + k0 + my_s];
    __syncthreads();
    // pivot search of the panel's first column
    {
      double v = -1.0;
      int vi = INT32_MAX;
      for (int i = k0 + tid; i < nc; i += kBT) {
        const double a = fabs(pan[i * ps]);
        if (a > v) {
          v = a;
          vi = i;
        }
      }
      wave_argmax_post(v, vi, redv, redi);
    }
    __syncthreads();
    for (int t = 0; t < bw; ++t) {
      const int k = k0 + t;
      double bv;
      int p;
      argmax_result(redv, redi, &bv, &p);
      if (!(bv > 0.0)) {  // exactly singular (uniform across the workgroup)
        status = 1;
        break;
      }
      if (tid == 0) piv[k] = p;
      if (tid < bw) {
        prow[tid] = pan[p * ps + tid];
        krow[tid] = pan[k * ps + tid];
      }
      __syncthreads();
      // step t on every panel row (row p takes row k's values: the interchange), and the next
      // column's pivot candidates as they are produced
      const double inv = 1.0 / prow[t];
      double cv = -1.0;
      int ci = INT32_MAX;
      for (int i = my_r0; i < nc; i += rstep) {
        if (my_s >= bw) continue;
        const int s = my_s;
        double nv;
        if (i == k) {
          nv = (s == t) ? inv : prow[s] * inv;
        } else {
          const double src = (i == p) ? krow[s] : pan[i * ps + s];
          const double f = (i == p) ? krow[t] : pan[i * ps + t];
          if (f == 0.0) {
            nv = src;
          } else {
            nv = (s == t) ? -f * inv : src - f * (prow[s] * inv);
          }
        }
        pan[i * ps + s] = nv;
        if (s == t + 1 && i > k) {
          const double a = fabs(nv);
          if (a > cv) {
            cv = a;
            ci = i;
          }
        }
      }
      wave_argmax_post(cv, ci, redv, redi);
      __syncthreads();
    }
    if (status) break;
    stamp(4);
    // the panel's interchanges on the row map (the panel itself was interchanged in LDS)
    if (tid == 0)
      for (int t = 0; t < bw; ++t) {
        const int k = k0 + t, p = piv[k];
        const int tmp = phys[k];
        phys[k] = phys[p];
        phys[p] = tmp;
      }
    __syncthreads();
    // the other columns: M <- T M, T the identity with its panel columns replaced by the
    // factorised panel, B = column j's (interchanged) panel rows
    const int ncol = nc - bw;
    auto load_B = [&](int j, double* B) {
#pragma unroll
      for (int t = 0; t < kBMaxPanel; ++t)
        B[t] = t < bw ? AH[(int64_t)phys[k0 + t] * nc + j] : 0.0;
    };
    if (ncol >= kBT) {  // a thread per column (several each)
      for (int jj = tid; jj < ncol; jj += kBT) {
        const int j = jj < k0 ? jj : jj + bw;
        double B[kBMaxPanel];
        load_B(j, B);
        panel_update(AH, pan, ps, phys, B, nc, bw, k0, j, 0, nc);
      }
    } else if (ncol > 0) {  // fewer columns than threads: each column split into row ranges
      const int parts = max(1, min(kBT / ncol, nc));
      const int chunk = (nc + parts - 1) / parts;
      const int jj = tid % ncol, part = tid / ncol;
      const bool active = part < parts;
      const int j = jj < k0 ? jj : jj + bw;
      double B[kBMaxPanel];
      if (active) load_B(j, B);
      __syncthreads();  // every part has read B before the panel rows are rewritten
      if (active) {
        const int i0 = part * chunk, i1 = min(nc, i0 + chunk);
        if (i0 < i1) panel_update(AH, pan, ps, phys, B, nc, bw, k0, j, i0, i1);
      }
    }
    for (int i = my_r0; i < nc; i += rstep)
      if (my_s < bw) AH[(int64_t)phys[i] * nc + k0 + my_s] = pan[i * ps + my_s];
    __syncthreads();
    stamp(5);
  }
  if (status == 0) {
    // undo the row interchanges as column interchanges (last to first): the final column
    // permutation sigma, then one gather pass AI[i][k] = X[i][sigma[k]], X[i] = AH[phys[i]]
    if (tid == 0) {
      for (int k = 0; k < nc; ++k) sig[k] = k;
      for (int k = nc - 1; k >= 0; --k) {
        const int q = piv[k];
        if (q != k) {
          const int tmp = sig[k];
          sig[k] = sig[q];
          sig[q] = tmp;
        }
      }
    }
    __syncthreads();
    for (int64_t q = tid; q < (int64_t)nc * nc; q += kBT) {
      const int64_t i = q / nc;
      const int k = (int)(q - i * nc);
      AI[q] = AH[(int64_t)phys[i] * nc + sig[k]];
    }
  }
  __syncthreads();
  stamp(1);
  if (tid == 0) stat[1] = status;
}

// one workgroup per problem: the cycles (reads the setup kernel's inverse and status)
template <bool R_LDS>
__global__ __launch_bounds__(kBT) void k_amg2v_cycles(const BDesc* __restrict__ descs,
                                                      char* __restrict__ arena) {
  extern __shared__ double lds[];
  __shared__ double redv[kBWaves];
  const BDesc D = descs[blockIdx.x];
  const int tid = threadIdx.x;
  const int n = D.n, nc = D.nc;
  const double* __restrict__ b = at<double>(arena, D.b);
  const double* __restrict__ AI = at<double>(arena, D.AI);
  double* x_out = at<double>(arena, D.x_out);
  double* err = at<double>(arena, D.err_out);
  int32_t* stat = at<int32_t>(arena, D.stat_out);
  const int KA = D.KA, KP = D.KP, KT = D.KT;
  const int32_t* __restrict__ akc = at<int32_t>(arena, D.ak_col);
  const double* __restrict__ akv = at<double>(arena, D.ak_val);
  const int32_t* __restrict__ ppc = at<int32_t>(arena, D.pp_col);
  const double* __restrict__ ppv = at<double>(arena, D.pp_val);
  const int32_t* __restrict__ ptc = at<int32_t>(arena, D.pt_row);
  const double* __restrict__ ptv = at<double>(arena, D.pt_val);
  int64_t* tstat = at<int64_t>(arena, D.stat_out + 8);
  int64_t t_mark = D.timing ? wall_clock64() : 0;
  auto stamp = [&](int slot) {
    if (D.timing && tid == 0) {
      const int64_t t = wall_clock64();
      tstat[slot] += t - t_mark;
      t_mark = t;
    }
  };
  const int status = stat[1];

  // ---------------------------------------------------------------- cycles
  double* xs = lds;                                     // n
  double* rcs = xs + n;                                 // nc: restricted residual
  double* es = rcs + nc;                                // nc: coarse correction
  double* rs = R_LDS ? es + nc : at<double>(arena, D.rg);  // n: residual
  double* stage = R_LDS ? rs + n : es + nc;             // GS staging area
  const double* __restrict__ x0 = at<double>(arena, D.x0);
  #pragma unroll 1
  for (int i = tid; i < n; i += kBT) xs[i] = x0[i];
  __syncthreads();
  if (status != 0) {  // multigrid.py:167-170: x returned untouched, no iteration
    #pragma unroll 1
    for (int i = tid; i < n; i += kBT) x_out[i] = xs[i];
    if (tid == 0) stat[0] = 0;
    return;
  }
  // weighted-Jacobi weights (1/a_ii) * w, a_ii = the sum of the stored diagonal entries
  // (csr_diagonal)
  double* dwg = at<double>(arena, D.dinv);
  if (D.smoother == 1) {
    #pragma unroll 1
    for (int i = tid; i < n; i += kBT) {
      double d = 0.0;
      for (int k = 0; k < KA; ++k) {
        const int c = akc[(int64_t)k * n + i];
        if (c < 0) break;
        if (c == i) d += akv[(int64_t)k * n + i];
      }
      dwg[i] = (1.0 / d) * D.omega;
    }
  }

  // (b - A x)_i in csr_matvec's order (0 + a_1 x_1 + ... in stored order, then b_i - y)
  auto resid_row = [&](int i) -> double { return b[i] - packed_dot(akc, akv, n, i, KA, xs); };

  const int32_t* __restrict__ lptr = at<int32_t>(arena, D.lev_ptr);
  const int32_t* __restrict__ clev = at<int32_t>(arena, D.chunk_lev);
  const int32_t* __restrict__ pkr = at<int32_t>(arena, D.pk_row);
  const int32_t* __restrict__ pkc = at<int32_t>(arena, D.pk_col);
  const double* __restrict__ pkv = at<double>(arena, D.pk_val);
  const double* __restrict__ pkd = at<double>(arena, D.pk_diag);
  const double* __restrict__ bl = at<double>(arena, D.b_lvl);
  const int K = D.K, cap = D.cap;
  // staging of a chunk of levels (slot-major like the arena copy: bank-conflict free)
  double* sv = stage;                                       // cap*K values
  double* sd = sv + (int64_t)cap * K;                       // cap diagonals
  double* sb = sd + cap;                                    // cap right-hand sides
  int32_t* sc = reinterpret_cast<int32_t*>(sb + cap);       // cap*K columns
  int32_t* sr = sc + (int64_t)cap * K;                      // cap rows
  int32_t* slp = sr + cap;                                  // level starts of the chunk

  auto gs_sweep = [&]() {
    // pyamg gauss_seidel: rsum over the off-diagonals in stored order, diag = the last stored
    // diagonal entry, x_i = (b_i - rsum) / diag unless diag == 0
    for (int ch = 0; ch < D.n_chunks; ++ch) {
      const int l0 = clev[ch], l1 = clev[ch + 1];
      const int P0 = lptr[l0], cnt = lptr[l1] - P0;
      if (cnt <= cap) {
        for (int s2 = 0; s2 < K; ++s2)
          for (int q = tid; q < cnt; q += kBT) {
            sc[s2 * cap + q] = pkc[(int64_t)s2 * n + P0 + q];
            sv[s2 * cap + q] = pkv[(int64_t)s2 * n + P0 + q];
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
          #pragma unroll 1
          for (int p = a + tid; p < z; p += kBT) {
            const double rsum = packed_dot(sc, sv, cap, p, K, xs);
            const double dg = sd[p];
            if (dg != 0.0) xs[sr[p]] = (sb[p] - rsum) / dg;
          }
          __syncthreads();
        }
      } else {  // one level wider than the staging area: straight from the arena
        for (int l = l0; l < l1; ++l) {
          const int a = lptr[l], z = lptr[l + 1];
          #pragma unroll 1
          for (int p = a + tid; p < z; p += kBT) {
            const double rsum = packed_dot(pkc, pkv, n, p, K, xs);
            const double dg = pkd[p];
            if (dg != 0.0) xs[pkr[p]] = (bl[p] - rsum) / dg;
          }
          __syncthreads();
        }
      }
    }
  };

  auto smooth = [&](int nu) {
    stamp(3);
    for (int it = 0; it < nu; ++it) {
      if (D.smoother == 0) {
        gs_sweep();
      } else {  // MLAMG.py:143-146: x += Dinv_w (b - A x)
        #pragma unroll 1
        for (int i = tid; i < n; i += kBT) rs[i] = resid_row(i);
        __syncthreads();
        #pragma unroll 1
        for (int i = tid; i < n; i += kBT) xs[i] = xs[i] + dwg[i] * rs[i];
        __syncthreads();
      }
    }
    stamp(2);
  };

  int iters = 0;
  for (int itn = 0; itn < D.max_iter; ++itn) {
    smooth(D.nu_pre);
    #pragma unroll 1
    for (int i = tid; i < n; i += kBT) rs[i] = resid_row(i);
    __syncthreads();
    #pragma unroll 1
    for (int j = tid; j < nc; j += kBT)  // P^T r: csc_matvec's order
      rcs[j] = packed_dot(ptc, ptv, nc, j, KT, rs);
    __syncthreads();
    {  // e = A_H^-1 r_H: wave per row, k_gemv's order
      const int w = tid >> 6, lane = tid & 63;
      #pragma unroll 1
      for (int j = w; j < nc; j += kBWaves) {
        const double* rw = AI + (int64_t)j * nc;
        double s = 0.0;
        int l = lane;
        for (; l + 7 * 64 < nc; l += 8 * 64) {
          double m[8], v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            m[u] = rw[l + u * 64];
            v[u] = rcs[l + u * 64];
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) s += m[u] * v[u];
        }
        for (; l < nc; l += 64) s += rw[l] * rcs[l];
        s = bw_sum(s);
        if (lane == 0) es[j] = s;
      }
    }
    __syncthreads();
    #pragma unroll 1
    for (int i = tid; i < n; i += kBT)  // x += P e
      xs[i] = xs[i] + packed_dot(ppc, ppv, n, i, KP, es);
    __syncthreads();
    smooth(D.nu_post);
    double part = 0.0;
    if (D.norm_mode == 0) {
      #pragma unroll 1
      for (int i = tid; i < n; i += kBT) {
        const double ri = resid_row(i);
        part += ri * ri;
      }
    } else {
      #pragma unroll 1
      for (int i = tid; i < n; i += kBT) part += xs[i] * xs[i];
    }
    const double nrm = sqrt(block_sum(part, redv));
    if (tid == 0) err[itn] = nrm;
    iters = itn + 1;
    if (D.tol >= 0.0 && nrm <= D.tol) break;
  }
  #pragma unroll 1
  for (int i = tid; i < n; i += kBT) x_out[i] = xs[i];
  stamp(3);
  if (tid == 0) stat[0] = iters;
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

// rows of a CSR into a slot-major fixed-width layout (col -1 / value 0 pads); width = the
// longest row (>= 1)
int pack_rows(int64_t rows, const int32_t* ip, const int32_t* ij, const double* v,
              std::vector<int32_t>& col, std::vector<double>& val) {
  int w = 1;
  for (int64_t i = 0; i < rows; ++i) w = std::max(w, ip[i + 1] - ip[i]);
  col.assign((size_t)w * rows, -1);
  val.assign((size_t)w * rows, 0.0);
  for (int64_t i = 0; i < rows; ++i)
    for (int32_t k = ip[i]; k < ip[i + 1]; ++k) {
      col[(size_t)(k - ip[i]) * rows + i] = ij[k];
      val[(size_t)(k - ip[i]) * rows + i] = v[k];
    }
  return w;
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
    std::vector<int32_t> lev, pkr, pkc, clev, akc, ppc, ptc;
    std::vector<double> pkv, pkd, akv, ppv, ptv;
    int K = 1, KA = 1, KP = 1, KT = 1, nlev = 0, panel = 8, cap = 0;
  };
  static const bool timing = std::getenv("MLAMG_BATCH_TIMING") != nullptr;
  std::vector<Plan> plans(count);
  std::vector<BDesc> desc(count);
  // residual in LDS when every problem leaves room for it
  bool r_lds = true;
  for (int q = 0; q < count; ++q) {
    const size_t need = (size_t)probs[q].n * 16 + (size_t)probs[q].n_c * 16 + 16 * 1024;
    if (need > kBLdsBytes) r_lds = false;
  }
  Layout lay;
  const int64_t desc_off = lay.take(sizeof(BDesc) * count);
  size_t lds_setup = 0, lds_cycles = 0;
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
    L.KA = pack_rows(n, P.A_indptr, P.A_indices, P.A_data, L.akc, L.akv);
    L.KP = pack_rows(n, P.P_indptr, P.P_indices, P.P_data, L.ppc, L.ppv);
    {  // P^T: entries of coarse column j in ascending fine row
      std::vector<int32_t> tp(nc + 1, 0);
      for (int64_t k = 0; k < P.P_nnz; ++k) tp[P.P_indices[k] + 1]++;
      for (int64_t j = 0; j < nc; ++j) tp[j + 1] += tp[j];
      std::vector<int32_t> ti(P.P_nnz);
      std::vector<double> tv(P.P_nnz);
      std::vector<int32_t> fill(tp.begin(), tp.end() - 1);
      for (int64_t i = 0; i < n; ++i)
        for (int32_t k = P.P_indptr[i]; k < P.P_indptr[i + 1]; ++k) {
          const int32_t j = P.P_indices[k];
          ti[fill[j]] = (int32_t)i;
          tv[fill[j]++] = P.P_data[k];
        }
      L.KT = pack_rows(nc, tp.data(), ti.data(), tv.data(), L.ptc, L.ptv);
    }
    if (L.KA > kBMaxK + 1 || L.KP > kBMaxKP || L.KT > kBMaxKT) {
      set_error("amg2v_batch: rows of A, P or P^T longer than the batched solver's slots");
      return MLAMG_EUNSUPPORTED;
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
            L.pkc[(size_t)s2 * n + p] = P.A_indices[k];
            L.pkv[(size_t)s2 * n + p] = P.A_data[k];
            ++s2;
          }
        }
      }
    }
    // panel width: the widest power of two <= 16 whose n_c x (b+1) panel (+ pivots and the
    // final column permutation) fits
    int pb = kBMaxPanel;
    auto setup_lds = [&](int b) { return (size_t)nc * (b + 1) * 8 + 16 * b + (size_t)nc * 12; };
    while (pb > 4 && setup_lds(pb) > kBLdsBytes) pb >>= 1;
    MLAMG_REQUIRE(setup_lds(pb) <= kBLdsBytes, "coarse too large");
    L.panel = pb;
    // GS staging chunks: runs of consecutive levels with <= cap rows, cap from the LDS left
    // after the cycle vectors (a wider level is swept straight from the arena)
    const size_t vec_lds = (size_t)n * 8 * (r_lds ? 2 : 1) + (size_t)nc * 16;
    if (smoother == 0) {
      const size_t per_pos = 12 * (size_t)L.K + 24;
      const size_t room = kBLdsBytes > vec_lds + 64 ? kBLdsBytes - vec_lds - 64 : 0;
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
    lds_setup = std::max(lds_setup, setup_lds(pb));
    lds_cycles = std::max(lds_cycles, vec_lds + (size_t)L.cap * (12 * L.K + 24) + 8);
    BDesc& D = desc[q];
    std::memset(&D, 0, sizeof(D));
    D.n = (int32_t)n;
    D.nc = (int32_t)nc;
    D.smoother = smoother;
    D.nu_pre = nu_pre;
    D.nu_post = nu_post;
    D.norm_mode = norm_mode;
    D.max_iter = max_iter;
    D.K = L.K;
    D.KA = L.KA;
    D.KP = L.KP;
    D.KT = L.KT;
    D.nlev = L.nlev;
    D.panel = pb;
    D.n_chunks = L.clev.empty() ? 0 : (int32_t)L.clev.size() - 1;
    D.cap = L.cap;
    D.timing = timing ? 1 : 0;
    D.tol = tol;
    D.omega = jacobi_weight;
    D.ak_col = lay.take(4 * L.akc.size());
    D.ak_val = lay.take(8 * L.akv.size());
    D.pp_col = lay.take(4 * L.ppc.size());
    D.pp_val = lay.take(8 * L.ppv.size());
    D.pt_row = lay.take(4 * L.ptc.size());
    D.pt_val = lay.take(8 * L.ptv.size());
    D.lev_ptr = lay.take(4 * L.lev.size());
    D.chunk_lev = lay.take(4 * L.clev.size());
    D.pk_row = lay.take(4 * L.pkr.size());
    D.pk_col = lay.take(4 * L.pkc.size());
    D.pk_val = lay.take(8 * L.pkv.size());
    D.pk_diag = lay.take(8 * L.pkd.size());
    D.b_lvl = lay.take(8 * L.pkr.size());
    D.b = lay.take(8 * n);
    D.x0 = lay.take(8 * n);
  }
  MLAMG_REQUIRE(lds_setup <= kBLdsBytes + 1024 && lds_cycles <= kBLdsBytes + 1024,
                "LDS budget exceeded");
  const size_t in_bytes = lay.off;
  for (int q = 0; q < count; ++q) {
    BDesc& D = desc[q];
    D.AH = lay.take((size_t)8 * D.nc * D.nc);
    D.AI = lay.take((size_t)8 * D.nc * D.nc);
    D.rg = lay.take(8 * (size_t)D.n);
    D.dinv = lay.take(8 * (size_t)D.n);
  }
  const size_t out_begin = lay.off;
  for (int q = 0; q < count; ++q) {
    BDesc& D = desc[q];
    D.x_out = lay.take(8 * (size_t)D.n);
    D.err_out = lay.take(8 * (size_t)std::max(max_iter, 1));
    D.stat_out = lay.take(8 + 8 * 6);
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
  auto put = [&](int64_t off, const void* src, size_t bytes) {
    if (bytes) std::memcpy(hb + off, src, bytes);
  };
  for (int q = 0; q < count; ++q) {
    const mlamg_amg2v_problem& P = probs[q];
    const BDesc& D = desc[q];
    const Plan& L = plans[q];
    const int64_t n = P.n;
    put(D.ak_col, L.akc.data(), 4 * L.akc.size());
    put(D.ak_val, L.akv.data(), 8 * L.akv.size());
    put(D.pp_col, L.ppc.data(), 4 * L.ppc.size());
    put(D.pp_val, L.ppv.data(), 8 * L.ppv.size());
    put(D.pt_row, L.ptc.data(), 4 * L.ptc.size());
    put(D.pt_val, L.ptv.data(), 8 * L.ptv.size());
    put(D.lev_ptr, L.lev.data(), 4 * L.lev.size());
    put(D.chunk_lev, L.clev.data(), 4 * L.clev.size());
    put(D.pk_row, L.pkr.data(), 4 * L.pkr.size());
    put(D.pk_col, L.pkc.data(), 4 * L.pkc.size());
    put(D.pk_val, L.pkv.data(), 8 * L.pkv.size());
    put(D.pk_diag, L.pkd.data(), 8 * L.pkd.size());
    if (!L.pkr.empty()) {
      double* blv = reinterpret_cast<double*>(hb + D.b_lvl);
      for (size_t p = 0; p < L.pkr.size(); ++p) blv[p] = P.b[L.pkr[p]];
    }
    put(D.b, P.b, 8 * n);
    put(D.x0, P.x0, 8 * n);
  }
  char* arena = static_cast<char*>(scratch(total, 11));
  MLAMG_REQUIRE(arena, "device arena allocation failed");
  MLAMG_HIP(hipMemcpyAsync(arena, hb, in_bytes, hipMemcpyHostToDevice, s));
  const BDesc* dd = reinterpret_cast<const BDesc*>(arena + desc_off);
  hipLaunchKernelGGL(k_amg2v_setup, dim3((unsigned)count), dim3(kBT), lds_setup, s, dd, arena);
  if (r_lds)
    hipLaunchKernelGGL(k_amg2v_cycles<true>, dim3((unsigned)count), dim3(kBT), lds_cycles, s,
                       dd, arena);
  else
    hipLaunchKernelGGL(k_amg2v_cycles<false>, dim3((unsigned)count), dim3(kBT), lds_cycles, s,
                       dd, arena);
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
                   "%.3f ms (panels %.3f, updates %.3f), smoothing %.3f ms, rest of cycles "
                   "%.3f ms\n",
                   q, (long long)P.n, (long long)P.n_c, st[0], ts[0] * 1e-5,
                   (ts[1] + ts[4] + ts[5]) * 1e-5, ts[4] * 1e-5, ts[5] * 1e-5, ts[2] * 1e-5,
                   ts[3] * 1e-5);
    }
    std::memcpy(P.x_out, hb + (D.x_out - out_begin), 8 * (size_t)P.n);
    if (max_iter > 0) std::memcpy(P.err_out, hb + (D.err_out - out_begin), 8 * (size_t)st[0]);
  }
  return MLAMG_OK;
}

}  // extern "C"
