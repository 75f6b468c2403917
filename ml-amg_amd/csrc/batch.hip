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

#include <sched.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <type_traits>
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
#ifndef MLAMG_GS_SCHED_FENCE  // build-time A/B knob: scheduling barrier after a level's stores
#define MLAMG_GS_SCHED_FENCE 1
#endif
constexpr int kExtCoarseMin = 300;  // single calls above this n_c: device-wide coarse factor
constexpr size_t kBLdsBytes = 156 * 1024;

struct BDesc {
  int32_t n, nc, smoother, nu_pre, nu_post, norm_mode, max_iter;
  int32_t K, KA, KP, KT, nlev, panel, n_chunks, cap, timing;
  int32_t spd;    // A symmetric: try the inverse Cholesky factor before Gauss-Jordan
  int32_t chol_nb;  // its panel width (4..16, from n_c)
  int32_t setup_mode;  // 0: Galerkin + coarse inverse here; 1: neither (k_galerkin_rows and the
                       // device-wide factorisation of dense.hip); 2: Galerkin only (the batched
                       // device-wide factorisation follows); 3: nothing (a relaunch's bystander)
  int32_t gs_rw;  // one-wave sweep (rows of K = 4 or 8 slots, levels <= 64 * gs_rw rows), 1 or 2
                  // rows per lane; 0: the workgroup sweeps each level
  int32_t gs_db;   // one-wave sweep: double-buffered chunk staging (chunks of >= 3 levels)
  int32_t gs_rp;   // one-wave sweep, one buffer: the next chunk prefetched into registers
  int32_t phased;  // single large problem: each cycle is two launches, the workgroup's half
                   // cycles and the coarse solve on every CU (k_amg2v_coarse); r_H, e_H global
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
  int64_t rcg, eg, yg;  // phased: r_H, e_H and L^-1 r_H in the arena
  int64_t done_ctr;     // phased: problems finished (one counter for the launch)
  // the problem's values as the caller stores them (A.data, P.data) and its shape's gather maps
  // (shared by every problem with the same sparsity): the packed value arrays above are
  // gathered from them on the device (gather_values), so only the caller's values travel
  int64_t a_raw, p_raw;
  int64_t a_map, p_map, t_map, g_map, d_map, pk_row0;
  // banded coarse solve (band_ld = half-bandwidth + 1, 0: dense): the factor in the band
  // solve's lane layouts F (forward) and G (backward), reciprocal diagonal
  int32_t band_ld, pad0;
  int64_t lc, lr, rinv;
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

// packed_dot for R rows at once (rows[u] < 0: no row): every row's loads of a slot group are
// issued before any gather, so R rows cost the round trips of one; each row sums in slot order
template <int R>
__device__ __forceinline__ void packed_dot_rows(const int32_t* __restrict__ col,
                                                const double* __restrict__ val, int stride,
                                                const int* rows, int width, const double* src,
                                                double* y) {
  constexpr int G = R >= 4 ? 2 : 4;  // R * G slots in flight: registers stay below 128
#pragma unroll
  for (int u = 0; u < R; ++u) y[u] = 0.0;
  for (int k0 = 0; k0 < width; k0 += G) {
    int c[R][G];
    double v[R][G], g[R][G];
#pragma unroll
    for (int u = 0; u < R; ++u)
#pragma unroll
      for (int q = 0; q < G; ++q) {
        const bool in = rows[u] >= 0 && k0 + q < width;
        const int at = (k0 + q) * stride + (rows[u] >= 0 ? rows[u] : 0);
        c[u][q] = in ? col[at] : -1;
        v[u][q] = in ? val[at] : 0.0;
      }
#pragma unroll
    for (int u = 0; u < R; ++u)
#pragma unroll
      for (int q = 0; q < G; ++q) g[u][q] = src[c[u][q] >= 0 ? c[u][q] : 0];
    bool more = false;
#pragma unroll
    for (int u = 0; u < R; ++u) {
#pragma unroll
      for (int q = 0; q < G; ++q)
        if (c[u][q] >= 0) y[u] += v[u][q] * g[u][q];
      more |= c[u][G - 1] >= 0;
    }
    if (!more) break;
  }
}

// out[j] = sum over the row's span of M[j][k] v[k]: a wave takes four rows at a time (rows
// w, w + 16, w + 32, w + 48 of its group) and streams them in 64-column chunks at absolute
// positions k = o + lane, four chunks per pass (16 matrix loads per lane in flight, the vector
// loads shared by the four rows); lane partial sums in chunk order, then a butterfly (fixed
// order). SPAN 0: [0, nc) (the Gauss-Jordan inverse), 1: [0, j] (L^-1, lower), 2: [j, nc)
// (L^-T, upper).
template <int SPAN>
__device__ __forceinline__ void rows_dot(const double* __restrict__ M, int nc,
                                         const double* v, double* out, int tid) {
  constexpr int R = 4, U = 4;
  const int w = tid >> 6, lane = tid & 63;
  for (int j0 = w; j0 < nc; j0 += R * kBWaves) {
    int lo[R], hi[R];
    const double* rp[R];
    int omin = nc, omax = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int j = j0 + r * kBWaves;
      const bool ok = j < nc;
      lo[r] = ok ? (SPAN == 2 ? j : 0) : 0;
      hi[r] = ok ? (SPAN == 1 ? j + 1 : nc) : 0;
      rp[r] = M + (int64_t)(ok ? j : j0) * nc;
      if (ok) {
        omin = min(omin, lo[r]);
        omax = max(omax, hi[r]);
      }
    }
    double sum[R];
#pragma unroll
    for (int r = 0; r < R; ++r) sum[r] = 0.0;
    for (int o = omin & ~63; o < omax; o += U * 64) {
      double m[R][U], x[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = o + u * 64 + lane;
        x[u] = k < nc ? v[k] : 0.0;
#pragma unroll
        for (int r = 0; r < R; ++r) m[r][u] = (k >= lo[r] && k < hi[r]) ? rp[r][k] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < R; ++r) sum[r] = fma(m[r][u], x[u], sum[r]);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const double t = bw_sum(sum[r]);
      const int j = j0 + r * kBWaves;
      if (lane == 0 && j < nc) out[j] = t;
    }
  }
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

// In-place inverse Cholesky factor of an SPD matrix: M (nc x nc, row-major, lower triangle read)
// becomes L^-1 (lower triangle; the upper triangle is left as scratch), A = L L^T. Right-looking
// blocked elimination of [A | I] by NB-column panels: per panel the diagonal block is factorised
// (L11) in LDS, L21 = A21 L11^-T and the panel's final rows Z = L11^-1 [X_top | I] are formed by
// triangular solves, then every trailing row i takes
//   M[i, 0:k1]  <- [X_i, 0] - L21_i Z          (the rows of L^-1 being accumulated)
//   M[i, k1:i]  <- M[i, k1:i] - L21_i L21^T     (the Schur complement, lower triangle)
// in 16x16 fp64 MFMA tiles over LDS operands: nc^3/3 multiply-adds, no pivoting. Returns
// false (uniformly) on a non-positive pivot: the caller falls back to Gauss-Jordan.
typedef double mfma_d4 __attribute__((ext_vector_type(4)));

template <int NB, class Stamp>
__device__ bool chol_inverse(double* __restrict__ M, int nc, double* lds, int tid, Stamp stamp) {
  constexpr int ds = NB + 1;
  double* Dg = lds;                           // NB x ds: diagonal block -> L11
  double* Li = Dg + NB * ds;                  // NB: 1 / diag(L11)
  double* P21 = Li + NB * ds;                 // (nc - k1) x ds: A21 -> L21
  double* Z = P21 + (int64_t)nc * ds;         // NB x nc: the panel's rows of L^-1
  __shared__ int fail;
  const int lane = tid & 63;
  auto wave_sync = [] {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  for (int k0 = 0; k0 < nc; k0 += NB) {
    const int bw = min(NB, nc - k0), k1 = k0 + bw;
    if (tid < 64) {
      // wave 0: the diagonal block, factorised (right-looking, wave-synchronous steps) with its
      // reciprocal diagonal, while the other waves stage the panel below it and [X_top | I]
      for (int q = lane; q < NB * NB; q += 64) {
        const int rr = q / NB, cc = q % NB;
        Dg[rr * ds + cc] = (rr < bw && cc <= rr) ? M[(int64_t)(k0 + rr) * nc + k0 + cc] : 0.0;
      }
      wave_sync();
      // each lane owns entries q = lane + 64 e of the block; a step reads its column-t
      // factors, then (after every lane has read) writes the step's new values
      constexpr int E = (NB * NB + 63) / 64;
      bool ok = true;
      for (int t = 0; t < bw; ++t) {
        const double dtt = Dg[t * ds + t];
        if (!(dtt > 0.0)) {  // same value in every lane
          ok = false;
          break;
        }
        const double sq = sqrt(dtt);
        double nv[E];
        bool wr[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const int q = lane + 64 * e, rr = q / NB, cc = q % NB;
          wr[e] = q < NB * NB && rr < bw && cc <= rr && cc >= t;
          nv[e] = 0.0;
          if (wr[e]) {
            if (cc == t)
              nv[e] = rr == t ? sq : Dg[rr * ds + t] / sq;
            else
              nv[e] = Dg[rr * ds + cc] - (Dg[rr * ds + t] / sq) * (Dg[cc * ds + t] / sq);
          }
        }
        wave_sync();
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const int q = lane + 64 * e;
          if (wr[e]) Dg[(q / NB) * ds + q % NB] = nv[e];
        }
        wave_sync();
      }
      if (ok && lane < bw) Li[lane] = 1.0 / Dg[lane * ds + lane];  // reciprocal diagonal
      if (lane == 0) fail = ok ? 0 : 1;
    } else {
      // A21 (rows below the panel; bw == NB whenever such rows exist) and X_top into LDS
      const int t2 = tid - 64, nt2 = kBT - 64;
      for (int64_t q = t2; q < (int64_t)(nc - k1) * NB; q += nt2) {
        const int i = (int)(q / NB), s = (int)(q % NB);
        P21[(int64_t)i * ds + s] = M[(int64_t)(k1 + i) * nc + k0 + s];
      }
      for (int64_t q = t2; q < (int64_t)bw * k0; q += nt2) {
        const int t = (int)(q / k0), j = (int)(q % k0);
        Z[(int64_t)t * nc + j] = M[(int64_t)(k0 + t) * nc + j];
      }
      for (int q = t2; q < bw * bw; q += nt2) {  // [X_top | I]: the identity columns
        const int t = q / bw, jj = q % bw;
        Z[(int64_t)t * nc + k0 + jj] = t == jj ? 1.0 : 0.0;
      }
    }
    __syncthreads();
    if (fail) return false;  // uniform
    stamp(4);
    // L21 = A21 L11^-T and Z = L11^-1 [X_top | I] by triangular solves with L11, a row of L21
    // or a column of Z per thread, in place (entry t needs only entries s < t): the identity
    // columns make Z's last bw columns L11^-1
    for (int i = tid; i < nc - k1; i += kBT) {
      double* row = P21 + (int64_t)i * ds;
      for (int t = 0; t < NB; ++t) {
        double l = row[t];
        for (int s = 0; s < t; ++s) l = fma(-row[s], Dg[t * ds + s], l);
        row[t] = l * Li[t];
      }
    }
    for (int j = tid; j < k1; j += kBT) {
      for (int t = 0; t < bw; ++t) {
        double z = Z[(int64_t)t * nc + j];
        for (int s = 0; s < t; ++s) z = fma(-Dg[t * ds + s], Z[(int64_t)s * nc + j], z);
        z *= Li[t];
        Z[(int64_t)t * nc + j] = z;
        M[(int64_t)(k0 + t) * nc + j] = z;
      }
    }
    __syncthreads();
    if (k1 < nc) {
      // 16 x 16 tiles over rows [k1, nc) x columns [0, i], a wave per tile, on the fp64 matrix
      // cores: D = C + (-L21 rows) x W, W = Z (columns < k1) or L21^T (columns >= k1), NB/4
      // v_mfma_f64_16x16x4 steps. Lane l supplies A[row l&15][k l>>4] and B[k l>>4][col l&15]
      // and holds D[row (l>>4) + 4 r][col l&15]. Row block rb has a16 + rb + 1 column blocks,
      // C(rb) tiles precede it; a tile may straddle k0 or k1 (sources are picked per element).
      const int w = tid >> 6, lr = lane & 15, lk = lane >> 4;
      const int64_t a16 = (k1 + 15) / 16, nrb = (nc - k1 + 15) / 16;
      auto C = [&](int64_t rb) { return rb * (a16 + 1) + rb * (rb - 1) / 2; };
      const int64_t T = C(nrb);
      const int last = nc - k1 - 1;
      auto coords = [&](int64_t q, int& i0, int& j0) {
        const double bq = (double)a16 + 0.5;
        int64_t rb = (int64_t)(-bq + sqrt(bq * bq + 2.0 * (double)q));
        while (rb > 0 && C(rb) > q) --rb;
        while (C(rb + 1) <= q) ++rb;
        i0 = k1 + 16 * (int)rb;
        j0 = 16 * (int)(q - C(rb));
      };
      auto load_c = [&](int i0, int j0, mfma_d4& acc) {
        const int jc = j0 + lr;
        const bool zero = jc >= k0 && jc < k1;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = i0 + lk + 4 * r;
          acc[r] = (!zero && i < nc && jc < nc) ? M[(int64_t)i * nc + jc] : 0.0;
        }
      };
      // the next tile's C is loaded before this tile's MFMAs (its global round trip overlaps)
      int i0 = 0, j0 = 0;
      mfma_d4 acc;
      if (w < T) {
        coords(w, i0, j0);
        load_c(i0, j0, acc);
      }
      for (int64_t q = w; q < T; q += kBWaves) {
        int i0n = i0, j0n = j0;
        mfma_d4 accn = acc;
        if (q + kBWaves < T) {
          coords(q + kBWaves, i0n, j0n);
          load_c(i0n, j0n, accn);
        }
        const int jc = j0 + lr;  // this lane's output column
        const double* arow = P21 + (int64_t)min(i0 + lr - k1, last) * ds;
        const bool from_z = jc < k1;
        const double* brow = P21 + (int64_t)min(max(jc - k1, 0), last) * ds;
        const int jz = min(jc, k1 - 1);
#pragma unroll
        for (int kk = 0; kk < NB; kk += 4) {
          const int k = kk + lk;
          const double av = -arow[k];
          const double bv = from_z ? Z[(int64_t)k * nc + jz] : brow[k];
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = i0 + lk + 4 * r;
          if (i < nc && jc < nc) M[(int64_t)i * nc + jc] = acc[r];
        }
        i0 = i0n;
        j0 = j0n;
        acc = accn;
      }
      __syncthreads();
    }
    stamp(5);
  }
  return true;
}

// The packed value arrays of one problem from its raw CSR values and its shape's maps (index
// into A.data / P.data, -1 = pad -> 0.0): exactly the values the host packing used to store.
// Four independent map loads per thread before their gathers. The sweep's diagonal and row
// order are value dependent: a zero diagonal under the one-wave sweep writes the sink slot.
__device__ void gather_values(const BDesc& D, char* arena, int tid) {
  const double* __restrict__ av = at<double>(arena, D.a_raw);
  const double* __restrict__ pv = at<double>(arena, D.p_raw);
  auto gather = [&](int64_t map_off, int64_t out_off, int64_t cnt, const double* __restrict__ src) {
    const int32_t* __restrict__ m = at<int32_t>(arena, map_off);
    double* __restrict__ o = at<double>(arena, out_off);
    #pragma unroll 1
    for (int64_t q0 = tid; q0 < cnt; q0 += 4 * kBT) {
      int32_t k[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) k[u] = q0 + u * kBT < cnt ? m[q0 + u * kBT] : -1;
      double v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = k[u] >= 0 ? src[k[u]] : 0.0;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (q0 + u * kBT < cnt) o[q0 + u * kBT] = v[u];
    }
  };
  gather(D.a_map, D.ak_val, (int64_t)D.KA * D.n, av);
  gather(D.p_map, D.pp_val, (int64_t)D.KP * D.n, pv);
  gather(D.t_map, D.pt_val, (int64_t)D.KT * D.nc, pv);
  if (D.smoother == 0) {
    gather(D.g_map, D.pk_val, (int64_t)D.K * D.n, av);
    const int32_t* __restrict__ dm = at<int32_t>(arena, D.d_map);
    const int32_t* __restrict__ r0 = at<int32_t>(arena, D.pk_row0);
    const double* __restrict__ b = at<double>(arena, D.b);
    double* __restrict__ pkd = at<double>(arena, D.pk_diag);
    double* __restrict__ bl = at<double>(arena, D.b_lvl);
    int32_t* __restrict__ pkr = at<int32_t>(arena, D.pk_row);
    #pragma unroll 1
    for (int p = tid; p < D.n; p += kBT) {
      const int32_t k = dm[p], r = r0[p];
      double d = k >= 0 ? av[k] : 0.0;  // the last stored diagonal entry, as the sweep takes it
      bl[p] = b[r];
      int32_t row = r;
      if (D.gs_rw && d == 0.0) {  // pyamg leaves x_i alone: write the sink slot
        d = 1.0;
        row = D.n + 1;
      }
      pkd[p] = d;
      pkr[p] = row;
    }
  }
  __syncthreads();
}

// ---------------------------------------------------------------- banded coarse operators
// The coarse operators of the reference's grids are narrow-banded: aggregates numbered along
// the grid couple only to neighbours, so A_H = P^T A P has half-bandwidth b = (aggregates per
// grid row) + 1 (23 at 64^2 with 3 x 3 boxes, 44 at 128^2). For b < 64 the coarse solve is a
// banded Cholesky factor A_H = L L^T (n_c b^2 / 2 multiply-adds instead of the dense inverse's
// n_c^3 / 3 + ...) and two band substitutions per cycle (4 n_c b bytes instead of 8 n_c^2).
// Held, like the dense paths, to fp64 rounding of a direct solve; chosen per problem from its own
// pattern, so a problem's results do not depend on its batch.
constexpr int kBandMax = 63;  // half-bandwidth limit: rows (j, j + b] within the 64 lanes
// coarse size limit: the substitutions run on one wave, ~45 ns per row and direction; a single
// call with a larger coarse operator is faster with the device-wide dense factor and its coarse
// solve spread over the CUs (128^2: 13 vs 26 ms). Every batch-eligible size (n_c <= 1024, the
// Python engine's FUSED_BATCH_MAX_NC) is below it, so batches and single calls choose alike.
constexpr int kBandMaxNc = 1024;

__device__ __forceinline__ double readlane_d(double v, int l) {
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)x, l);
  const int hi = __builtin_amdgcn_readlane((int)(x >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// pointers in a given address space (1 global, 3 LDS): loads through them are global / LDS
// instructions, not flat ones, so the compiler counts them on their own counters and a
// prefetch stays in flight (a flat load in a non-inlined function waits on every counter)
template <int AS>
using as_ptr = __attribute__((address_space(AS))) double*;
template <int AS>
using as_cptr = const __attribute__((address_space(AS))) double*;

// Right-looking banded Cholesky of AH (dense n_c x n_c, only |i - k| <= b read) over a sliding
// window of the b + 1 active rows in LDS (row i in slot i mod (b + 1), its entries k in
// [i - b, i) in column slots k mod (b + 1); diagonals in their own ring, slot i mod (b + 2)).
// Column j: l_i = a_ij / l_jj for i in (j, j + b], a_ik -= l_i l_k for j < k <= i <= j + b,
// and row j + b + 1 enters the slots row j leaves: one barrier per column (the entering row and
// every update touch slots column j does not read). The entering rows are loaded from AH two
// columns ahead. Out, in the band solve's lane layout (step j's 64 lane values contiguous, steps
// padded by kBandPad zero steps on either side, see band_solve): F[j][i mod 64] = L[i][j] / L[j][j]
// for i in (j, j + b], G[i][j mod 64] = L[i][j], RI[j] = 1 / L[j][j]. Returns false
// (uniformly) on a non-positive pivot.
constexpr int kBandPad = 32;  // zero steps before and after the band solve's lane layout
__device__ __forceinline__ int64_t band_at(int j, int l) { return (int64_t)(j + kBandPad) * 64 + l; }

// LDS ordering between the lanes of one wave: its LDS operations complete in issue order, so a
// wavefront-scope fence (no wait on global memory: prefetches and stores stay in flight) only
// keeps the compiler from moving LDS accesses across it
__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One workgroup, a (row, column) pair of column j's update per thread: rings of power-of-two
// sizes (slot = index & mask, no integer division), >= b + 2 rows and diagonals, rows stored
// with an odd stride (conflict-free LDS columns).
__device__ bool band_chol(const double* __restrict__ AH_, int nc, int b, double* lds,
                          double* __restrict__ F_, double* __restrict__ G_,
                          double* __restrict__ RI_, int tid) {
  const as_cptr<1> AH = (as_cptr<1>)AH_;
  const as_ptr<1> F = (as_ptr<1>)F_, G = (as_ptr<1>)G_, RI = (as_ptr<1>)RI_;
  int w = 1;
  while (w < b + 2) w <<= 1;
  const int m = w - 1, ws = w + 1;
  const as_ptr<3> off = (as_ptr<3>)lds;  // w rows of stride ws
  const as_ptr<3> dg = off + w * ws;     // w
  // zeros outside the band, and on the padding steps
  for (int64_t q = tid; q < (int64_t)(nc + 2 * kBandPad) * 64; q += kBT) {
    F[q] = 0.0;
    G[q] = 0.0;
  }
  for (int q = tid; q < nc + 2 * kBandPad; q += kBT) RI[q] = 0.0;
  for (int q = tid; q < (b + 1) * (b + 1); q += kBT) {
    const int i = q / (b + 1), k = q - i * (b + 1);
    if (i < nc && k < i) off[(i & m) * ws + (k & m)] = AH[(int64_t)i * nc + k];
  }
  for (int i = tid; i <= b && i < nc; i += kBT) dg[i & m] = AH[(int64_t)i * nc + i];
  // this thread's pairs (di, dk), 1 <= dk <= di <= b (rows j + di, j + dk): b <= 63 gives at
  // most 2016 pairs, two per thread
  int pdi[2] = {0, 0}, pdk[2] = {0, 0};
  const int npairs = b * (b + 1) / 2;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int p = tid + u * kBT;
    if (p < npairs) {
      int di = (int)((1.0 + sqrt(1.0 + 8.0 * (double)p)) * 0.5);
      while (di * (di - 1) / 2 > p) --di;
      while (di * (di + 1) / 2 <= p) ++di;
      pdi[u] = di;
      pdk[u] = p - di * (di - 1) / 2 + 1;
    }
  }
  // entering-row entries of this thread (tid <= b): row j + b + 1, column j + 1 + tid
  auto enter_val = [&](int j) -> double {
    const int ni = j + b + 1, k = j + 1 + tid;
    return tid <= b && ni < nc ? AH[(int64_t)ni * nc + (k < ni ? k : ni)] : 0.0;
  };
  double pre0 = enter_val(0), pre1 = enter_val(1);
  __syncthreads();
  auto column = [&](int j, double v) -> bool {
    const double d = dg[j & m];
    if (!(d > 0.0)) return false;  // every thread read the same pivot
    const double ljj = sqrt(d), r = 1.0 / ljj;
    const int cj = j & m;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int di = pdi[u], dk = pdk[u];
      const int i = j + di, k = j + dk;
      if (di == 0 || i >= nc) continue;
      const double li = off[(i & m) * ws + cj] * r;
      if (dk == di) {
        dg[i & m] = dg[i & m] - li * li;
        F[band_at(j, i & 63)] = li * r;
        G[band_at(i, j & 63)] = li;
      } else {
        const double lk = off[(k & m) * ws + cj] * r;
        off[(i & m) * ws + (k & m)] = off[(i & m) * ws + (k & m)] - li * lk;
      }
    }
    if (tid == 0) RI[j + kBandPad] = r;
    // the entering row (raw A_H: no column <= j has reached it), loaded two columns before
    const int ni = j + b + 1;
    if (ni < nc && tid <= b) {
      const int k = j + 1 + tid;
      if (k < ni) off[(ni & m) * ws + (k & m)] = v;
      else dg[ni & m] = v;
    }
    __syncthreads();
    return true;
  };
  for (int j = 0; j < nc; j += 2) {  // two columns per trip: each prefetch has a column to land
    const double v0 = pre0;
    pre0 = enter_val(j + 2);
    if (!column(j, v0)) return false;
    if (j + 1 >= nc) break;
    const double v1 = pre1;
    pre1 = enter_val(j + 3);
    if (!column(j + 1, v1)) return false;
  }
  return true;
}

// e = A_H^-1 r by L y = r, L^T e = y on ONE wave (the caller's wave 0): right-looking
// substitution over a window of 64 rows, row i on lane i mod 64. Step j: every lane reads the
// owner lane's partial sum s_j (readlane) and each window row i in (j, j + b] takes
// s_i -= (L_ij / l_jj) s_j, the band factor's value for (step j, this lane) read straight from
// the lane layout (zeros outside the band and on the padding steps: no index arithmetic, no
// conditions), so a step is readlane -> fused multiply-add. Row j's lane then holds row j + 64:
// after the step (any b < 64), or, when b <= 64 - D (LATE), for the D owners of a block at its
// end (row j + 64 takes its first update D or more steps later; an owner's sum is final from
// its step on). A block's values (D steps) are loaded one block ahead, so they stay in flight
// while the previous block computes; the owners store y_j = s_j / l_jj at the block's end.
// Backward the same over rows descending with G (L's rows) scaled by 1 / l_jj at load. r, y, e
// live in address spaces RS, YS, ES (1 global, 3 LDS). (Not inlined: its own registers; the
// cycle kernel saves its registers around the call once per coarse solve instead of spilling
// in its sweeps.)
template <int RS, int YS, int ES, bool LATE>
__device__ __noinline__ void band_solve(const double* __restrict__ F_,
                                        const double* __restrict__ G_,
                                        const double* __restrict__ RI_, int nc,
                                        const double* r_, double* y_, double* e_, int lane) {
  constexpr int D = 8;
  const as_cptr<1> F = (as_cptr<1>)F_, G = (as_cptr<1>)G_, RI = (as_cptr<1>)RI_;
  const as_cptr<RS> r = (as_cptr<RS>)r_;
  const as_ptr<YS> y = (as_ptr<YS>)y_;
  const as_ptr<ES> e = (as_ptr<ES>)e_;
  const int last = nc - 1;
  const int nblk = (nc + D - 1) / D;  // blocks of D steps; padding steps are exact no-ops
  // ---- forward: step j = q D + d; lane holds the row = lane (mod 64) in [j, j + 64)
  {
    double s = lane < nc ? r[lane] : 0.0;
    // block q: c[d] = F[j][lane]; p[0] = 1 / l of this lane's row in the block (owners);
    // p[1] = the row entering this lane (LATE: after the block; else lane d: at step j0 + d)
    double cf[2][D], pv[2][2];
    auto load = [&](int q, double (&c)[D], double (&p)[2]) {
      const int j0 = q * D;
      const int own = (j0 & ~63) + lane;
      p[0] = RI[min(own, nc) + kBandPad];
      const int nr = LATE ? own + 64 : j0 + lane + 64;
      p[1] = r[min(nr, last)];
      if (!(nr < nc && (LATE || lane < D))) p[1] = 0.0;
#pragma unroll
      for (int d = 0; d < D; ++d) c[d] = F[band_at(j0 + d, lane)];
    };
    auto steps = [&](int q, const double (&c)[D], const double (&p)[2]) {
      const int j0 = q * D;
      const bool mine = lane >= (j0 & 63) && lane < (j0 & 63) + D;
      double keep = 0.0;
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const int j = j0 + d;
        const double sj = readlane_d(s, j & 63);
        if (LATE) {
          s = __builtin_fma(-c[d], sj, s);
        } else {
          const bool own = lane == (j & 63);
          keep = own ? sj : keep;
          s = own ? readlane_d(p[1], d) : __builtin_fma(-c[d], sj, s);
        }
      }
      if (LATE) keep = s;
      const int jj = (j0 & ~63) + lane;
      if (mine && jj < nc) y[jj] = keep * p[0];
      if (LATE && mine) s = p[1];
    };
    load(0, cf[0], pv[0]);
    for (int q = 0; q < nblk; q += 2) {
      load(q + 1, cf[1], pv[1]);
      steps(q, cf[0], pv[0]);
      load(q + 2, cf[0], pv[0]);
      steps(q + 1, cf[1], pv[1]);
    }
  }
  // y stored by the owner lanes, read by every lane below
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  // ---- backward: step j = last - (q D + d); lane holds the row = lane (mod 64) in (j - 64, j]
  {
    const int k0 = last - ((last - lane) & 63);
    double s = k0 >= 0 ? y[k0] : 0.0;
    double cf[2][D], pv[2][2];
    auto load = [&](int q, double (&c)[D], double (&p)[2]) {
      const int hi = last - q * D;
      const int own = hi - ((hi - lane) & 63);  // this lane's row in (hi - 64, hi]
      p[0] = RI[max(own, -1) + kBandPad];
      const int nr = LATE ? own - 64 : hi - lane - 64;
      p[1] = y[max(nr, 0)];
      if (!(nr >= 0 && (LATE || lane < D))) p[1] = 0.0;
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const int j = hi - d;
        c[d] = G[band_at(j, lane)] * RI[j + kBandPad];
      }
    };
    auto steps = [&](int q, const double (&c)[D], const double (&p)[2]) {
      const int hi = last - q * D;
      const int jj = hi - ((hi - lane) & 63);
      const bool mine = jj > hi - D;
      double keep = 0.0;
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const int j = hi - d;
        const double sj = readlane_d(s, j & 63);
        if (LATE) {
          s = __builtin_fma(-c[d], sj, s);
        } else {
          const bool own = lane == (j & 63);
          keep = own ? sj : keep;
          s = own ? readlane_d(p[1], d) : __builtin_fma(-c[d], sj, s);
        }
      }
      if (LATE) keep = s;
      if (mine && jj >= 0) e[jj] = keep * p[0];
      if (LATE && mine) s = p[1];
    };
    load(0, cf[0], pv[0]);
    for (int q = 0; q < nblk; q += 2) {
      load(q + 1, cf[1], pv[1]);
      steps(q, cf[0], pv[0]);
      load(q + 2, cf[0], pv[0]);
      steps(q + 1, cf[1], pv[1]);
    }
  }
}

// A_H = P^T A P (dense, row j = coarse row j; accumulation order of the packed rows)
__device__ void dense_galerkin(const BDesc& D, char* arena, double* AH, int tid) {
  const int n = D.n, nc = D.nc, KA = D.KA, KP = D.KP, KT = D.KT;
  const int32_t* __restrict__ akc = at<int32_t>(arena, D.ak_col);
  const double* __restrict__ akv = at<double>(arena, D.ak_val);
  const int32_t* __restrict__ ppc = at<int32_t>(arena, D.pp_col);
  const double* __restrict__ ppv = at<double>(arena, D.pp_val);
  const int32_t* __restrict__ ptc = at<int32_t>(arena, D.pt_row);
  const double* __restrict__ ptv = at<double>(arena, D.pt_val);
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
}

// The Galerkin product of a single problem on the whole GPU (setup_mode 1): a workgroup per
// block of R coarse rows, each row accumulated by one thread in LDS in dense_galerkin's order
// (so A_H is bitwise the workgroup kernel's) instead of by read-modify-writes to global memory
// (a chain of ~800 dependent round trips per row), then written out coalesced.
__global__ __launch_bounds__(256) void k_galerkin_rows(const BDesc* __restrict__ descs,
                                                       char* __restrict__ arena, int R) {
  extern __shared__ double rows_lds[];
  const BDesc D = descs[0];
  const int n = D.n, nc = D.nc, KA = D.KA, KP = D.KP, KT = D.KT;
  const int j0 = blockIdx.x * R, nr = min(R, nc - j0);
  if (nr <= 0) return;
  for (int q = threadIdx.x; q < nr * nc; q += 256) rows_lds[q] = 0.0;
  __syncthreads();
  if ((int)threadIdx.x < nr) {
    const int32_t* __restrict__ akc = at<int32_t>(arena, D.ak_col);
    const double* __restrict__ akv = at<double>(arena, D.ak_val);
    const int32_t* __restrict__ ppc = at<int32_t>(arena, D.pp_col);
    const double* __restrict__ ppv = at<double>(arena, D.pp_val);
    const int32_t* __restrict__ ptc = at<int32_t>(arena, D.pt_row);
    const double* __restrict__ ptv = at<double>(arena, D.pt_val);
    const int j = j0 + threadIdx.x;
    double* row = rows_lds + (int64_t)threadIdx.x * nc;
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
  double* AH = at<double>(arena, D.AH) + (int64_t)j0 * nc;
  for (int q = threadIdx.x; q < nr * nc; q += 256) AH[q] = rows_lds[q];
}

// one workgroup per problem: Galerkin product and coarse inverse (operator mode in stat[2]:
// 1 = inverse Cholesky factor L^-1 in AH's lower triangle and its transpose in AI's upper
// triangle, 0 = the Gauss-Jordan inverse in AI)
__global__ __launch_bounds__(kBT) void k_amg2v_setup(const BDesc* __restrict__ descs,
                                                     char* __restrict__ arena, int band_pass) {
  extern __shared__ double lds[];
  __shared__ double redv[kBWaves];
  __shared__ int redi[kBWaves];
  const BDesc D = descs[blockIdx.x];
  const int tid = threadIdx.x;
  const int nc = D.nc;
  double* AH = at<double>(arena, D.AH);
  double* AI = at<double>(arena, D.AI);
  int32_t* stat = at<int32_t>(arena, D.stat_out);

  // phase wall times (100 MHz clock) when requested: [galerkin, inverse, smoothing, rest,
  // panels, updates]
  int64_t* tstat = at<int64_t>(arena, D.stat_out + 16);
  int64_t t_mark = D.timing ? wall_clock64() : 0;
  auto stamp = [&](int slot) {
    if (D.timing && tid == 0) {
      const int64_t t = wall_clock64();
      tstat[slot] += t - t_mark;
      t_mark = t;
    }
  };
  if (D.setup_mode == 3) return;
  if (band_pass) {
    // after k_amg2v_band: only a band factor that met a non-positive pivot continues, to
    // Gauss-Jordan on its A_H (which the band factor only read)
    if (D.band_ld == 0 || stat[2] == 2) return;
  } else {
    gather_values(D, arena, tid);
    if (D.timing && tid == 0)
      for (int q = 0; q < 8; ++q) tstat[q] = 0;
    if (tid == 0) {  // phased cycles: done flag, half cycles run
      stat[3] = 0;
      tstat[7] = 0;
    }
    if (D.setup_mode == 1) {  // A_H from k_galerkin_rows, the inverse from dense.hip
      if (tid == 0) {
        stat[1] = 0;
        stat[2] = 0;
      }
      return;
    }
    dense_galerkin(D, arena, AH, tid);
    stamp(0);
    if (D.setup_mode == 2 || D.band_ld > 0) {
      // the inverse from dense.hip's batched factorisation, or the band factor of k_amg2v_band
      if (tid == 0) {
        stat[1] = 0;
        stat[2] = D.band_ld > 0 ? 2 : 0;
      }
      return;
    }
  }

  if (D.spd && !band_pass) {
    // the panel width is the problem's own (a function of n_c alone): a problem's roundings do
    // not depend on the batch it is launched with
    const bool ok = D.chol_nb == 16   ? chol_inverse<16>(AH, nc, lds, tid, stamp)
                    : D.chol_nb == 8  ? chol_inverse<8>(AH, nc, lds, tid, stamp)
                                      : chol_inverse<4>(AH, nc, lds, tid, stamp);
    if (ok) {
      // AI[j][i] = L^-1[i][j] (i >= j): the rows of L^-T for the second solve phase
      for (int64_t q = tid; q < (int64_t)nc * nc; q += kBT) {
        const int64_t i = q / nc;
        const int j = (int)(q - i * nc);
        if (j <= i) AI[(int64_t)j * nc + i] = AH[q];
      }
      __syncthreads();
      stamp(1);
      if (tid == 0) {
        stat[1] = 0;
        stat[2] = 1;
      }
      return;
    }
    __syncthreads();
    dense_galerkin(D, arena, AH, tid);  // not SPD in floating point: Gauss-Jordan on a fresh A_H
  }

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
  if (tid == 0) {
    stat[1] = status;
    stat[2] = 0;
  }
}

// The banded Cholesky factor of every problem with a band (one workgroup each, after
// k_amg2v_setup's Galerkin product); a non-positive pivot sets stat[2] = 0, and the band pass of
// k_amg2v_setup that follows inverts that A_H by Gauss-Jordan instead.
__global__ __launch_bounds__(kBT) void k_amg2v_band(const BDesc* __restrict__ descs,
                                                    char* __restrict__ arena) {
  extern __shared__ double lds[];
  const BDesc D = descs[blockIdx.x];
  if (D.setup_mode == 3 || D.band_ld == 0) return;
  int32_t* stat = at<int32_t>(arena, D.stat_out);
  int64_t* tstat = at<int64_t>(arena, D.stat_out + 16);
  const int64_t t0 = D.timing ? wall_clock64() : 0;
  const bool ok = band_chol(at<double>(arena, D.AH), D.nc, D.band_ld - 1, lds,
                            at<double>(arena, D.lc), at<double>(arena, D.lr),
                            at<double>(arena, D.rinv), threadIdx.x);
  if (threadIdx.x == 0) {
    if (!ok) stat[2] = 0;
    if (D.timing) tstat[1] += wall_clock64() - t0;
  }
}

// The coarse solve of phased problems on every CU, a wave per row; block b belongs to problem q
// with cblk[q] <= b < cblk[q + 1]. Each row is the one-workgroup rows_dot's: lane l sums the
// columns l, l + 64, ... of its span with fma (masked slots add 0 * x), then the butterfly, so
// the result is the one-workgroup cycle's bit for bit.
//   PH 1: mode 0 (full inverse in AI): e_H = A_H^-1 r_H; mode 1: y = L^-1 r_H (AH's rows, [0, j])
//   PH 2: mode 1 only: e_H = L^-T y (AI's rows, [j, n_c))
template <int PH>
__global__ __launch_bounds__(256) void k_amg2v_coarse(const BDesc* __restrict__ descs,
                                                      char* __restrict__ arena,
                                                      const int32_t* __restrict__ cblk,
                                                      int count) {
  int lo = 0, hi = count;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (cblk[mid] <= (int)blockIdx.x) lo = mid;
    else hi = mid;
  }
  const BDesc* D = descs + lo;
  const int32_t* stat = at<int32_t>(arena, D->stat_out);
  if (stat[3]) return;
  const int mode = stat[2];
  if (mode == 2) return;  // banded: solved by the problem's own workgroup (k_amg2v_cycles)
  if (PH == 2 && mode != 1) return;
  const int nc = D->nc;
  const int row = ((int)blockIdx.x - cblk[lo]) * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= nc) return;
  const bool tri = mode == 1;
  const double* __restrict__ M =
      at<double>(arena, PH == 1 && tri ? D->AH : D->AI) + (int64_t)row * nc;
  const double* __restrict__ v = at<double>(arena, PH == 1 ? D->rcg : D->yg);
  double* out = at<double>(arena, PH == 1 && tri ? D->yg : D->eg);
  const int k0 = PH == 2 ? row : 0, k1 = PH == 1 && tri ? row + 1 : nc;
  double s = 0.0;
  for (int o = k0 & ~63; o < k1; o += 4 * 64) {
    double m[4], x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = o + u * 64 + lane;
      m[u] = (k >= k0 && k < k1) ? M[k] : 0.0;
      x[u] = k < nc ? v[k] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) s = fma(m[u], x[u], s);
  }
  s = bw_sum(s);
  if (lane == 0) out[row] = s;
}

// one workgroup per problem: the cycles (reads the setup kernel's inverse and status).
// PHASED (a single problem): one launch runs the second half of cycle k - 1 (x += P e_H from
// k_amg2v_coarse, post-smoothing, norm, tolerance test) and the first half of cycle k
// (pre-smoothing, residual, r_H = P^T r), x kept in x_out between launches; stat[3] = done,
// tstat[7] = launches so far
// RP: the one-wave sweep's register-prefetched staging (gs_rp), instantiated for single phased
// problems only (its registers would otherwise add spills to every other variant)
template <bool R_LDS, bool PHASED, bool RP>
__global__ __launch_bounds__(kBT) void k_amg2v_cycles(const BDesc* __restrict__ descs,
                                                      char* __restrict__ arena) {
  extern __shared__ double lds[];
  __shared__ double redv[kBWaves];
  const BDesc D = descs[blockIdx.x];
  const int tid = threadIdx.x;
  const int n = D.n, nc = D.nc;
  const double* __restrict__ b = at<double>(arena, D.b);
  const double* __restrict__ AI = at<double>(arena, D.AI);
  const double* __restrict__ AH = at<double>(arena, D.AH);
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
  int64_t* tstat = at<int64_t>(arena, D.stat_out + 16);
  int64_t t_mark = D.timing ? wall_clock64() : 0;
  auto stamp = [&](int slot) {
    if (D.timing && tid == 0) {
      const int64_t t = wall_clock64();
      tstat[slot] += t - t_mark;
      t_mark = t;
    }
  };
  const int status = stat[1], mode = stat[2];
  int64_t phase = 0;
  if constexpr (PHASED) {
    if (stat[3]) return;  // finished in an earlier launch
    phase = tstat[7];
  }

  // ---------------------------------------------------------------- cycles
  double* xs = lds;                                     // n + 2: x, a zero slot, a sink slot
  double* rcs;                                          // nc: restricted residual
  double* es;                                           // nc: coarse correction
  double* rs;                                           // n: residual
  int64_t stage_off;
  if constexpr (PHASED) {
    rcs = at<double>(arena, D.rcg);
    es = at<double>(arena, D.eg);
    rs = R_LDS ? xs + n + 2 : at<double>(arena, D.rg);
    stage_off = ((R_LDS ? n + 2 + n : n + 2) + 1) & ~int64_t(1);
  } else {
    rcs = xs + n + 2;
    es = rcs + nc;
    rs = R_LDS ? es + nc : at<double>(arena, D.rg);
    stage_off = ((R_LDS ? (es - lds) + nc + n : (es - lds) + nc) + 1) & ~int64_t(1);
  }
  double* ys = rs;  // nc <= n: L^-1 r_H, in r's storage (r is dead from the restriction to the
                    // next residual)
  // GS staging area, 16-byte aligned (the one-wave sweep reads its rows with 16-byte loads)
  // (an even double offset from the LDS base: index arithmetic keeps the LDS address space,
  // which an integer round trip would lose to flat accesses)
  double* stage = lds + stage_off;
  const double* __restrict__ x0 = PHASED && phase > 0 ? x_out : at<double>(arena, D.x0);
  #pragma unroll 1
  for (int i = tid; i < n; i += kBT) xs[i] = x0[i];
  if (tid == 0) xs[n] = 0.0;  // pad columns of the one-wave sweep read it; nothing writes it
  __syncthreads();
  if (status != 0) {  // multigrid.py:167-170: x returned untouched, no iteration
    #pragma unroll 1
    for (int i = tid; i < n; i += kBT) x_out[i] = xs[i];
    if (tid == 0) {
      stat[0] = 0;
      stat[3] = 1;
      if (PHASED) atomicAdd(at<int32_t>(arena, D.done_ctr), 1);
    }
    return;
  }
  // weighted-Jacobi weights (1/a_ii) * w, a_ii = the sum of the stored diagonal entries
  // (csr_diagonal); a phased problem keeps them from its first launch
  double* dwg = at<double>(arena, D.dinv);
  if (D.smoother == 1 && phase == 0) {
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

  // (b - A x)_i in csr_matvec's order (0 + a_1 x_1 + ... in stored order, then b_i - y) for
  // the rows i = tid + kBT * q, four at a time; out (nullable) takes r, part += r_i^2 in row order
  auto resid_rows = [&](double* out, double* part) {
    #pragma unroll 1
    for (int i0 = tid; i0 < n; i0 += 4 * kBT) {
      int rows[4];
      double y[4], bb[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        rows[u] = i0 + u * kBT < n ? i0 + u * kBT : -1;
        bb[u] = rows[u] >= 0 ? b[rows[u]] : 0.0;
      }
      packed_dot_rows<4>(akc, akv, n, rows, KA, xs, y);
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (rows[u] >= 0) {
          const double ri = bb[u] - y[u];
          if (out) out[rows[u]] = ri;
          if (part) *part += ri * ri;
        }
    }
  };

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

  // One wave sweeps the staged levels of a chunk (one-wave layout: position-major rows of KM
  // slots, pads = column n, the zero slot, value 0.0; a zero diagonal or a lane past the level's
  // end writes the sink slot n + 1; position cnt is such a dummy). A level's rows are
  // independent and a wave's LDS accesses complete in order, so consecutive levels need no
  // workgroup barrier — only a wavefront fence that keeps the compiler from moving the next
  // level's x gathers above this level's stores. Level l+1's rows are loaded while level l
  // gathers and divides. The padded sum adds +0.0 products to a sum that started at +0.0 (never
  // -0.0), so it is bitwise pyamg's.
  auto wave_sweep = [&](auto km_tag, auto rw_tag, const double* stg, int nl, int cnt) {
    constexpr int KM = decltype(km_tag)::value, RW = decltype(rw_tag)::value;
    const int lane = tid & 63;
    const double* sv = stg;
    const double* sd = sv + (int64_t)(cap + 1) * KM;
    const double* sb = sd + (cap + 1);
    const int32_t* sc = reinterpret_cast<const int32_t*>(sb + (cap + 1));
    const int32_t* sr = sc + (int64_t)(cap + 1) * KM;
    const int32_t* slp = sr + (cap + 1);
    int c[RW][KM], row[RW];
    double v[RW][KM], d[RW], bv[RW];
    auto load_level = [&](int l, int (&cc)[RW][KM], double (&vv)[RW][KM], double* dd,
                          double* bb, int* rr) {
      const int a = slp[l], z = slp[l + 1];
#pragma unroll
      for (int u = 0; u < RW; ++u) {
        const int p = a + lane + 64 * u < z ? a + lane + 64 * u : cnt;
#pragma unroll
        for (int k = 0; k < KM; k += 4) {
          const int4 c4 = *reinterpret_cast<const int4*>(sc + (int64_t)p * KM + k);
          cc[u][k] = c4.x;
          cc[u][k + 1] = c4.y;
          cc[u][k + 2] = c4.z;
          cc[u][k + 3] = c4.w;
        }
#pragma unroll
        for (int k = 0; k < KM; k += 2) {
          const double2 v2 = *reinterpret_cast<const double2*>(sv + (int64_t)p * KM + k);
          vv[u][k] = v2.x;
          vv[u][k + 1] = v2.y;
        }
        dd[u] = sd[p];
        bb[u] = sb[p];
        rr[u] = sr[p];
      }
    };
    load_level(0, c, v, d, bv, row);
    #pragma unroll 1
    for (int l = 0; l < nl; ++l) {
      double g[RW][KM];
#pragma unroll
      for (int u = 0; u < RW; ++u)
#pragma unroll
        for (int k = 0; k < KM; ++k) g[u][k] = xs[c[u][k]];
      int c2[RW][KM], row2[RW];
      double v2[RW][KM], d2[RW], bv2[RW];
      load_level(l + 1 < nl ? l + 1 : l, c2, v2, d2, bv2, row2);
#pragma unroll
      for (int u = 0; u < RW; ++u) {
        double y = 0.0;
#pragma unroll
        for (int k = 0; k < KM; ++k) y += v[u][k] * g[u][k];
        xs[row[u]] = (bv[u] - y) / d[u];
      }
#if MLAMG_GS_SCHED_FENCE
      // keep the next level's register copies below the store: scheduled above it they made
      // the store wait for the next level's structure reads (s_waitcnt lgkmcnt(0) before the
      // division's last step), one LDS round trip on every level of the dependency chain
      __builtin_amdgcn_sched_barrier(0);
#endif
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int u = 0; u < RW; ++u) {
#pragma unroll
        for (int k = 0; k < KM; ++k) {
          c[u][k] = c2[u][k];
          v[u][k] = v2[u][k];
        }
        d[u] = d2[u];
        bv[u] = bv2[u];
        row[u] = row2[u];
      }
    }
  };

  auto gs_sweep = [&]() {
    // pyamg gauss_seidel: rsum over the off-diagonals in stored order, diag = the last stored
    // diagonal entry, x_i = (b_i - rsum) / diag unless diag == 0
    if (D.gs_rw > 0) {  // one-wave sweep, position-major rows of K (= 4 or 8) slots
      // gs_db: two staging buffers, wave 0 sweeps chunk ch from one while waves 1-15 stage
      // chunk ch + 1 into the other, so a chunk's global round trip hides behind the previous
      // sweep (when the LDS left holds two buffers of >= 3 levels; else one buffer, restaged
      // by the whole workgroup between chunks)
      const int64_t buf_doubles = (((int64_t)(cap + 1) * (3 * K + 6) + 1) / 2 + 1) & ~int64_t(1);
      auto stage_chunk = [&](int ch, double* wv, int t0, int nt) {
        double* wd = wv + (int64_t)(cap + 1) * K;
        double* wb = wd + (cap + 1);
        int32_t* wc = reinterpret_cast<int32_t*>(wb + (cap + 1));
        int32_t* wr = wc + (int64_t)(cap + 1) * K;
        int32_t* wl = wr + (cap + 1);
        const int l0 = clev[ch], l1 = clev[ch + 1];
        const int P0 = lptr[l0], cnt = lptr[l1] - P0;
        for (int q = t0; q < cnt * K; q += nt) {
          wc[q] = pkc[(int64_t)P0 * K + q];
          wv[q] = pkv[(int64_t)P0 * K + q];
        }
        for (int q = t0; q < cnt; q += nt) {
          wd[q] = pkd[P0 + q];
          wb[q] = bl[P0 + q];
          wr[q] = pkr[P0 + q];
        }
        if (t0 < K) {  // the dummy position
          wc[cnt * K + t0] = n;
          wv[cnt * K + t0] = 0.0;
        }
        if (t0 == 0) {
          wd[cnt] = 1.0;
          wb[cnt] = 0.0;
          wr[cnt] = n + 1;
        }
        for (int q = t0; q <= l1 - l0; q += nt) wl[q] = lptr[l0 + q] - P0;
      };
      const bool db = D.gs_db != 0;
      constexpr bool rp = RP;
      // gs_rp (one buffer, chunks of <= 959 positions and <= 1920 slots): waves 1-15 load chunk
      // ch + 1 into registers while wave 0 sweeps ch, and write it into the buffer after the
      // sweep's barrier, so only an LDS copy separates two sweeps
      int rg_c[2] = {0, 0}, rg_r = 0, rg_l = 0;
      double rg_v[2] = {0.0, 0.0}, rg_d = 0.0, rg_b = 0.0;
      // half-steps h = 2 ch - 1 (staging of chunk 0), 2 ch (wave 0 sweeps ch; with db, waves
      // 1-15 stage ch + 1 meanwhile; with rp they load it), 2 ch + 1 (without db: waves 1-15
      // stage ch + 1, with rp from their registers)
      for (int h = -1; h < 2 * D.n_chunks; ++h) {
        const int ch = h < 0 ? -1 : h >> 1;
        const bool sweep_half = h >= 0 && (h & 1) == 0;
        const int nx = ch + 1;
        if (!sweep_half && db && h >= 0) continue;  // uniform: nothing to stage after a sweep
        double* cur = stage + (db ? (ch & 1) * buf_doubles : 0);
        if (sweep_half && tid < 64) {
          const int l0 = clev[ch], l1 = clev[ch + 1];
          const int cnt = lptr[l1] - lptr[l0];
          if (K == 4 && D.gs_rw == 1)
            wave_sweep(std::integral_constant<int, 4>(), std::integral_constant<int, 1>(), cur,
                       l1 - l0, cnt);
          else if (K == 4)
            wave_sweep(std::integral_constant<int, 4>(), std::integral_constant<int, 2>(), cur,
                       l1 - l0, cnt);
          else
            wave_sweep(std::integral_constant<int, 8>(), std::integral_constant<int, 1>(), cur,
                       l1 - l0, cnt);
        } else if (RP && h >= 0 && nx < D.n_chunks && tid >= 64) {
          const int t0 = tid - 64;
          const int l0 = clev[nx], l1 = clev[nx + 1];
          const int P0 = lptr[l0], cnt = lptr[l1] - P0;
          if (sweep_half) {  // global -> registers, under the sweep
#pragma unroll
            for (int u = 0; u < 2; ++u) {
              const int q = t0 + u * (kBT - 64);
              if (q < cnt * K) {
                rg_c[u] = pkc[(int64_t)P0 * K + q];
                rg_v[u] = pkv[(int64_t)P0 * K + q];
              }
            }
            if (t0 < cnt) {
              rg_d = pkd[P0 + t0];
              rg_b = bl[P0 + t0];
              rg_r = pkr[P0 + t0];
            }
            if (t0 <= l1 - l0) rg_l = lptr[l0 + t0] - P0;
          } else {  // registers -> the buffer (the sweep of ch is done)
            double* wv = stage;
            double* wd = wv + (int64_t)(cap + 1) * K;
            double* wb = wd + (cap + 1);
            int32_t* wc = reinterpret_cast<int32_t*>(wb + (cap + 1));
            int32_t* wr = wc + (int64_t)(cap + 1) * K;
            int32_t* wl = wr + (cap + 1);
#pragma unroll
            for (int u = 0; u < 2; ++u) {
              const int q = t0 + u * (kBT - 64);
              if (q < cnt * K) {
                wc[q] = rg_c[u];
                wv[q] = rg_v[u];
              }
            }
            if (t0 < cnt) {
              wd[t0] = rg_d;
              wb[t0] = rg_b;
              wr[t0] = rg_r;
            }
            if (t0 <= l1 - l0) wl[t0] = rg_l;
            if (t0 < K) {  // the dummy position
              wc[cnt * K + t0] = n;
              wv[cnt * K + t0] = 0.0;
            }
            if (t0 == 0) {
              wd[cnt] = 1.0;
              wb[cnt] = 0.0;
              wr[cnt] = n + 1;
            }
          }
        } else if (!rp && nx < D.n_chunks && (sweep_half == db || h < 0) && (tid >= 64 || !db)) {
          // without db wave 0 is idle here and stages too
          stage_chunk(nx, stage + (db ? (nx & 1) * buf_doubles : 0), db ? tid - 64 : tid,
                      db ? kBT - 64 : kBT);
        } else if (rp && h < 0) {
          stage_chunk(0, stage, tid, kBT);
        }
        __syncthreads();
      }
      return;
    }
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

  // the banded coarse solve on wave 0 (the band's rows need not fit the LDS)
  // (r_H, e_H: LDS, or global when PHASED; the intermediate in r's storage: LDS when R_LDS)
  auto band_coarse = [&](const double* rh, double* yv, double* ev) {
    if (tid < 64) {
      const int bw = D.band_ld - 1;
      const double* F = at<double>(arena, D.lc);
      const double* G = at<double>(arena, D.lr);
      const double* ri = at<double>(arena, D.rinv);
      constexpr int VS = PHASED ? 1 : 3, YS = R_LDS ? 3 : 1;
      if (bw <= 56) band_solve<VS, YS, VS, true>(F, G, ri, nc, rh, yv, ev, tid);
      else band_solve<VS, YS, VS, false>(F, G, ri, nc, rh, yv, ev, tid);
    }
  };

  auto smooth = [&](int nu) {
    stamp(3);
    for (int it = 0; it < nu; ++it) {
      if (D.smoother == 0) {
        gs_sweep();
      } else {  // MLAMG.py:143-146: x += Dinv_w (b - A x)
        resid_rows(rs, nullptr);
        __syncthreads();
        #pragma unroll 1
        for (int i = tid; i < n; i += kBT) xs[i] = xs[i] + dwg[i] * rs[i];
        __syncthreads();
      }
    }
    stamp(2);
  };

  // x += P e_H, post-smoothing, err[itn]; true when the tolerance is met
  auto second_half = [&](int itn) -> bool {
    #pragma unroll 1
    for (int i0 = tid; i0 < n; i0 += 4 * kBT) {  // x += P e
      int rows[4];
      double y[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) rows[u] = i0 + u * kBT < n ? i0 + u * kBT : -1;
      packed_dot_rows<4>(ppc, ppv, n, rows, KP, es, y);
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (rows[u] >= 0) xs[rows[u]] = xs[rows[u]] + y[u];
    }
    __syncthreads();
    smooth(D.nu_post);
    double part = 0.0;
    if (D.norm_mode == 0) {
      resid_rows(nullptr, &part);
    } else {
      #pragma unroll 1
      for (int i = tid; i < n; i += kBT) part += xs[i] * xs[i];
    }
    const double nrm = sqrt(block_sum(part, redv));
    if (tid == 0) err[itn] = nrm;
    return D.tol >= 0.0 && nrm <= D.tol;
  };

  if constexpr (PHASED) {
    const int k = (int)phase;
    bool fin = D.max_iter == 0;
    if (k > 0) fin = second_half(k - 1) || k == D.max_iter;
    if (!fin) {
      smooth(D.nu_pre);
      resid_rows(rs, nullptr);
      __syncthreads();
      #pragma unroll 1
      for (int j0 = tid; j0 < nc; j0 += 2 * kBT) {  // P^T r: csc_matvec's order
        int rows[2] = {j0, j0 + kBT < nc ? j0 + kBT : -1};
        double y[2];
        packed_dot_rows<2>(ptc, ptv, nc, rows, KT, rs, y);
        rcs[j0] = y[0];
        if (rows[1] >= 0) rcs[rows[1]] = y[1];
      }
      __syncthreads();
      stamp(3);
      if (mode == 2) {  // banded: this workgroup's wave 0 solves (k_amg2v_coarse skips it)
        band_coarse(rcs, ys, es);
        __syncthreads();
        stamp(6);
      }
    }
    #pragma unroll 1
    for (int i = tid; i < n; i += kBT) x_out[i] = xs[i];
    stamp(3);
    if (tid == 0) {
      tstat[7] = phase + 1;
      if (fin) {
        stat[0] = k;
        stat[3] = 1;
        atomicAdd(at<int32_t>(arena, D.done_ctr), 1);
      }
    }
    return;
  } else {
    int iters = 0;
    for (int itn = 0; itn < D.max_iter; ++itn) {
      smooth(D.nu_pre);
      resid_rows(rs, nullptr);
      __syncthreads();
      #pragma unroll 1
      for (int j0 = tid; j0 < nc; j0 += 2 * kBT) {  // P^T r: csc_matvec's order
        int rows[2] = {j0, j0 + kBT < nc ? j0 + kBT : -1};
        double y[2];
        packed_dot_rows<2>(ptc, ptv, nc, rows, KT, rs, y);
        rcs[j0] = y[0];
        if (rows[1] >= 0) rcs[rows[1]] = y[1];
      }
      __syncthreads();
      stamp(3);
      if (mode == 2) {  // banded: L y = r_H, L^T e = y on wave 0
        band_coarse(rcs, ys, es);
      } else if (mode == 1) {  // e = L^-T (L^-1 r_H)
        rows_dot<1>(AH, nc, rcs, ys, tid);
        __syncthreads();
        rows_dot<2>(AI, nc, ys, es, tid);
      } else {  // e = A_H^-1 r_H (Gauss-Jordan inverse)
        rows_dot<0>(AI, nc, rcs, es, tid);
      }
      __syncthreads();
      stamp(6);
      iters = itn + 1;
      if (second_half(itn)) break;
    }
    #pragma unroll 1
    for (int i = tid; i < n; i += kBT) x_out[i] = xs[i];
    stamp(3);
    if (tid == 0) stat[0] = iters;
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

// A == A^T exactly (values included): then A_H = P^T A P is symmetric and, A being SPD, the
// coarse solve can take the inverse Cholesky factor
bool csr_symmetric(int64_t n, const int32_t* ip, const int32_t* ij, const double* v) {
  const int64_t nnz = ip[n];
  std::vector<int32_t> tp(n + 1, 0), ti(nnz);
  std::vector<double> tv(nnz);
  for (int64_t k = 0; k < nnz; ++k) tp[ij[k] + 1]++;
  for (int64_t j = 0; j < n; ++j) tp[j + 1] += tp[j];
  std::vector<int32_t> fill(tp.begin(), tp.end() - 1);
  for (int64_t i = 0; i < n; ++i)
    for (int32_t k = ip[i]; k < ip[i + 1]; ++k) {
      ti[fill[ij[k]]] = (int32_t)i;
      tv[fill[ij[k]]++] = v[k];
    }
  // row i of A^T lists its columns ascending; compare with row i of A sorted by column
  std::vector<std::pair<int32_t, double>> row;
  for (int64_t i = 0; i < n; ++i) {
    if (ip[i + 1] - ip[i] != tp[i + 1] - tp[i]) return false;
    row.clear();
    for (int32_t k = ip[i]; k < ip[i + 1]; ++k) row.emplace_back(ij[k], v[k]);
    std::sort(row.begin(), row.end(),
              [](const std::pair<int32_t, double>& a, const std::pair<int32_t, double>& b) {
                return a.first < b.first;
              });
    for (size_t q = 0; q < row.size(); ++q)
      if (row[q].first != ti[tp[i] + q] || !(row[q].second == tv[tp[i] + q])) return false;
  }
  return true;
}

// f(0 .. count-1) on up to MLAMG_HOST_THREADS (default: the CPUs this process may run on, at
// most 16) host threads; the calling thread takes a share. Small counts run inline.
// Persistent host workers for parallel_for (creating and joining 15 threads per call cost
// ~0.5 ms of a 48-grid batch). One job at a time; a caller that finds the pool busy (another
// host thread's batch) runs its loop inline.
class HostPool {
 public:
  explicit HostPool(int workers) {
    for (int t = 0; t < workers; ++t) th_.emplace_back([this] { loop(); });
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int workers() const { return (int)th_.size(); }
  // f(0 .. count-1) on the workers and the calling thread; false when the pool is busy
  bool run(int count, const std::function<void(int)>& f) {
    if (getpid() != pid_) return false;  // a forked child has no workers
    std::unique_lock<std::mutex> busy(run_mu_, std::try_to_lock);
    if (!busy.owns_lock()) return false;
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = &f;
      count_ = count;
      next_.store(0);
      active_ = (int)th_.size();
      ++gen_;
    }
    cv_.notify_all();
    for (int q = next_.fetch_add(1); q < count; q = next_.fetch_add(1)) f(q);
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [this] { return active_ == 0; });
    job_ = nullptr;
    return true;
  }

 private:
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)>* job;
      int count;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        job = job_;
        count = count_;
      }
      for (int q = next_.fetch_add(1); q < count; q = next_.fetch_add(1)) (*job)(q);
      std::lock_guard<std::mutex> lk(mu_);
      if (--active_ == 0) done_cv_.notify_all();
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_, run_mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* job_ = nullptr;
  int count_ = 0, active_ = 0;
  uint64_t gen_ = 0;
  std::atomic<int> next_{0};
  bool stop_ = false;
  pid_t pid_ = getpid();
};

int host_threads() {
  static const int max_threads = [] {
    int t = 16;
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) t = std::min(t, CPU_COUNT(&set));
    if (const char* e = std::getenv("MLAMG_HOST_THREADS")) t = std::max(1, std::atoi(e));
    return std::max(1, t);
  }();
  return max_threads;
}

HostPool& host_pool() {  // one pool for every parallel_for of the process
  static HostPool pool(host_threads() - 1);
  return pool;
}

template <class F>
void parallel_for(int count, F&& f) {
  if (host_threads() <= 1 || count < 4) {
    for (int q = 0; q < count; ++q) f(q);
    return;
  }
  const std::function<void(int)> fn = [&](int q) { f(q); };
  if (!host_pool().run(count, fn))
    for (int q = 0; q < count; ++q) f(q);
}

// ---------------------------------------------------------------- problem patterns and shapes
// Everything the host derives from a problem's index arrays alone is computed once per distinct
// sparsity pattern and kept across calls (a dataset's grids share few patterns: the reference's
// farms loop over grids of a handful of sizes); per problem only the caller's values travel
// (A.data, P.data, b, x0) and are placed into the packed layouts on the device.
//   Pattern: the arrays (for the exact match), the exact-symmetry pairing of A's entries and the
//            half-bandwidth of A_H = P^T A P — independent of the batch's flags;
//   Shape:   a pattern's level schedule, packed column layouts and value maps for one set of
//            batch flags (smoother, phased, residual in LDS, single call).
struct Pattern {
  int64_t n = 0, nc = 0, annz = 0, pnnz = 0;
  uint64_t key = 0;
  std::vector<int32_t> aip, aij, pip, pij;
  // sym[k] = index of entry (j, i) for entry k = (i, j); sym_ok false when an entry has no
  // mirror; dups when a row repeats a column (the value test then sorts, csr_symmetric)
  std::vector<int32_t> sym;
  bool sym_ok = false, dups = false;
  int band = 0;  // half-bandwidth of A_H's structure (lower part)
  size_t bytes() const { return 4 * (aip.size() + aij.size() + pip.size() + pij.size() + sym.size()); }
};

struct Shape {
  std::shared_ptr<const Pattern> pat;
  int smoother = 0, phased = 0, r_lds = 0, single = 0;
  // slot-major packed columns (-1 pads) and, per slot, the index of its value in A.data /
  // P.data (-1: pad, value 0.0)
  std::vector<int32_t> akc, amap, ppc, pmap, ptc, tmap;
  // Gauss-Seidel sweep in level order: lev/clev (level and chunk starts), pkc/gmap the
  // off-diagonal slots (position-major for the one-wave sweep), dmap the last stored diagonal
  // entry of each position (-1: none), pkr0 the position's row
  std::vector<int32_t> lev, clev, pkc, gmap, dmap, pkr0;
  bool chol_fits = false;
  int K = 1, KA = 1, KP = 1, KT = 1, nlev = 0, panel = 8, cap = 0, chol_nb = 4;
  int gs_rw = 0, gs_db = 0, gs_rp = 0;
  size_t lds_base = 0, lds_chol = 0, lds_cycles = 0;
  int code = MLAMG_OK;
  std::string err;
  size_t bytes() const {
    size_t b = 0;
    for (const auto* v : {&akc, &amap, &ppc, &pmap, &ptc, &tmap, &lev, &clev, &pkc, &gmap, &dmap,
                          &pkr0})
      b += 4 * v->size();
    return b;
  }
};

uint64_t mix_bytes(const void* data, size_t bytes, uint64_t h) {
  const unsigned char* p = static_cast<const unsigned char*>(data);
  constexpr uint64_t M1 = 0x9E3779B97F4A7C15ull, M2 = 0xC2B2AE3D27D4EB4Full;
  uint64_t a = h ^ M1, b = h + M2, c = h * M1 + 1, d = h ^ M2;
  size_t i = 0;
  for (; i + 32 <= bytes; i += 32) {  // four independent lanes
    uint64_t w[4];
    std::memcpy(w, p + i, 32);
    a = (a ^ w[0]) * M1;
    b = (b ^ w[1]) * M2;
    c = (c ^ w[2]) * M1;
    d = (d ^ w[3]) * M2;
    a ^= a >> 29;
    b ^= b >> 31;
    c ^= c >> 27;
    d ^= d >> 33;
  }
  for (; i < bytes; ++i) a = (a ^ p[i]) * M1;
  uint64_t r = a ^ (b * M1) ^ (c * M2) ^ (d + M1) ^ bytes;
  r ^= r >> 32;
  return r * M2;
}

uint64_t pattern_key(const mlamg_amg2v_problem& P) {
  int64_t hdr[4] = {P.n, P.n_c, P.A_nnz, P.P_nnz};
  uint64_t h = mix_bytes(hdr, sizeof(hdr), 0x5A17u);
  h = mix_bytes(P.A_indptr, 4 * (size_t)(P.n + 1), h);
  h = mix_bytes(P.A_indices, 4 * (size_t)P.A_nnz, h);
  h = mix_bytes(P.P_indptr, 4 * (size_t)(P.n + 1), h);
  return mix_bytes(P.P_indices, 4 * (size_t)P.P_nnz, h);
}

bool same_pattern(const mlamg_amg2v_problem& a, const mlamg_amg2v_problem& b) {
  if (a.n != b.n || a.n_c != b.n_c || a.A_nnz != b.A_nnz || a.P_nnz != b.P_nnz) return false;
  auto eq = [](const int32_t* x, const int32_t* y, int64_t cnt) {
    return x == y || cnt == 0 || std::memcmp(x, y, 4 * (size_t)cnt) == 0;
  };
  return eq(a.A_indptr, b.A_indptr, a.n + 1) && eq(a.A_indices, b.A_indices, a.A_nnz) &&
         eq(a.P_indptr, b.P_indptr, a.n + 1) && eq(a.P_indices, b.P_indices, a.P_nnz);
}

bool pattern_matches(const Pattern& S, const mlamg_amg2v_problem& P) {
  mlamg_amg2v_problem q{};
  q.n = S.n;
  q.n_c = S.nc;
  q.A_nnz = S.annz;
  q.P_nnz = S.pnnz;
  q.A_indptr = S.aip.data();
  q.A_indices = S.aij.data();
  q.P_indptr = S.pip.data();
  q.P_indices = S.pij.data();
  return same_pattern(q, P);
}

// bounded most-recently-used lists (count and bytes); one lock for both
std::mutex g_shape_mu;
std::vector<std::shared_ptr<const Pattern>> g_patterns;
std::vector<std::shared_ptr<const Shape>> g_shapes;
constexpr size_t kCacheCount = 64;
constexpr size_t kCacheBytes = size_t(256) << 20;

template <class T>
void cache_trim(std::vector<std::shared_ptr<const T>>& v) {
  size_t total = 0;
  for (const auto& t : v) total += t->bytes();
  while (v.size() > 1 && (v.size() > kCacheCount || total > kCacheBytes)) {
    total -= v.front()->bytes();
    v.erase(v.begin());
  }
}

std::shared_ptr<const Pattern> pattern_lookup(uint64_t key, const mlamg_amg2v_problem& P) {
  std::lock_guard<std::mutex> lk(g_shape_mu);
  for (size_t i = g_patterns.size(); i-- > 0;)
    if (g_patterns[i]->key == key && pattern_matches(*g_patterns[i], P)) {
      auto s = g_patterns[i];
      g_patterns.erase(g_patterns.begin() + (long)i);
      g_patterns.push_back(s);
      return s;
    }
  return nullptr;
}

std::shared_ptr<const Shape> shape_lookup(const Pattern* pat, int smoother, int phased,
                                          int r_lds, int single) {
  std::lock_guard<std::mutex> lk(g_shape_mu);
  for (size_t i = g_shapes.size(); i-- > 0;) {
    const Shape& S = *g_shapes[i];
    if (S.pat.get() == pat && S.smoother == smoother && S.phased == phased &&
        S.r_lds == r_lds && S.single == single) {
      auto s = g_shapes[i];
      g_shapes.erase(g_shapes.begin() + (long)i);
      g_shapes.push_back(s);
      return s;
    }
  }
  return nullptr;
}

void pattern_insert(const std::shared_ptr<const Pattern>& s) {
  std::lock_guard<std::mutex> lk(g_shape_mu);
  g_patterns.push_back(s);
  cache_trim(g_patterns);
}

void shape_insert(const std::shared_ptr<const Shape>& s) {
  std::lock_guard<std::mutex> lk(g_shape_mu);
  g_shapes.push_back(s);
  cache_trim(g_shapes);
}

// rows of a CSR pattern into a slot-major fixed-width layout: col (-1 pads) and the index of
// each slot's value (-1 pads); width = the longest row (>= 1)
int pack_map(int64_t rows, const int32_t* ip, const int32_t* ij, std::vector<int32_t>& col,
             std::vector<int32_t>& map) {
  int w = 1;
  for (int64_t i = 0; i < rows; ++i) w = std::max(w, ip[i + 1] - ip[i]);
  col.assign((size_t)w * rows, -1);
  map.assign((size_t)w * rows, -1);
  for (int64_t i = 0; i < rows; ++i)
    for (int32_t k = ip[i]; k < ip[i + 1]; ++k) {
      col[(size_t)(k - ip[i]) * rows + i] = ij[k];
      map[(size_t)(k - ip[i]) * rows + i] = k;
    }
  return w;
}

std::shared_ptr<Pattern> analyse_pattern(const mlamg_amg2v_problem& P, uint64_t key) {
  auto Sp = std::make_shared<Pattern>();
  Pattern& S = *Sp;
  const int64_t n = P.n, nnz = P.A_nnz;
  const int32_t *ip = P.A_indptr, *ij = P.A_indices;
  S.n = n;
  S.nc = P.n_c;
  S.annz = nnz;
  S.pnnz = P.P_nnz;
  S.key = key;
  S.aip.assign(ip, ip + n + 1);
  S.aij.assign(ij, ij + nnz);
  S.pip.assign(P.P_indptr, P.P_indptr + n + 1);
  S.pij.assign(P.P_indices, P.P_indices + P.P_nnz);
  // A's structural transpose pairing
  std::vector<int32_t> tp(n + 1, 0), tk(nnz), tr(nnz);
  for (int64_t k = 0; k < nnz; ++k) tp[ij[k] + 1]++;
  for (int64_t j = 0; j < n; ++j) tp[j + 1] += tp[j];
  std::vector<int32_t> fill(tp.begin(), tp.end() - 1);
  for (int64_t i = 0; i < n; ++i)
    for (int32_t k = ip[i]; k < ip[i + 1]; ++k) {  // column j: rows ascending
      tr[fill[ij[k]]] = (int32_t)i;
      tk[fill[ij[k]]++] = k;
    }
  S.sym.assign(nnz, -1);
  S.sym_ok = true;
  std::vector<std::pair<int32_t, int32_t>> row;
  for (int64_t i = 0; i < n; ++i) {
    row.clear();
    for (int32_t k = ip[i]; k < ip[i + 1]; ++k) row.emplace_back(ij[k], k);
    std::sort(row.begin(), row.end());
    for (size_t q = 1; q < row.size(); ++q)
      if (row[q].first == row[q - 1].first) S.dups = true;
    if (ip[i + 1] - ip[i] != tp[i + 1] - tp[i]) {
      S.sym_ok = false;
      continue;
    }
    // column i of A (entries (r, i), r ascending) against row i's columns ascending
    for (size_t q = 0; q < row.size(); ++q) {
      if (tr[tp[i] + q] != row[q].first) S.sym_ok = false;
      S.sym[row[q].second] = tk[tp[i] + q];
    }
  }
  if (S.dups) S.sym_ok = false;
  // half-bandwidth of A_H: (P^T A P)_IJ != 0 needs P_iI, A_ik, P_kJ != 0, so the lowest J of
  // any coarse row I of fine row i is the lowest P column over i's A neighbours
  std::vector<int32_t> pmin(n, INT32_MAX);
  for (int64_t i = 0; i < n; ++i)
    for (int32_t k = P.P_indptr[i]; k < P.P_indptr[i + 1]; ++k)
      pmin[i] = std::min(pmin[i], P.P_indices[k]);
  int band = 0;
  for (int64_t i = 0; i < n; ++i) {
    int32_t am = INT32_MAX;
    for (int32_t k = ip[i]; k < ip[i + 1]; ++k) am = std::min(am, pmin[ij[k]]);
    if (am == INT32_MAX) continue;
    for (int32_t k = P.P_indptr[i]; k < P.P_indptr[i + 1]; ++k)
      band = std::max(band, P.P_indices[k] - am);
  }
  S.band = band;
  return Sp;
}

// chol_lds / setup_lds: LDS bytes of the inverse-Cholesky factor (two NB x (NB+1) blocks, the
// L21 panel and the Z rows) and of the Gauss-Jordan panel (n_c x (b+1), pivots, permutation)
size_t chol_lds(int nb, int64_t nc) {
  return (size_t)8 * (2 * nb * (nb + 1) + (size_t)nc * (nb + 1) + (size_t)nb * nc);
}
size_t band_lds(int b) {  // band_chol's rings: w x (w + 1) window, w diagonals
  size_t w = 1;
  while (w < (size_t)b + 2) w <<= 1;
  return 8 * (w * (w + 1) + w);
}
size_t gj_lds(int b, int64_t nc) { return (size_t)nc * (b + 1) * 8 + 16 * b + (size_t)nc * 12; }

// the structure analysis of one pattern (P already validated)
std::shared_ptr<Shape> analyse_shape(const mlamg_amg2v_problem& P,
                                     const std::shared_ptr<const Pattern>& pat, int smoother,
                                     int phased, int r_lds, int single) {
  auto Sp = std::make_shared<Shape>();
  Shape& L = *Sp;
  const int64_t n = P.n, nc = P.n_c;
  L.pat = pat;
  L.smoother = smoother;
  L.phased = phased;
  L.r_lds = r_lds;
  L.single = single;
  L.KA = pack_map(n, P.A_indptr, P.A_indices, L.akc, L.amap);
  L.KP = pack_map(n, P.P_indptr, P.P_indices, L.ppc, L.pmap);
  {  // P^T: entries of coarse column j in ascending fine row
    std::vector<int32_t> tp(nc + 1, 0);
    for (int64_t k = 0; k < P.P_nnz; ++k) tp[P.P_indices[k] + 1]++;
    for (int64_t j = 0; j < nc; ++j) tp[j + 1] += tp[j];
    std::vector<int32_t> ti(P.P_nnz), tk(P.P_nnz);
    std::vector<int32_t> fill(tp.begin(), tp.end() - 1);
    for (int64_t i = 0; i < n; ++i)
      for (int32_t k = P.P_indptr[i]; k < P.P_indptr[i + 1]; ++k) {
        const int32_t j = P.P_indices[k];
        ti[fill[j]] = (int32_t)i;
        tk[fill[j]++] = k;
      }
    L.KT = pack_map(nc, tp.data(), ti.data(), L.ptc, L.tmap);
    // pack_map stored positions into ti/tk; map them back to P.data indices
    for (auto& m : L.tmap)
      if (m >= 0) m = tk[m];
  }
  if (L.KA > kBMaxK + 1 || L.KP > kBMaxKP || L.KT > kBMaxKT) {
    L.code = MLAMG_EUNSUPPORTED;
    L.err = "amg2v_batch: rows of A, P or P^T longer than the batched solver's slots";
    return Sp;
  }
  int chol_nb = 16;  // the widest panel that fits (wider panels lengthen the per-thread
                     // triangular solves more than they save in trailing passes)
  while (chol_nb > 4 && chol_lds(chol_nb, nc) > kBLdsBytes) chol_nb >>= 1;
  L.chol_nb = chol_nb;
  L.chol_fits = chol_lds(chol_nb, nc) <= kBLdsBytes;
  L.lds_chol = chol_lds(chol_nb, nc);
  // cycle vectors in LDS: x (+ zero and sink slots), r when it fits (L^-1 r_H shares it), r_H,
  // e_H; the sweep's staging area gets the rest
  const size_t vec_lds = (size_t)n * 8 * (r_lds ? 2 : 1) + 16 + (phased ? 0 : (size_t)nc * 16);
  const size_t room = kBLdsBytes > vec_lds + 64 ? kBLdsBytes - vec_lds - 64 : 0;
  int gs_rw = 0;
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
      L.code = MLAMG_EUNSUPPORTED;
      L.err = "amg2v_batch: a row of A has more than 32 off-diagonal entries";
      return Sp;
    }
    L.lev.assign(L.nlev + 1, 0);
    for (int64_t i = 0; i < n; ++i) L.lev[level[i] + 1]++;
    for (int l = 0; l < L.nlev; ++l) L.lev[l + 1] += L.lev[l];
    int wmax = 0;
    for (int l = 0; l < L.nlev; ++l) wmax = std::max(wmax, L.lev[l + 1] - L.lev[l]);
    // one-wave sweep: rows of 4 slots and levels of <= 128 rows, or 8 slots and <= 64 rows,
    // and a staging area that holds the widest level (+ the dummy position)
    const int km = maxoff <= 4 ? 4 : maxoff <= 8 ? 8 : 0;
    if (km == 4 && wmax <= 128) gs_rw = wmax <= 64 ? 1 : 2;
    if (km == 8 && wmax <= 64) gs_rw = 1;
    if (gs_rw && (int)std::min<size_t>(4096, room / (12 * km + 24)) - 1 < wmax) gs_rw = 0;
    // two staging buffers when each still holds >= 3 of the widest levels
    static const bool no_db = std::getenv("MLAMG_BATCH_NO_DB") != nullptr;  // A/B knob
    if (gs_rw && !no_db &&
        (int)std::min<size_t>(4096, room / (2 * (12 * km + 24) + 16)) - 1 >= 3 * wmax)
      L.gs_db = 1;
    L.K = gs_rw ? km : std::max(maxoff, 1);
    const int64_t K = L.K;
    L.pkr0.resize(n);
    L.pkc.assign((size_t)n * K, gs_rw ? (int32_t)n : -1);
    L.gmap.assign((size_t)n * K, -1);
    L.dmap.assign(n, -1);
    std::vector<int32_t> fill(L.lev.begin(), L.lev.end() - 1);
    for (int64_t i = 0; i < n; ++i) {
      const int32_t p = fill[level[i]]++;
      L.pkr0[p] = (int32_t)i;
      int s2 = 0;
      for (int32_t k = P.A_indptr[i]; k < P.A_indptr[i + 1]; ++k) {
        if (P.A_indices[k] == i) {
          L.dmap[p] = k;  // the last stored diagonal entry, as the sweep takes it
        } else {
          // slot-major for the workgroup sweep, position-major for the one-wave sweep
          const size_t at = gs_rw ? (size_t)p * K + s2 : (size_t)s2 * n + p;
          L.pkc[at] = P.A_indices[k];
          L.gmap[at] = k;
          ++s2;
        }
      }
    }
  }
  // panel width: the widest power of two <= 16 whose n_c x (b+1) panel (+ pivots and the
  // final column permutation) fits
  int pb = kBMaxPanel;
  while (pb > 4 && gj_lds(pb, nc) > kBLdsBytes) pb >>= 1;
  if (gj_lds(pb, nc) > kBLdsBytes) {
    L.code = MLAMG_EINVAL;
    L.err = "coarse too large";
    return Sp;
  }
  L.panel = pb;
  // GS staging chunks: runs of consecutive levels with <= cap rows, cap from the LDS left
  // after the cycle vectors, one position kept for the one-wave sweep's dummy (a level wider
  // than cap is swept by the workgroup straight from the arena)
  if (smoother == 0) {
    const size_t per_pos = (12 * (size_t)L.K + 24) * (L.gs_db ? 2 : 1);
    const size_t slack = L.gs_db ? 32 : 0;
    L.cap = (int)std::min<size_t>(4096, (room > slack ? room - slack : 0) / per_pos) - 1;
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
  static const bool no_rp = std::getenv("MLAMG_BATCH_NO_RP") != nullptr;  // A/B knob
  if (phased && single && gs_rw && !L.gs_db && !no_rp && L.cap + 1 <= kBT - 64 &&
      L.cap * L.K <= 2 * (kBT - 64))
    L.gs_rp = 1;
  L.lds_base = gj_lds(pb, nc);
  L.lds_cycles = vec_lds + 16 + (size_t)(L.cap + 1) * (12 * L.K + 24) * (L.gs_db ? 2 : 1) + 40;
  L.gs_rw = gs_rw;
  return Sp;
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
  // ---- host: validation, patterns (flag-independent analysis), per-problem value checks, the
  // batch's strategy, shapes (flag-dependent analysis); patterns and shapes cached across calls
  static const bool timing = std::getenv("MLAMG_BATCH_TIMING") != nullptr;
  const auto t_begin = std::chrono::steady_clock::now();
  std::vector<BDesc> desc(count);
  const bool no_cache = std::getenv("MLAMG_BATCH_NO_SHAPE_CACHE") != nullptr;  // A/B knob
  const bool no_band = std::getenv("MLAMG_BATCH_NO_BAND") != nullptr;         // A/B knob
  // 1. validation and the pattern key of every problem (host threads)
  std::vector<int> vcode(count, MLAMG_OK);
  std::vector<const char*> verr(count, nullptr);
  std::vector<uint64_t> key(count, 0);
  parallel_for(count, [&](int q) {
    const mlamg_amg2v_problem& P = probs[q];
    auto fail = [&](const char* m) {
      vcode[q] = MLAMG_EINVAL;
      verr[q] = m;
    };
    const int64_t n = P.n, nc = P.n_c;
    if (!(n >= 1 && n <= kBMaxN)) return fail("problem rows out of range for the batched solver");
    if (!(nc >= 1 && nc <= kBMaxNc && nc <= n)) return fail("coarse size out of range");
    if (!(valid_csr(n, n, P.A_nnz, P.A_indptr, P.A_indices) && P.A_data))
      return fail("A is not a valid n x n CSR");
    if (!(valid_csr(n, nc, P.P_nnz, P.P_indptr, P.P_indices) && P.P_data))
      return fail("P is not a valid n x n_c CSR");
    if (!(P.b && P.x0 && P.x_out && (max_iter == 0 || P.err_out))) return fail("NULL vector");
    key[q] = pattern_key(P);
  });
  for (int q = 0; q < count; ++q)
    if (vcode[q] != MLAMG_OK) {
      set_error(std::string(verr[q]) + " (problem " + std::to_string(q) + ")");
      return vcode[q];
    }
  // 2. group by key (a representative per distinct key), members compared in full (a key
  // collision leaves the member its own pattern); patterns from the cache or analysed
  std::vector<int> rep(count);
  {
    std::vector<std::pair<uint64_t, int>> order(count);
    for (int q = 0; q < count; ++q) order[q] = {key[q], q};
    std::sort(order.begin(), order.end());
    for (int t = 0; t < count; ++t)
      rep[order[t].second] = t > 0 && order[t].first == order[t - 1].first
                                 ? rep[order[t - 1].second]
                                 : order[t].second;
  }
  parallel_for(count, [&](int q) {
    if (rep[q] != q && !same_pattern(probs[q], probs[rep[q]])) rep[q] = q;
  });
  std::vector<std::shared_ptr<const Pattern>> pat(count);
  std::vector<int> todo;
  for (int q = 0; q < count; ++q)
    if (rep[q] == q) {
      if (!no_cache) pat[q] = pattern_lookup(key[q], probs[q]);
      if (!pat[q]) todo.push_back(q);
    }
  parallel_for((int)todo.size(), [&](int t) {
    const int q = todo[t];
    auto S = analyse_pattern(probs[q], key[q]);
    if (!no_cache) pattern_insert(S);
    pat[q] = S;
  });
  for (int q = 0; q < count; ++q) pat[q] = pat[rep[q]];
  // 3. per problem: A == A^T exactly (values included) -> an SPD coarse operator, factored as a
  // band when its structure is narrow, else as a dense inverse Cholesky factor
  std::vector<char> sym(count, 0), band(count, 0);
  parallel_for(count, [&](int q) {
    const Pattern& S = *pat[q];
    const mlamg_amg2v_problem& P = probs[q];
    bool s = false;
    if (S.sym_ok) {
      s = true;
      for (int64_t k = 0; k < S.annz && s; ++k) s = P.A_data[k] == P.A_data[S.sym[k]];
    } else if (S.dups) {
      s = csr_symmetric(P.n, P.A_indptr, P.A_indices, P.A_data);
    }
    sym[q] = s ? 1 : 0;
    band[q] = s && !no_band && S.band <= kBandMax && S.nc <= kBandMaxNc &&
              band_lds(S.band) <= kBLdsBytes ? 1 : 0;
  });
  // 4. strategy. A single problem with a large dense coarse operator: the coarse inverse from
  // the device-wide factorisation (dense.hip) and phased cycles, the coarse solve on every CU.
  // Batches holding such problems run phased too (each problem's cycles on its workgroup, the
  // dense coarse solves spread over the CUs; banded problems solve on their own workgroup)
  static const int ext_min = [] {
    const char* e = std::getenv("MLAMG_BATCH_EXT_MIN");
    return e ? std::atoi(e) : kExtCoarseMin;
  }();
  const bool no_ext = std::getenv("MLAMG_BATCH_NO_EXT") != nullptr;
  bool big_dense = false;
  for (int q = 0; q < count; ++q) big_dense = big_dense || (!band[q] && probs[q].n_c > ext_min);
  const bool ext_ok = count == 1 && big_dense && !no_ext;
  const bool phased_batch = count > 1 && big_dense && !no_ext &&
                            !std::getenv("MLAMG_BATCH_NO_PHASED_BATCH");
  const bool phased = (ext_ok || phased_batch) && !std::getenv("MLAMG_BATCH_NO_PHASED");
  // residual in LDS when every problem leaves room for it (phased: r_H, e_H live in the arena)
  bool r_lds = true;
  for (int q = 0; q < count; ++q) {
    const size_t need = (size_t)probs[q].n * 16 + 16 + (phased ? 0 : (size_t)probs[q].n_c * 16) +
                        16 * 1024;
    if (need > kBLdsBytes) r_lds = false;
  }
  const int single = count == 1 ? 1 : 0;
  // 5. shapes for these flags (cached per pattern)
  std::vector<std::shared_ptr<const Shape>> shape(count);
  todo.clear();
  for (int q = 0; q < count; ++q)
    if (rep[q] == q) {
      if (!no_cache) shape[q] = shape_lookup(pat[q].get(), smoother, phased, r_lds, single);
      if (!shape[q]) todo.push_back(q);
    }
  parallel_for((int)todo.size(), [&](int t) {
    const int q = todo[t];
    auto S = analyse_shape(probs[q], pat[q], smoother, phased, r_lds, single);
    if (S->code == MLAMG_OK && !no_cache) shape_insert(S);
    shape[q] = S;
  });
  for (int q = 0; q < count; ++q) shape[q] = shape[rep[q]];
  for (int q = 0; q < count; ++q)
    if (shape[q]->code != MLAMG_OK) {
      set_error(shape[q]->err + " (problem " + std::to_string(q) + ")");
      return shape[q]->code;
    }
  // the dense inverse Cholesky factor where no band is taken and it fits one workgroup's LDS
  std::vector<char> spd(count, 0);
  for (int q = 0; q < count; ++q) spd[q] = sym[q] && !band[q] && shape[q]->chol_fits ? 1 : 0;
  const auto t_analysed = std::chrono::steady_clock::now();
  // ---- layout: each distinct shape's structure once, then every problem's values
  Layout lay;
  const int64_t desc_off = lay.take(sizeof(BDesc) * count);
  size_t lds_setup = 0, lds_cycles = 0, lds_band = 0;
  bool any_band = false;
  for (int q = 0; q < count; ++q) any_band = any_band || band[q];
  struct ShapeOffs {
    int64_t akc, amap, ppc, pmap, ptc, tmap, lev, clev, pkc, gmap, dmap, pkr0;
  };
  std::vector<const Shape*> uniq;
  std::vector<ShapeOffs> uoff;
  std::vector<int> uidx(count, -1);
  for (int q = 0; q < count; ++q) {
    if (rep[q] != q) {
      uidx[q] = uidx[rep[q]];
      continue;
    }
    const Shape& S = *shape[q];
    ShapeOffs o;
    o.akc = lay.take(4 * S.akc.size());
    o.amap = lay.take(4 * S.amap.size());
    o.ppc = lay.take(4 * S.ppc.size());
    o.pmap = lay.take(4 * S.pmap.size());
    o.ptc = lay.take(4 * S.ptc.size());
    o.tmap = lay.take(4 * S.tmap.size());
    o.lev = lay.take(4 * S.lev.size());
    o.clev = lay.take(4 * S.clev.size());
    o.pkc = lay.take(4 * S.pkc.size());
    o.gmap = lay.take(4 * S.gmap.size());
    o.dmap = lay.take(4 * S.dmap.size());
    o.pkr0 = lay.take(4 * S.pkr0.size());
    uidx[q] = (int)uniq.size();
    uniq.push_back(&S);
    uoff.push_back(o);
  }
  for (int q = 0; q < count; ++q) {
    const Shape& L = *shape[q];
    const ShapeOffs& o = uoff[uidx[q]];
    lds_setup = std::max(lds_setup, std::max(L.lds_base, spd[q] ? L.lds_chol : size_t(0)));
    if (band[q]) lds_band = std::max(lds_band, band_lds(pat[q]->band));
    lds_cycles = std::max(lds_cycles, L.lds_cycles);
    const mlamg_amg2v_problem& P = probs[q];
    const int64_t n = P.n;
    BDesc& D = desc[q];
    std::memset(&D, 0, sizeof(D));
    D.n = (int32_t)n;
    D.nc = (int32_t)P.n_c;
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
    D.panel = L.panel;
    D.n_chunks = L.clev.empty() ? 0 : (int32_t)L.clev.size() - 1;
    D.cap = L.cap;
    D.timing = timing ? 1 : 0;
    D.spd = spd[q];
    D.band_ld = band[q] ? pat[q]->band + 1 : 0;
    D.chol_nb = L.chol_nb;
    D.gs_rw = L.gs_rw;
    D.gs_db = L.gs_db;
    D.gs_rp = L.gs_rp;
    D.phased = phased ? 1 : 0;
    D.tol = tol;
    D.omega = jacobi_weight;
    D.ak_col = o.akc;
    D.a_map = o.amap;
    D.pp_col = o.ppc;
    D.p_map = o.pmap;
    D.pt_row = o.ptc;
    D.t_map = o.tmap;
    D.lev_ptr = o.lev;
    D.chunk_lev = o.clev;
    D.pk_col = o.pkc;
    D.g_map = o.gmap;
    D.d_map = o.dmap;
    D.pk_row0 = o.pkr0;
    D.a_raw = lay.take(8 * (size_t)P.A_nnz);
    D.p_raw = lay.take(8 * (size_t)P.P_nnz);
    D.b = lay.take(8 * n);
    D.x0 = lay.take(8 * n);
  }
  // phased: each problem's first coarse-solve block (k_amg2v_coarse), a row per wave
  const int64_t cblk_off = phased ? lay.take(4 * (size_t)(count + 1)) : 0;
  std::vector<int32_t> cblk(count + 1, 0);
  for (int q = 0; q < count; ++q) cblk[q + 1] = cblk[q] + (int32_t)((desc[q].nc + 3) / 4);
  MLAMG_REQUIRE(lds_setup <= kBLdsBytes + 1024 && lds_cycles <= kBLdsBytes + 1024,
                "LDS budget exceeded");
  const size_t in_bytes = lay.off;
  for (int q = 0; q < count; ++q) {
    BDesc& D = desc[q];
    const Shape& L = *shape[q];
    // the packed values, gathered on the device (gather_values)
    D.ak_val = lay.take(8 * L.akc.size());
    D.pp_val = lay.take(8 * L.ppc.size());
    D.pt_val = lay.take(8 * L.ptc.size());
    D.pk_val = lay.take(8 * L.pkc.size());
    D.pk_diag = lay.take(8 * L.pkr0.size());
    D.pk_row = lay.take(4 * L.pkr0.size());
    D.b_lvl = lay.take(8 * L.pkr0.size());
    D.AH = lay.take((size_t)8 * D.nc * D.nc);
    D.AI = lay.take((size_t)8 * D.nc * D.nc);
    D.rg = lay.take(8 * (size_t)D.n);
    D.dinv = lay.take(8 * (size_t)D.n);
    if (D.band_ld > 0) {  // the band solve's lane layouts (band_chol), padded
      D.lc = lay.take((size_t)8 * 64 * (D.nc + 2 * kBandPad));
      D.lr = lay.take((size_t)8 * 64 * (D.nc + 2 * kBandPad));
      D.rinv = lay.take((size_t)8 * (D.nc + 2 * kBandPad));
    }
    if (phased) {
      D.rcg = lay.take(8 * (size_t)D.nc);
      D.eg = lay.take(8 * (size_t)D.nc);
      D.yg = lay.take(8 * (size_t)D.nc);
    }
  }
  const int64_t done_off = phased ? lay.take(sizeof(int32_t)) : 0;
  for (int q = 0; q < count; ++q) desc[q].done_ctr = done_off;
  const size_t out_begin = lay.off;
  for (int q = 0; q < count; ++q) {
    BDesc& D = desc[q];
    D.x_out = lay.take(8 * (size_t)D.n);
    D.err_out = lay.take(8 * (size_t)std::max(max_iter, 1));
    D.stat_out = lay.take(16 + 8 * 8);
  }
  const size_t total = lay.off;
  // a single problem with a large SPD coarse operator takes the device-wide coarse factorisation
  const bool ext_coarse = ext_ok && spd[0];
  if (ext_coarse) desc[0].setup_mode = 1;
  // a phased batch factors its large SPD operators device-wide too, all in one launch sequence.
  // The factor is chosen by the problem's own n_c, as a single call chooses it (the batched and
  // the single device-wide factors run the same code per operator): a problem's results do not
  // depend on the batch it is launched with
  const bool batch_ext = phased && count > 1 && !std::getenv("MLAMG_BATCH_NO_BATCH_EXT");
  if (batch_ext)
    for (int q = 0; q < count; ++q)
      if (spd[q] && desc[q].nc > ext_min) desc[q].setup_mode = 2;
  // ---- pack the inputs into pinned host memory, one copy in
  HostPinned& H = g_batch_host;
  const size_t host_need = std::max(in_bytes, total - out_begin);
  if (H.cap < host_need) {
    if (H.p) (void)hipHostFree(H.p);
    H.p = nullptr;
    H.cap = 0;
    const size_t grow = host_need + host_need / 2;  // geometric: batches of similar size reuse it
    MLAMG_HIP(hipHostMalloc(&H.p, grow, hipHostMallocDefault));
    H.cap = grow;
  }
  char* hb = static_cast<char*>(H.p);
  const auto t_pinned = std::chrono::steady_clock::now();
  std::memcpy(hb + desc_off, desc.data(), sizeof(BDesc) * count);
  if (phased) std::memcpy(hb + cblk_off, cblk.data(), 4 * (size_t)(count + 1));
  auto put = [&](int64_t off, const void* src, size_t bytes) {
    if (bytes) std::memcpy(hb + off, src, bytes);
  };
  const int nu = (int)uniq.size();
  parallel_for(nu + count, [&](int t) {
    if (t < nu) {  // a shape's structure
      const Shape& S = *uniq[t];
      const ShapeOffs& o = uoff[t];
      put(o.akc, S.akc.data(), 4 * S.akc.size());
      put(o.amap, S.amap.data(), 4 * S.amap.size());
      put(o.ppc, S.ppc.data(), 4 * S.ppc.size());
      put(o.pmap, S.pmap.data(), 4 * S.pmap.size());
      put(o.ptc, S.ptc.data(), 4 * S.ptc.size());
      put(o.tmap, S.tmap.data(), 4 * S.tmap.size());
      put(o.lev, S.lev.data(), 4 * S.lev.size());
      put(o.clev, S.clev.data(), 4 * S.clev.size());
      put(o.pkc, S.pkc.data(), 4 * S.pkc.size());
      put(o.gmap, S.gmap.data(), 4 * S.gmap.size());
      put(o.dmap, S.dmap.data(), 4 * S.dmap.size());
      put(o.pkr0, S.pkr0.data(), 4 * S.pkr0.size());
      return;
    }
    const int q = t - nu;  // a problem's values
    const mlamg_amg2v_problem& P = probs[q];
    const BDesc& D = desc[q];
    put(D.a_raw, P.A_data, 8 * (size_t)P.A_nnz);
    put(D.p_raw, P.P_data, 8 * (size_t)P.P_nnz);
    put(D.b, P.b, 8 * (size_t)P.n);
    put(D.x0, P.x0, 8 * (size_t)P.n);
  });
  const auto t_filled = std::chrono::steady_clock::now();
  char* arena = static_cast<char*>(scratch(total, 11));
  MLAMG_REQUIRE(arena, "device arena allocation failed");
  const auto t_packed = std::chrono::steady_clock::now();
  MLAMG_HIP(hipMemcpyAsync(arena, hb, in_bytes, hipMemcpyHostToDevice, s));
  const BDesc* dd = reinterpret_cast<const BDesc*>(arena + desc_off);
  hipLaunchKernelGGL(k_amg2v_setup, dim3((unsigned)count), dim3(kBT), lds_setup, s, dd, arena, 0);
  if (any_band) {  // band factors, then Gauss-Jordan for any that met a non-positive pivot
    hipLaunchKernelGGL(k_amg2v_band, dim3((unsigned)count), dim3(kBT), lds_band, s, dd, arena);
    hipLaunchKernelGGL(k_amg2v_setup, dim3((unsigned)count), dim3(kBT), lds_setup, s, dd, arena, 1);
  }
  if (ext_coarse) {
    const int nc = desc[0].nc;
    const int R = std::max(1, std::min(64, (int)((size_t)128 * 1024 / (8 * (size_t)nc))));
    hipLaunchKernelGGL(k_galerkin_rows, dim3((unsigned)((nc + R - 1) / R)), dim3(256),
                       (size_t)R * nc * 8, s, dd, arena, R);
    // a single call with a large SPD coarse operator: the device-wide inverse Cholesky factor
    // (all CUs) instead of one workgroup's; Gauss-Jordan in the setup kernel when not SPD
    const BDesc& D = desc[0];
    bool spd = false;
    MLAMG_TRY(dense_chol_inverse(reinterpret_cast<double*>(arena + D.AH), D.nc,
                                 reinterpret_cast<double*>(arena + D.AI), &spd, s));
    if (!spd) {
      BDesc& Dh = *reinterpret_cast<BDesc*>(hb + desc_off);
      Dh.setup_mode = 0;
      Dh.spd = 0;
      MLAMG_HIP(hipMemcpyAsync(arena + desc_off, hb + desc_off, sizeof(BDesc),
                               hipMemcpyHostToDevice, s));
      MLAMG_HIP(hipStreamSynchronize(s));
      hipLaunchKernelGGL(k_amg2v_setup, dim3(1), dim3(kBT), lds_setup, s, dd, arena, 0);
    }
  }
  if (batch_ext) {
    std::vector<DenseJob> jobs;
    std::vector<int> who;
    for (int q = 0; q < count; ++q)
      if (desc[q].setup_mode == 2) {
        DenseJob J{};
        J.M = reinterpret_cast<double*>(arena + desc[q].AH);
        J.inv = reinterpret_cast<double*>(arena + desc[q].AI);
        J.n = desc[q].nc;
        jobs.push_back(J);
        who.push_back(q);
      }
    std::unique_ptr<bool[]> ok(new bool[std::max<size_t>(jobs.size(), 1)]);
    MLAMG_TRY(dense_chol_inverse_batch(jobs.data(), (int)jobs.size(), ok.get(), s));
    bool any_failed = false;
    for (size_t j = 0; j < jobs.size(); ++j) any_failed = any_failed || !ok[j];
    if (any_failed) {  // Gauss-Jordan in the setup kernel for those, the others untouched
      BDesc* Dh = reinterpret_cast<BDesc*>(hb + desc_off);
      for (int q = 0; q < count; ++q) Dh[q].setup_mode = 3;
      for (size_t j = 0; j < jobs.size(); ++j)
        if (!ok[j]) {
          Dh[who[j]].setup_mode = 0;
          Dh[who[j]].spd = 0;
        }
      MLAMG_HIP(hipMemcpyAsync(arena + desc_off, hb + desc_off, sizeof(BDesc) * count,
                               hipMemcpyHostToDevice, s));
      MLAMG_HIP(hipStreamSynchronize(s));
      hipLaunchKernelGGL(k_amg2v_setup, dim3((unsigned)count), dim3(kBT), lds_setup, s, dd,
                         arena, 0);
    }
  }
  if (phased) {
    // cycle k = launches A_k (second half of cycle k - 1, first half of cycle k) and B_k (the
    // coarse solve); A_max_iter ends it. Every launch after the one that met the tolerance
    // returns at once; with a tolerance the host queues batches of cycles and reads the done
    // flag of the batch before the one it just queued, so the GPU never waits for the host.
    const bool rp = count == 1 && desc[0].gs_rp != 0;
    const dim3 ga((unsigned)count);
    auto launch_a = [&]() {
      if (r_lds && rp)
        hipLaunchKernelGGL((k_amg2v_cycles<true, true, true>), ga, dim3(kBT), lds_cycles, s, dd,
                           arena);
      else if (r_lds)
        hipLaunchKernelGGL((k_amg2v_cycles<true, true, false>), ga, dim3(kBT), lds_cycles, s, dd,
                           arena);
      else if (rp)
        hipLaunchKernelGGL((k_amg2v_cycles<false, true, true>), ga, dim3(kBT), lds_cycles, s,
                           dd, arena);
      else
        hipLaunchKernelGGL((k_amg2v_cycles<false, true, false>), ga, dim3(kBT), lds_cycles, s,
                           dd, arena);
    };
    const unsigned coarse_blocks = (unsigned)cblk[count];
    const int32_t* cb = reinterpret_cast<const int32_t*>(arena + cblk_off);
    // mode-1 problems (one-workgroup inverse Cholesky factor) need the second, L^-T, pass
    bool two_pass = false;
    for (int q = 0; q < count; ++q)
      two_pass = two_pass || (spd[q] && desc[q].setup_mode == 0);
    MLAMG_HIP(hipMemsetAsync(arena + done_off, 0, sizeof(int32_t), s));
    const int total_a = max_iter + 1;
    // per host thread: two pinned done-count slots and their events (freed at thread exit)
    struct PhaseFlags {
      int32_t* host = nullptr;
      hipEvent_t ev[2] = {nullptr, nullptr};
      ~PhaseFlags() {
        for (auto e : ev)
          if (e) (void)hipEventDestroy(e);
        if (host) (void)hipHostFree(host);
      }
    };
    static thread_local PhaseFlags pf;
    if (!pf.host) {
      MLAMG_HIP(hipHostMalloc(&pf.host, 2 * sizeof(int32_t), hipHostMallocDefault));
      for (auto& e : pf.ev) MLAMG_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    int32_t* flag_host = pf.host;
    hipEvent_t* flag_ev = pf.ev;
    const int32_t* done_dev = reinterpret_cast<const int32_t*>(arena + done_off);
    constexpr int kPhaseBatch = 4;
    int a = 0;
    for (int batch = 0; a < total_a; ++batch) {
      const int na = tol >= 0.0 ? std::min(kPhaseBatch, total_a - a) : total_a - a;
      for (int q = 0; q < na; ++q, ++a) {
        launch_a();
        if (a < max_iter) {
          hipLaunchKernelGGL(k_amg2v_coarse<1>, dim3(coarse_blocks), dim3(256), 0, s, dd, arena,
                             cb, count);
          if (two_pass)
            hipLaunchKernelGGL(k_amg2v_coarse<2>, dim3(coarse_blocks), dim3(256), 0, s, dd,
                               arena, cb, count);
        }
      }
      MLAMG_HIP(hipGetLastError());
      if (tol < 0.0 || a >= total_a) break;
      MLAMG_HIP(hipMemcpyAsync(flag_host + (batch & 1), done_dev, sizeof(int32_t),
                               hipMemcpyDeviceToHost, s));
      MLAMG_HIP(hipEventRecord(flag_ev[batch & 1], s));
      if (batch > 0) {
        MLAMG_HIP(hipEventSynchronize(flag_ev[(batch - 1) & 1]));
        if (flag_host[(batch - 1) & 1] >= count) break;
      }
    }
  } else if (r_lds) {
    hipLaunchKernelGGL((k_amg2v_cycles<true, false, false>), dim3((unsigned)count), dim3(kBT),
                       lds_cycles, s, dd, arena);
  } else {
    hipLaunchKernelGGL((k_amg2v_cycles<false, false, false>), dim3((unsigned)count), dim3(kBT),
                       lds_cycles, s, dd, arena);
  }
  MLAMG_HIP(hipGetLastError());
  // the host staging buffer is reused for the outputs: the copy-in above completed before the
  // kernel (same stream), and the copy-out below is ordered after it
  MLAMG_HIP(hipMemcpyAsync(hb, arena + out_begin, total - out_begin, hipMemcpyDeviceToHost, s));
  MLAMG_HIP(hipStreamSynchronize(s));
  if (timing) {
    const auto t_done = std::chrono::steady_clock::now();
    auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    std::fprintf(stderr,
                 "[amg2v_batch] %d problems: host %.3f ms (analysis %.3f, layout + pinned buffer "
                 "%.3f, fill %.3f, device arena %.3f), copy in + kernels + copy out %.3f ms "
                 "(%.2f MB in)\n",
                 count, ms(t_begin, t_packed), ms(t_begin, t_analysed), ms(t_analysed, t_pinned),
                 ms(t_pinned, t_filled), ms(t_filled, t_packed), ms(t_packed, t_done),
                 in_bytes * 1e-6);
  }
  for (int q = 0; q < count; ++q) {
    mlamg_amg2v_problem& P = probs[q];
    const BDesc& D = desc[q];
    const int32_t* st = reinterpret_cast<const int32_t*>(hb + (D.stat_out - out_begin));
    P.iters_out = st[0];
    P.status_out = st[1];
    if (timing) {
      const int64_t* ts = reinterpret_cast<const int64_t*>(st + 4);
      std::fprintf(stderr,
                   "[amg2v_batch] problem %d n=%lld n_c=%lld iters=%d: galerkin %.3f ms, inverse "
                   "(%s) %.3f ms (panels %.3f, updates %.3f), smoothing (%s) %.3f ms, rest of "
                   "cycles %.3f ms (coarse solve %.3f ms)\n",
                   q, (long long)P.n, (long long)P.n_c, st[0], ts[0] * 1e-5,
                   st[2] == 2 ? "band cholesky" : st[2] == 1 ? "cholesky" : "gauss-jordan",
                   (ts[1] + ts[4] + ts[5]) * 1e-5, ts[4] * 1e-5, ts[5] * 1e-5,
                   D.gs_rw ? "one wave" : "workgroup", ts[2] * 1e-5, (ts[3] + ts[6]) * 1e-5,
                   ts[6] * 1e-5);
    }
    std::memcpy(P.x_out, hb + (D.x_out - out_begin), 8 * (size_t)P.n);
    if (max_iter > 0) std::memcpy(P.err_out, hb + (D.err_out - out_begin), 8 * (size_t)st[0]);
  }
  return MLAMG_OK;
}

}  // extern "C"
