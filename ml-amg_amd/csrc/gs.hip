// Lexicographic Gauss-Seidel sweeps, pyamg semantics:
//   gauss_seidel (the smoother of the reference driver, ns/lib/multigrid.py:175,184):
//     for i in 0..n-1: rsum = sum_{j != i} A_ij x_j (stored order); diag = A_ii (last one);
//                      if diag != 0: x_i = (b_i - rsum) / diag
//   block_gauss_seidel with 1 x 1 blocks (the pre/post smoother and the candidate improvement of
//   pyamg's smoothed_aggregation_solver, which ns/preconditioner/PyAMG.py:94 builds; amg_core
//   block_gauss_seidel): rsum = b_i; rsum -= (0 + A_ij x_j) for j != i in stored order;
//     x_i = 0 + Dinv_i rsum, Dinv_i = pinv(A_ii) = 1 / A_ii (0 when A_ii = 0)
//   sweep 'forward' (rows 0..n-1), 'backward' (n-1..0) or 'symmetric' (forward, then backward,
//   per iteration).
// Row i reads x_j of rows swept before it after their update and the others before theirs.
// Level scheduling keeps exactly that order on the GPU: level(i) = 1 + max level(j) over rows j
// swept before i and coupled to i in either direction (a_ij or a_ji nonzero), so every row of a
// level sees final values of all earlier-coupled rows and old values of all later-coupled rows;
// rows inside a level are independent. Results are therefore bit for bit those of the sequential
// sweep.
#include "common.hpp"

#include <chrono>
#include <cstdio>
#include <cstdlib>

struct mlamg_gs {
  const mlamg_csr* A = nullptr;
  bool block = false;        // block_gauss_seidel arithmetic (pk_diag then holds Dinv)
  bool backward = false;     // rows swept n-1..0
  mlamg_gs* bwd = nullptr;   // symmetric sweep: the backward schedule of the same operator
  int32_t n_levels = 0;
  int32_t max_level_rows = 0;
  std::vector<int32_t> level_ptr;  // host
  int32_t* d_level_ptr = nullptr;  // device copy
  int32_t* rows = nullptr;         // device, rows grouped by level (ascending within a level)
  // level-ordered copy for the pipelined one-workgroup sweep (k_gs_pipe): position p = the p-th
  // row of `rows`; its off-diagonal entries in stored order in slots pk_col/pk_val[p*K .. p*K+K)
  // (column -1 pads), its diagonal (the last stored one, as the sequential sweep takes it; 0.0
  // when absent) in pk_diag[p]; b_lvl[p] = b[rows[p]] is refreshed per sweep. Every load of a
  // level's structure is then independent of the others. Snapshot of A at mlamg_gs_create.
  int32_t pk_k = 0;  // slots per row (4 or 8), 0 = no packed copy
  int32_t* pk_col = nullptr;
  double* pk_val = nullptr;
  double* pk_diag = nullptr;
  double* b_lvl = nullptr;
  int32_t max_off = 0;  // longest off-diagonal count
  // level-ordered (row, first entry, length, 0) per position for the wave-cooperative sweep
  // (rows with more than 8 off-diagonals, at most 128 entries per row; nullptr: none)
  int32_t* wpos = nullptr;
  int32_t max_len = 0;
  // ring sweep (k_gs_ring): slot columns classified earlier (ring position) / later (-(c + 2))
  int32_t* rcol = nullptr;
  double* rpv = nullptr;  // per slot: a, the later-swept product, or 0 (k_gs_ring_prep)
  uint16_t* rcode = nullptr;  // per slot: ring slot / kGsRingLater / kGsRingPad
  // the long-row ring sweep (k_gs_wring): SPAN slots per position, step table, ring
  int32_t wr_lpr = 0, wr_epl = 0, wr_steps = 0, wr_log2 = 0;
  int32_t* wr_code = nullptr;
  double* wr_pv = nullptr;
  int32_t* wr_len = nullptr;
  double* wr_d = nullptr;
  int2* wr_st = nullptr;
  size_t wr_lds = 0;
  double* rxl = nullptr;      // the sweep's values in level order
  int32_t ring_log2_r = 0;
  // windowed one-wave sweep (k_gs_win): x by level-order position in an LDS ring of 2^ring_log2
  // slots; wcol = the packed columns as positions (pads -1); chunks of levels staged into two
  // LDS buffers of win_cap + 1 positions; win_w = the widest level distance of a coupling
  int32_t win_rw = 0;  // 64-row slots per level (0: no windowed sweep)
  int32_t ring_log2 = 0, win_cap = 0, win_w = 0, n_chunks = 0;
  int32_t* wcol = nullptr;
  int32_t* d_clev = nullptr;  // the chunk plan (8 ints per chunk) + level starts
  double* win_xl = nullptr;  // x in level order (the window's old-x source)
  size_t win_lds = 0;
};

namespace mlamg {

// the two row updates: gauss_seidel (BLK false) sums the off-diagonal products from +0.0 and
// divides b_i minus the sum by the diagonal; block_gauss_seidel (BLK true) subtracts each product
// (gemm's 0 + a x) from b_i and multiplies by Dinv_i (gemm's 0 + d r)
template <bool BLK>
__device__ __forceinline__ double gs_init(double bi) { return BLK ? bi : 0.0; }
template <bool BLK>
__device__ __forceinline__ double gs_acc(double s, double a, double xj) {
  return BLK ? s - (0.0 + a * xj) : s + a * xj;
}
// d: the diagonal (gauss_seidel) or Dinv (block)
template <bool BLK>
__device__ __forceinline__ double gs_fin(double s, double bi, double d) {
  return BLK ? 0.0 + d * s : (bi - s) / d;
}
// gauss_seidel leaves a zero-diagonal row alone; block_gauss_seidel updates every row
template <bool BLK>
__device__ __forceinline__ bool gs_upd(double d) { return BLK || d != 0.0; }

template <bool BLK>
__device__ __forceinline__ void gs_row(const int32_t* __restrict__ ip,
                                       const int32_t* __restrict__ ij,
                                       const double* __restrict__ ax, int32_t i, double* x,
                                       const double* __restrict__ b) {
  double s = gs_init<BLK>(b[i]), diag = 0.0;
  for (int k = ip[i]; k < ip[i + 1]; ++k) {
    const int32_t j = ij[k];
    if (j == i) diag = ax[k];
    else s = gs_acc<BLK>(s, ax[k], x[j]);
  }
  if (BLK) diag = diag != 0.0 ? 1.0 / diag : 0.0;
  if (gs_upd<BLK>(diag)) x[i] = gs_fin<BLK>(s, b[i], diag);
}

template <bool BLK>
__global__ __launch_bounds__(256) void k_gs_level(const int32_t* __restrict__ ip,
                                                  const int32_t* __restrict__ ij,
                                                  const double* __restrict__ ax,
                                                  const int32_t* __restrict__ rows, int32_t cnt,
                                                  double* x, const double* __restrict__ b,
                                                  const int32_t* done) {
  if (done && *done) return;
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= cnt) return;
  gs_row<BLK>(ip, ij, ax, rows[t], x, b);
}

// The whole sweep in one workgroup: levels in order, a barrier between consecutive levels
// (workgroup-scope visibility of the x updates). For operators whose levels are narrow, where
// one launch per level would make the sweep launch-bound.
constexpr int kGsBlock = 1024;
constexpr int kGsBlockMaxLevelRows = 8 * kGsBlock;

template <bool BLK>
__global__ __launch_bounds__(kGsBlock) void k_gs_block(const int32_t* __restrict__ ip,
                                                       const int32_t* __restrict__ ij,
                                                       const double* __restrict__ ax,
                                                       const int32_t* __restrict__ rows,
                                                       const int32_t* __restrict__ lptr,
                                                       int32_t n_levels, int iterations, double* x,
                                                       const double* __restrict__ b,
                                                       const int32_t* done) {
  if (done && *done) return;
  for (int it = 0; it < iterations; ++it) {
    for (int32_t l = 0; l < n_levels; ++l) {
      const int32_t a = lptr[l], z = lptr[l + 1];
      for (int32_t t = a + (int32_t)threadIdx.x; t < z; t += kGsBlock) gs_row<BLK>(ip, ij, ax, rows[t], x, b);
      __syncthreads();
    }
  }
}

// One workgroup, rows with many off-diagonals (coarse Galerkin operators: 10-120 entries): LPR
// lanes per row (8, or 16 past 64 entries), EPL entries per lane, 1024 / LPR rows per pass. A row's lanes gather their entries'
// x values in parallel and leave the products (and the diagonal) in LDS in stored order; the
// row's first lane then folds them in that order — the same products, in the same order, as
// gs_row — and stores x_i. The next level's first pass (position info from the level-ordered
// `wpos` = (row, first entry, length), then its columns and values: none of it depends on x) is
// loaded while this level computes, so a level's critical path is its x gathers, the fold and
// the barrier.
constexpr int kGsWaveBlock = 1024;
constexpr int kGsWaveMaxLPR = 16;  // lanes per row: 8 for rows of <= 64 entries (128 rows per
                                   // pass), 16 up to 128 entries

template <int EPL>
struct GsWaveRow {
  int32_t row, len;
  double bi;
  int32_t col[EPL];
  double val[EPL];
};

// a position's (row, first entry, length): w.x < 0 marks no row
__device__ __forceinline__ int4 gs_wave_pos(int32_t t, int32_t z, const int4* __restrict__ wpos) {
  return t < z ? wpos[t] : make_int4(-1, 0, 0, 0);
}

// the row's b and entries from its position info
template <int LPR, int EPL>
__device__ __forceinline__ void gs_wave_entries(GsWaveRow<EPL>& r, int4 w, int lane,
                                                const int32_t* __restrict__ ij,
                                                const double* __restrict__ ax,
                                                const double* __restrict__ b) {
  const bool live = w.x >= 0;
  r.row = w.x;  // an empty row still updates (block_gauss_seidel: x_i = 0 + 0 b_i)
  r.len = w.z;
  r.bi = live ? b[w.x] : 0.0;
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    const int k = lane + e * LPR;
    const bool ok = k < w.z;
    r.col[e] = ok ? ij[w.y + k] : -1;
    r.val[e] = ok ? ax[w.y + k] : 0.0;
  }
}

template <int LPR, int EPL>
__device__ __forceinline__ void gs_wave_load(GsWaveRow<EPL>& r, int32_t t, int32_t z, int lane,
                                             const int4* __restrict__ wpos,
                                             const int32_t* __restrict__ ij,
                                             const double* __restrict__ ax,
                                             const double* __restrict__ b) {
  gs_wave_entries<LPR, EPL>(r, gs_wave_pos(t, z, wpos), lane, ij, ax, b);
}

template <int LPR, int EPL, bool BLK>
__global__ __launch_bounds__(kGsWaveBlock) void k_gs_wave(const int4* __restrict__ wpos,
                                                         const int32_t* __restrict__ ij,
                                                         const double* __restrict__ ax,
                                                         const int32_t* __restrict__ lptr,
                                                         int32_t n_levels, int iterations,
                                                         double* x, const double* __restrict__ b,
                                                         const int32_t* done) {
  constexpr int ROWS = kGsWaveBlock / LPR;  // rows per pass
  constexpr int SPAN = LPR * EPL;             // LDS slots per row
  __shared__ double pv[ROWS * SPAN];
  __shared__ int32_t pc[ROWS * SPAN];
  if (done && *done) return;
  const int tid = threadIdx.x;
  const int g = tid / LPR, lane = tid % LPR;
  double* gv = pv + g * SPAN;
  int32_t* gc = pc + g * SPAN;
  for (int it = 0; it < iterations; ++it) {
    GsWaveRow<EPL> cur, nxt;
    gs_wave_load<LPR, EPL>(cur, lptr[0] + g, lptr[1], lane, wpos, ij, ax, b);
    // positions two levels ahead, entries one level ahead (the entries need the positions)
    int4 w1 = n_levels > 1 ? gs_wave_pos(lptr[1] + g, lptr[2], wpos) : make_int4(-1, 0, 0, 0);
    int4 w2 = make_int4(-1, 0, 0, 0);
    for (int32_t l = 0; l < n_levels; ++l) {
      const int32_t a = lptr[l], z = lptr[l + 1];
      // passes over the level's rows (uniform for the workgroup: the LDS fences are per wave)
      for (int32_t t0 = a; t0 < z; t0 += ROWS) {
        if (t0 > a) gs_wave_load<LPR, EPL>(cur, t0 + g, z, lane, wpos, ij, ax, b);
        double p[EPL];
#pragma unroll
        for (int e = 0; e < EPL; ++e) {
          const int32_t j = cur.col[e];
          const double xj = (j >= 0 && j != cur.row) ? x[j] : 0.0;
          p[e] = j == cur.row ? cur.val[e] : (BLK ? 0.0 + cur.val[e] * xj : cur.val[e] * xj);
        }
        if (t0 == a) {
          if (l + 1 < n_levels) gs_wave_entries<LPR, EPL>(nxt, w1, lane, ij, ax, b);
          if (l + 2 < n_levels) w2 = gs_wave_pos(lptr[l + 2] + g, lptr[l + 3], wpos);
        }
#pragma unroll
        for (int e = 0; e < EPL; ++e) {
          const int k = lane + e * LPR;
          gv[k] = p[e];
          gc[k] = cur.col[e];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane == 0 && cur.row >= 0) {
          double s = gs_init<BLK>(cur.bi), diag = 0.0;
          int k = 0;
          // 8 LDS reads in flight, then the 8 ordered steps
          for (; k + 8 <= cur.len; k += 8) {
            double v[8];
            int32_t c[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              v[u] = gv[k + u];
              c[u] = gc[k + u];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              if (c[u] == cur.row) diag = v[u];
              else s = BLK ? s - v[u] : s + v[u];
            }
          }
          for (; k < cur.len; ++k) {
            const double v = gv[k];
            if (gc[k] == cur.row) diag = v;
            else s = BLK ? s - v : s + v;
          }
          if (BLK) diag = diag != 0.0 ? 1.0 / diag : 0.0;
          if (gs_upd<BLK>(diag)) x[cur.row] = gs_fin<BLK>(s, cur.bi, diag);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
      __syncthreads();
      cur = nxt;
      w1 = w2;
    }
  }
}

// Pipelined one-workgroup sweep for narrow schedules (every level <= R * 1024 rows, every row
// <= K = 4 or 8 off-diagonals): the level-ordered structure (row id, diagonal, b, columns,
// values) of level l+1 is loaded while level l computes, so a level's critical path is only
// its x gathers (which depend on the level before), the ordered sum, the store and the barrier.
// Same products, same order, same division as gs_row: bitwise the sequential sweep.
template <int R, int K>
struct GsRows {
  int32_t row[R];
  double diag[R], bi[R];
  int32_t col[R][K];
  double val[R][K];
};

// position p's structure: independent loads only (no pointer chasing), one round trip
template <int R, int K>
__device__ __forceinline__ void gs_pipe_load(GsRows<R, K>& q, int32_t a, int32_t z,
                                             const int32_t* __restrict__ rows,
                                             const int32_t* __restrict__ pcol,
                                             const double* __restrict__ pval,
                                             const double* __restrict__ pdiag,
                                             const double* __restrict__ blvl) {
#pragma unroll
  for (int u = 0; u < R; ++u) {
    const int32_t p = a + (int32_t)threadIdx.x + u * kGsBlock;
    const bool ok = p < z;
    q.row[u] = ok ? rows[p] : -1;
    q.diag[u] = ok ? pdiag[p] : 0.0;
    q.bi[u] = ok ? blvl[p] : 0.0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      q.col[u][k] = ok ? pcol[(int64_t)p * K + k] : -1;
      q.val[u][k] = ok ? pval[(int64_t)p * K + k] : 0.0;
    }
  }
}

template <int R, int K, bool BLK>
__global__ __launch_bounds__(kGsBlock) void k_gs_pipe(const int32_t* __restrict__ rows,
                                                      const int32_t* __restrict__ lptr,
                                                      int32_t n_levels,
                                                      const int32_t* __restrict__ pcol,
                                                      const double* __restrict__ pval,
                                                      const double* __restrict__ pdiag,
                                                      const double* __restrict__ blvl,
                                                      int iterations, double* x,
                                                      const int32_t* done) {
  if (done && *done) return;
  for (int it = 0; it < iterations; ++it) {
    GsRows<R, K> cur;
    gs_pipe_load<R, K>(cur, lptr[0], lptr[1], rows, pcol, pval, pdiag, blvl);
    for (int32_t l = 0; l < n_levels; ++l) {
      // this level's x gathers first (they read the previous level's updates) ...
      double xv[R][K];
#pragma unroll
      for (int u = 0; u < R; ++u)
#pragma unroll
        for (int k = 0; k < K; ++k) xv[u][k] = cur.col[u][k] >= 0 ? x[cur.col[u][k]] : 0.0;
      // ... then the next level's structure (independent of x) in flight meanwhile
      GsRows<R, K> nxt;
      if (l + 1 < n_levels)
        gs_pipe_load<R, K>(nxt, lptr[l + 1], lptr[l + 2], rows, pcol, pval, pdiag, blvl);
#pragma unroll
      for (int u = 0; u < R; ++u) {
        if (cur.row[u] < 0) continue;
        double rsum = gs_init<BLK>(cur.bi[u]);
#pragma unroll
        for (int k = 0; k < K; ++k)
          if (cur.col[u][k] >= 0) rsum = gs_acc<BLK>(rsum, cur.val[u][k], xv[u][k]);
        if (gs_upd<BLK>(cur.diag[u]))
          x[cur.row[u]] = gs_fin<BLK>(rsum, cur.bi[u], cur.diag[u]);
      }
      __syncthreads();
      if (l + 1 < n_levels) cur = nxt;
    }
  }
}

// Levels of 513..1024 rows with <= 4 off-diagonals (2-D five-point grids up to 1024^2): the
// pipelined walk with the x values of the last W levels in an LDS ring indexed by level-order
// position, W = the widest level distance of a coupling to an earlier level. A slot's column is
// host-classified: a row swept earlier (its updated value: the ring) or later (its old value,
// which nothing writes before the slot's own row is swept). The later-swept slots' products
// (0 + a x_old for block_gauss_seidel, a x_old for gauss_seidel: the very operation the sweep would
// do, so the same bits) are formed before the sweep by a parallel pass (k_gs_ring_prep), which also
// stores the old x of a zero-diagonal gauss_seidel row in place of its b. The sweep's loads thus
// depend on nothing the sweep computes: each level's structure goes out kGsRingSets - 1 levels
// ahead, all loads unconditional (positions past a level's end clamped to the last one and
// selected away), the level starts in LDS, and the register sets rotate by unrolling, not by
// copies (a copy of a register with a load in flight, or a branch join, makes the compiler wait
// for every outstanding load: that had put one or two memory round trips on each level's critical
// path, 2.5 us a level at 1024^2). Same products, same order, same division as gs_row.
constexpr int kGsRingK = 4;
constexpr int kGsRingSets = 6;                // levels in flight + 1
constexpr size_t kGsRingLdsMax = 150 * 1024;  // the ring, its sink slot and the level starts
constexpr uint32_t kGsRingPad = 0xFFFF, kGsRingLater = 0xFFFE;  // the 16-bit slot codes
struct GsRingRow {
  int32_t pos;  // unclamped
  bool ok;      // pos inside its level
  double diag, bi;
  uint2 code;  // 4 x 16 bits: the ring slot of an earlier-swept column, kGsRingLater, kGsRingPad
  double pv[kGsRingK];
};

template <bool BLK>
__device__ __forceinline__ double gs_prod(double a, double xj) {
  return BLK ? 0.0 + a * xj : a * xj;
}
template <bool BLK>
__device__ __forceinline__ double gs_acc_prod(double s, double t) {
  return BLK ? s - t : s + t;
}

// pv[p, k] = a (earlier-swept column: multiplied in the sweep), the product with the old x
// (later-swept), 0 (pad); blvl[p] = b[row], or x[row] for a zero-diagonal gauss_seidel row
template <bool BLK>
__global__ void k_gs_ring_prep(const int32_t* __restrict__ rows, int64_t n,
                               const int32_t* __restrict__ rcol, const double* __restrict__ pval,
                               const double* __restrict__ pdiag, const double* __restrict__ b,
                               const double* __restrict__ x, double* __restrict__ pv,
                               double* __restrict__ blvl, const int32_t* done) {
  if (done && *done) return;
  const int64_t p = blockIdx.x * 256ll + threadIdx.x;
  if (p >= n) return;
  const int32_t i = rows[p];
  blvl[p] = (!BLK && pdiag[p] == 0.0) ? x[i] : b[i];
#pragma unroll
  for (int k = 0; k < kGsRingK; ++k) {
    const int32_t c = rcol[p * kGsRingK + k];
    const double a = pval[p * kGsRingK + k];
    pv[p * kGsRingK + k] = c >= 0 ? a : (c == -1 ? 0.0 : gs_prod<BLK>(a, x[-(c + 2)]));
  }
}

__device__ __forceinline__ void gs_ring_struct(GsRingRow& q, int32_t a, int32_t z, int32_t last,
                                               const uint2* __restrict__ rcode,
                                               const double* __restrict__ pv,
                                               const double* __restrict__ pdiag,
                                               const double* __restrict__ blvl) {
  const int32_t p = a + (int32_t)threadIdx.x;
  q.ok = p < z;
  q.pos = p;
  const int64_t pc = q.ok ? p : last;
  q.diag = pdiag[pc];
  q.bi = blvl[pc];
  q.code = rcode[pc];
  const double2 v01 = *reinterpret_cast<const double2*>(pv + pc * kGsRingK);
  const double2 v23 = *reinterpret_cast<const double2*>(pv + pc * kGsRingK + 2);
  q.pv[0] = v01.x;
  q.pv[1] = v01.y;
  q.pv[2] = v23.x;
  q.pv[3] = v23.y;
}

// the row's new value into the ring and, in level order, into xl (a zero-diagonal gauss_seidel
// row's bi holds its old x: that is its value)
template <bool BLK>
__device__ __forceinline__ void gs_ring_row(const GsRingRow& q, double* ring, int32_t RM,
                                            double* __restrict__ xl) {
  const uint32_t c[4] = {q.code.x & 0xFFFFu, q.code.x >> 16, q.code.y & 0xFFFFu, q.code.y >> 16};
  double rsum = gs_init<BLK>(q.bi);
#pragma unroll
  for (int k = 0; k < kGsRingK; ++k) {
    const double r = ring[c[k] & (uint32_t)RM];
    const double t = c[k] < kGsRingLater ? gs_prod<BLK>(q.pv[k], r) : q.pv[k];
    const double u = gs_acc_prod<BLK>(rsum, t);
    rsum = c[k] != kGsRingPad ? u : rsum;
  }
  const double xi = gs_upd<BLK>(q.diag) ? gs_fin<BLK>(rsum, q.bi, q.diag) : q.bi;
  ring[q.ok ? (q.pos & RM) : RM + 1] = xi;  // slot RM + 1: the sink of the clamped lanes
  if (q.ok) xl[q.pos] = xi;
}

template <bool BLK>
__global__ __launch_bounds__(kGsBlock) void k_gs_ring(const int32_t* __restrict__ lptr,
                                                      int32_t n_levels,
                                                      const uint2* __restrict__ rcode,
                                                      const double* __restrict__ pv,
                                                      const double* __restrict__ pdiag,
                                                      const double* __restrict__ blvl,
                                                      int ring_log2, double* __restrict__ xl,
                                                      const int32_t* done) {
  extern __shared__ double ring[];  // 2^ring_log2 slots, the sink slot, then the level starts
  if (done && *done) return;
  const int32_t RM = (1 << ring_log2) - 1;
  int32_t* lp = reinterpret_cast<int32_t*>(ring + (RM + 2));
  for (int i = threadIdx.x; i <= n_levels; i += kGsBlock) lp[i] = lptr[i];
  __syncthreads();
  const int32_t nl = n_levels, last = lp[nl] - 1;
  auto lvl = [&](GsRingRow& q, int32_t l) {  // level l's structure (l >= nl: no row)
    const int32_t a = lp[l < nl ? l : nl], z = lp[l + 1 < nl ? l + 1 : nl];
    gs_ring_struct(q, a, z, last, rcode, pv, pdiag, blvl);
  };
  constexpr int NS = kGsRingSets;
  GsRingRow S[NS];
#pragma unroll
  for (int u = 0; u < NS - 1; ++u) lvl(S[u], u);
  // step l: level l + NS - 1's structure goes out (into the set level l - 1 used), level l is
  // swept; the steps past the last level sweep no row
  for (int32_t l = 0; l < nl; l += NS) {
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      lvl(S[(u + NS - 1) % NS], l + u + NS - 1);
      gs_ring_row<BLK>(S[u], ring, RM, xl);
      __syncthreads();
    }
  }
}

// Rows longer than 8 off-diagonals (Galerkin levels; the wave-cooperative sweep's rows) with the
// ring scheme of k_gs_ring: LPR lanes per row, each holding EPL slots of a level-ordered copy
// padded to SPAN = LPR EPL slots per position (no pointer chasing: a step's loads depend on the
// step index alone). Slot codes are fixed at setup: >= 0 the ring slot of an earlier-swept column
// at most Wr levels back, <= kGsWringFar - p an earlier-swept column further back (its value is
// read from xl at position p, two steps ahead: written at least Wr > NS levels before), or
// later-swept / diagonal / pad. The slots' values are formed before each sweep by
// k_gs_wring_prep (the later-swept products, the others' matrix values); the lanes form the
// earlier-swept products and the row's first lane folds them in stored order, as k_gs_wave does.
// A step is up to 1024 / LPR rows of one level (host table); the register sets of NS steps rotate
// by unrolling. Values go to xl in level order (one scatter after the sweep).
constexpr int32_t kGsWringPad = -1, kGsWringLater = -2, kGsWringDiag = -3, kGsWringFar = -16;
constexpr size_t kGsWringLdsMax = 150 * 1024;
template <int EPL>
constexpr int gs_wring_sets() {
  return 5;
}
// four slots per lane: 512-thread workgroups (two waves per SIMD: 256 VGPRs for the five sets)
template <int EPL>
constexpr int gs_wring_threads() {
  return EPL <= 2 ? 1024 : 512;
}

template <bool BLK>
__global__ void k_gs_wring_prep(const int32_t* __restrict__ rows, int64_t n,
                                const int32_t* __restrict__ ip, const int32_t* __restrict__ ij,
                                const double* __restrict__ ax, const int32_t* __restrict__ code,
                                int span, const double* __restrict__ b,
                                const double* __restrict__ x, double* __restrict__ pv,
                                double* __restrict__ blvl, double* __restrict__ dlvl,
                                const int32_t* done) {
  if (done && *done) return;
  const int64_t p = blockIdx.x * 256ll + threadIdx.x;
  if (p >= n) return;
  const int32_t i = rows[p], k0 = ip[i], len = ip[i + 1] - k0;
  double diag = 0.0;
  for (int k = 0; k < len; ++k) {
    const int32_t c = code[p * span + k];
    const double a = ax[k0 + k];
    pv[p * span + k] = c == kGsWringLater ? gs_prod<BLK>(a, x[ij[k0 + k]]) : a;
    if (c == kGsWringDiag) diag = a;  // the last stored diagonal entry counts
  }
  blvl[p] = (!BLK && diag == 0.0) ? x[i] : b[i];
  dlvl[p] = BLK ? (diag != 0.0 ? 1.0 / diag : 0.0) : diag;
}

template <int EPL>
struct GsWringRow {
  int32_t pos, len;
  bool ok;
  double bi, dg;
  int32_t code[EPL];
  double pv[EPL], xf[EPL];
};

template <int LPR, int EPL, bool BLK>
__global__ __launch_bounds__(gs_wring_threads<EPL>()) void k_gs_wring(const int2* __restrict__ steps, int32_t n_steps,
                                                   int32_t last, const int32_t* __restrict__ code,
                                                   const double* __restrict__ pv,
                                                   const int32_t* __restrict__ plen,
                                                   const double* __restrict__ blvl,
                                                   const double* __restrict__ dlvl,
                                                   int ring_log2, double* xl,
                                                   const int32_t* done) {
  constexpr int TPB = gs_wring_threads<EPL>();
  constexpr int ROWS = TPB / LPR, SPAN = LPR * EPL, NS = gs_wring_sets<EPL>();
  extern __shared__ double lds[];  // ring (2^ring_log2 + 2) | products | diag flags | steps
  if (done && *done) return;
  const int32_t RM = (1 << ring_log2) - 1;
  double* ring = lds;
  double* gv = ring + (RM + 3);
  uint16_t* gc = reinterpret_cast<uint16_t*>(gv + ROWS * SPAN);
  int2* st = reinterpret_cast<int2*>(gc + ROWS * SPAN + 4);
  for (int i = threadIdx.x; i < n_steps; i += TPB) st[i] = steps[i];
  __syncthreads();
  const int g = threadIdx.x / LPR, lane = threadIdx.x % LPR;
  auto load = [&](GsWringRow<EPL>& q, int32_t t) {  // step t's structure (t >= n_steps: none)
    const int2 d = st[t < n_steps ? t : n_steps - 1];
    q.ok = t < n_steps && g < d.y;
    q.pos = d.x + g;
    const int64_t pc = q.ok ? q.pos : last;
    q.len = plen[pc];
    q.bi = blvl[pc];
    q.dg = dlvl[pc];
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
      q.code[e] = code[pc * SPAN + lane + e * LPR];
      q.pv[e] = pv[pc * SPAN + lane + e * LPR];
    }
  };
  auto gather = [&](GsWringRow<EPL>& q) {  // the far columns' values (needs the codes)
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
      const int32_t c = q.code[e];
      q.xf[e] = xl[c <= kGsWringFar ? kGsWringFar - c : 0];
    }
  };
  double* myv = gv + g * SPAN;
  uint16_t* myc = gc + g * SPAN;
  auto sweep = [&](const GsWringRow<EPL>& q) {
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
      const int32_t c = q.code[e];
      const double r = ring[c & RM];
      const bool near = c >= 0, far = c <= kGsWringFar;
      myv[lane + e * LPR] = (near || far) ? gs_prod<BLK>(q.pv[e], near ? r : q.xf[e]) : q.pv[e];
      myc[lane + e * LPR] = (uint16_t)(c == kGsWringDiag);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (lane == 0 && q.ok) {
      double sum = gs_init<BLK>(q.bi);
      int k = 0;
      for (; k + 8 <= q.len; k += 8) {  // 8 LDS reads in flight, then the 8 ordered steps
        double v[8];
        uint32_t dflag[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          v[u] = myv[k + u];
          dflag[u] = myc[k + u];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (!dflag[u]) sum = gs_acc_prod<BLK>(sum, v[u]);
      }
      for (; k < q.len; ++k)
        if (!myc[k]) sum = gs_acc_prod<BLK>(sum, myv[k]);
      const double xi = gs_upd<BLK>(q.dg) ? gs_fin<BLK>(sum, q.bi, q.dg) : q.bi;
      ring[q.pos & RM] = xi;
      xl[q.pos] = xi;
    }
    __syncthreads();
  };
  // step t: step t + NS - 1's structure and step t + NS - 3's far values go out, step t is swept
  GsWringRow<EPL> S[NS];
#pragma unroll
  for (int u = 0; u < NS - 1; ++u) load(S[u], u);
  gather(S[0]);
  gather(S[1]);
  for (int32_t t = 0; t < n_steps; t += NS) {
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      load(S[(u + NS - 1) % NS], t + u + NS - 1);
      gather(S[(u + 2) % NS]);
      sweep(S[u]);
    }
  }
}

// Small systems (n <= kGsLdsMax): the same pipelined walk with x held in LDS for the whole sweep
// (x loaded once, written back once): a level's gathers and its updates are LDS accesses, so a
// level costs an LDS round trip and a barrier instead of a global-memory round trip.
constexpr int kGsLdsMax = 8192;  // 64 KB of x: within the default dynamic-LDS limit

template <int K, bool BLK>
__global__ __launch_bounds__(kGsBlock) void k_gs_lds(const int32_t* __restrict__ rows,
                                                     const int32_t* __restrict__ lptr,
                                                     int32_t n_levels, int64_t n,
                                                     const int32_t* __restrict__ pcol,
                                                     const double* __restrict__ pval,
                                                     const double* __restrict__ pdiag,
                                                     const double* __restrict__ blvl,
                                                     int iterations, double* x,
                                                     const int32_t* done) {
  extern __shared__ double xs[];
  if (done && *done) return;
  for (int64_t i = threadIdx.x; i < n; i += kGsBlock) xs[i] = x[i];
  __syncthreads();
  for (int it = 0; it < iterations; ++it) {
    GsRows<1, K> cur;
    gs_pipe_load<1, K>(cur, lptr[0], lptr[1], rows, pcol, pval, pdiag, blvl);
    for (int32_t l = 0; l < n_levels; ++l) {
      GsRows<1, K> nxt;
      if (l + 1 < n_levels)
        gs_pipe_load<1, K>(nxt, lptr[l + 1], lptr[l + 2], rows, pcol, pval, pdiag, blvl);
      if (cur.row[0] >= 0) {
        double xv[K];
#pragma unroll
        for (int k = 0; k < K; ++k) xv[k] = cur.col[0][k] >= 0 ? xs[cur.col[0][k]] : 0.0;
        double rsum = gs_init<BLK>(cur.bi[0]);
#pragma unroll
        for (int k = 0; k < K; ++k)
          if (cur.col[0][k] >= 0) rsum = gs_acc<BLK>(rsum, cur.val[0][k], xv[k]);
        if (gs_upd<BLK>(cur.diag[0])) xs[cur.row[0]] = gs_fin<BLK>(rsum, cur.bi[0], cur.diag[0]);
      }
      __syncthreads();
      if (l + 1 < n_levels) cur = nxt;
    }
  }
  for (int64_t i = threadIdx.x; i < n; i += kGsBlock) x[i] = xs[i];
}

// Windowed one-wave sweep for levels of <= 64 * RW rows: wave 0 walks the levels with x held by
// level-order position in an LDS ring (a level's rows read positions at most W levels away, so
// levels [l - W, l + W] are all a step needs); the 7 other waves meanwhile stage the next chunk
// of levels into the other buffer: the structure (values, columns as ring slots, diagonal, b,
// row id) and the old x of the levels entering the window, read from xl, a level-ordered copy of
// x (one independent load per position instead of rows[p] then x[rows[p]]), every load of a
// thread's positions issued before its first LDS store. Consecutive levels need only a wavefront
// fence; a chunk ends with a workgroup barrier.
// Pads point at the ring's zero slot (+0.0 products: the sum starts at +0.0 and never becomes
// -0.0, so bitwise neutral); a zero-diagonal row is left alone, as the sequential sweep does (its
// quotient goes to the sink slot). Updated values go to the ring and to xl (copied back to x by
// one coalesced pass after the launch: no scattered stores in the sweep). Same products,
// order and division: bitwise gs_row.
constexpr int kGsWinBlock = 512;
#ifndef MLAMG_GSWIN_LAB  // timing variants (tools/gs_win_lab.py): 1 = no sweep, 2 = no staging
#define MLAMG_GSWIN_LAB 0
#endif
constexpr int kGsWinStageU = 4;  // positions per staging thread with all loads in flight

// one staging buffer of cap + 1 positions (the last: the dummy of lanes past a level's end),
// 16-byte aligned sections: vals (cap+1) x KM | diag | b (doubles) | level starts
// (cap + 2 int32) | columns (cap+1) x KM (uint16 ring slots), after a 16-byte header (levels,
// first position, positions)
__host__ __device__ constexpr int64_t win_a16(int64_t b) { return (b + 15) & ~int64_t(15); }
__host__ __device__ constexpr int64_t win_buf_bytes(int64_t cap, int KM) {
  return 16 + win_a16(8 * (cap + 1) * KM) + 2 * win_a16(8 * (cap + 1)) + win_a16(4 * (cap + 2)) +
         win_a16(2 * (cap + 1) * KM);
}

template <int KM>
struct WinBuf {
  double* v;
  double* d;
  double* b;
  int32_t* l;
  uint16_t* c;
  int32_t* h;
  __device__ WinBuf(char* base, int cap) {
    char* p = base + 16;
    h = reinterpret_cast<int32_t*>(base);
    v = reinterpret_cast<double*>(p);
    p += win_a16(8 * (int64_t)(cap + 1) * KM);
    d = reinterpret_cast<double*>(p);
    p += win_a16(8 * (int64_t)(cap + 1));
    b = reinterpret_cast<double*>(p);
    p += win_a16(8 * (int64_t)(cap + 1));
    l = reinterpret_cast<int32_t*>(p);
    p += win_a16(4 * (int64_t)(cap + 2));
    c = reinterpret_cast<uint16_t*>(p);
  }
};

template <int KM>
struct WinCols {  // KM uint16 slots: one 8-byte (KM 4) or 16-byte (KM 8) LDS access
  typedef typename std::conditional<KM == 4, uint2, uint4>::type T;
};

template <int KM, int RW, int CW, bool BLK>
__global__ __launch_bounds__(kGsWinBlock) void k_gs_win(const int4* __restrict__ cdesc,
                                                     const int32_t* __restrict__ wlev,
                                                     int32_t nchunks,
                                                     const int32_t* __restrict__ wcol,
                                                     const double* __restrict__ pval,
                                                     const double* __restrict__ pdiag,
                                                     const double* __restrict__ blvl,
                                                     int ring_log2, int cap,
                                                     int iterations, double* xl,
                                                     const int32_t* done) {
  extern __shared__ double lds[];
  if (done && *done) return;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int RS = 1 << ring_log2, RM = RS - 1;
  double* ring = lds;  // RS slots + the zero slot (RS) + the sink slot (RS + 1)
  // the sweeping waves' level counters (CW > 1), then the staging buffers
  int32_t* flags = reinterpret_cast<int32_t*>(lds + RS + 2);
  char* bufs = reinterpret_cast<char*>(lds + ((RS + 4 + 1) & ~1));
  if (tid < 4) flags[tid] = 0;
  int seq = 0;
  const int64_t bb = win_buf_bytes(cap, KM);
  if (tid == 0) ring[RS] = 0.0;
  typedef typename WinCols<KM>::T CT;
  auto stage = [&](int ch, char* base, int t0, int nt) {
    WinBuf<KM> w(base, cap);
    // the chunk's plan (host-built): levels, first position and count, the old-x range entering
    // the window (levels [l0 + W, l1 + W) clipped; chunk 0: [0, l1 + W)) and its level starts
    const int4 c0 = cdesc[2 * ch], c1 = cdesc[2 * ch + 1];
    const int nl = c0.x, P0 = c0.y, cnt = c0.z, X0 = c0.w, xcnt = c1.x, woff = c1.y;
    if (t0 == 0) {
      w.h[0] = nl;
      w.h[1] = P0;
      w.h[2] = cnt;
    }
    const int tot = max(cnt + 1, xcnt);
    for (int q0 = t0; q0 < tot; q0 += nt * kGsWinStageU) {
      double v[kGsWinStageU][KM], d[kGsWinStageU], bv[kGsWinStageU], xo[kGsWinStageU];
      int32_t c[kGsWinStageU][KM], ls[kGsWinStageU];
#pragma unroll
      for (int u = 0; u < kGsWinStageU; ++u) {
        const int q = q0 + u * nt;
        ls[u] = wlev[woff + min(q, nl)];
        const bool in = q < cnt;
        const int64_t pp = in ? (int64_t)(P0 + q) : 0;
#pragma unroll
        for (int k = 0; k < KM; k += 4) {
          const int4 c4 = *reinterpret_cast<const int4*>(wcol + pp * KM + k);
          c[u][k] = c4.x;
          c[u][k + 1] = c4.y;
          c[u][k + 2] = c4.z;
          c[u][k + 3] = c4.w;
        }
#pragma unroll
        for (int k = 0; k < KM; k += 2) {
          const double2 v2 = *reinterpret_cast<const double2*>(pval + pp * KM + k);
          v[u][k] = v2.x;
          v[u][k + 1] = v2.y;
        }
        d[u] = pdiag[pp];
        bv[u] = blvl[pp];
        // written by wave 0 in the previous sweep of this launch: past L1
        xo[u] = q < xcnt ? __hip_atomic_load(xl + X0 + q, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT)
                         : 0.0;
      }
#pragma unroll
      for (int u = 0; u < kGsWinStageU; ++u) {
        const int q = q0 + u * nt;
        if (q <= cnt) {
          const bool dummy = q == cnt;  // lanes past a level's end: zero slots, sink target
          uint16_t cs[KM];
#pragma unroll
          for (int k = 0; k < KM; ++k)
            cs[k] = (uint16_t)(!dummy && c[u][k] >= 0 ? (c[u][k] & RM) : RS);
          *reinterpret_cast<CT*>(w.c + (int64_t)q * KM) = *reinterpret_cast<const CT*>(cs);
#pragma unroll
          for (int k = 0; k < KM; k += 2) {
            double2 v2;
            v2.x = dummy ? 0.0 : v[u][k];
            v2.y = dummy ? 0.0 : v[u][k + 1];
            *reinterpret_cast<double2*>(w.v + (int64_t)q * KM + k) = v2;
          }
          w.d[q] = dummy ? 0.0 : d[u];
          w.b[q] = dummy ? 0.0 : bv[u];
        }
        if (q < xcnt) ring[(X0 + q) & RM] = xo[u];
        if (q <= nl) w.l[q] = ls[u];
      }
    }
  };
  for (int it = 0; it < iterations; ++it) {
    stage(0, bufs, tid, kGsWinBlock);
    __syncthreads();
    for (int ch = 0; ch < nchunks; ++ch) {
      char* cur = bufs + (MLAMG_GSWIN_LAB == 2 ? 0 : (ch & 1) * bb);
      if (tid < 64 * CW && MLAMG_GSWIN_LAB != 1) {
        const WinBuf<KM> w(cur, cap);
        const int nl = w.h[0], P0 = w.h[1], cnt = w.h[2];
        int c[RW][KM], p[RW];
        double v[RW][KM], d[RW], bv[RW];
        auto load = [&](int l, int (&cc)[RW][KM], double (&vv)[RW][KM], double* dd, double* bq,
                        int* pq) {
          const int a = w.l[l], z = w.l[l + 1];
#pragma unroll
          for (int u = 0; u < RW; ++u) {
            const int q0 = a + lane + 64 * (wv + CW * u);
            const int q = q0 < z ? q0 : cnt;
            const CT c4 = *reinterpret_cast<const CT*>(w.c + (int64_t)q * KM);
            const uint16_t* cs = reinterpret_cast<const uint16_t*>(&c4);
#pragma unroll
            for (int k = 0; k < KM; ++k) cc[u][k] = cs[k];
#pragma unroll
            for (int k = 0; k < KM; k += 2) {
              const double2 v2 = *reinterpret_cast<const double2*>(w.v + (int64_t)q * KM + k);
              vv[u][k] = v2.x;
              vv[u][k + 1] = v2.y;
            }
            dd[u] = w.d[q];
            bq[u] = w.b[q];
            pq[u] = q;
          }
        };
        load(0, c, v, d, bv, p);
        #pragma unroll 1
        for (int l = 0; l < nl; ++l) {
          double g[RW][KM];
#pragma unroll
          for (int u = 0; u < RW; ++u)
#pragma unroll
            for (int k = 0; k < KM; ++k) g[u][k] = ring[c[u][k]];
          int c2[RW][KM], p2[RW];
          double v2[RW][KM], d2[RW], bv2[RW];
          load(l + 1 < nl ? l + 1 : l, c2, v2, d2, bv2, p2);
          // the RW rows' sums and divisions first, as one block (their dependency chains
          // interleave), then the stores
          double xi[RW];
#pragma unroll
          for (int u = 0; u < RW; ++u) {
            double y = gs_init<BLK>(bv[u]);
#pragma unroll
            for (int k = 0; k < KM; ++k) y = gs_acc<BLK>(y, v[u][k], g[u][k]);
            xi[u] = gs_fin<BLK>(y, bv[u], d[u]);
          }
          // the dummy, and a zero-diagonal row of gauss_seidel: left alone (the sink slot)
          bool up[RW];
#pragma unroll
          for (int u = 0; u < RW; ++u) up[u] = p[u] != cnt && gs_upd<BLK>(d[u]);
#pragma unroll
          for (int u = 0; u < RW; ++u) ring[up[u] ? ((P0 + p[u]) & RM) : RS + 1] = xi[u];
#pragma unroll
          for (int u = 0; u < RW; ++u)
            if (up[u]) xl[P0 + p[u]] = xi[u];
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          if (CW > 1) {
            // the level's other sweeping waves: a wave's LDS operations complete in issue
            // order, so a counter stored after the ring stores is seen after them; the spin
            // reads all counters until each has reached this level
            ++seq;
            asm volatile("" ::: "memory");
            if (lane == 0) *reinterpret_cast<volatile int32_t*>(flags + wv) = seq;
            for (;;) {
              bool ok = true;
#pragma unroll
              for (int w2 = 0; w2 < CW; ++w2)
                ok = ok && *reinterpret_cast<volatile int32_t*>(flags + w2) >= seq;
              if (ok) break;
            }
            asm volatile("" ::: "memory");
          }
#pragma unroll
          for (int u = 0; u < RW; ++u) {
#pragma unroll
            for (int k = 0; k < KM; ++k) {
              c[u][k] = c2[u][k];
              v[u][k] = v2[u][k];
            }
            d[u] = d2[u];
            bv[u] = bv2[u];
            p[u] = p2[u];
          }
        }
      } else if (tid >= 64 * CW && MLAMG_GSWIN_LAB != 2 && ch + 1 < nchunks) {
        stage(ch + 1, bufs + ((ch + 1) & 1) * bb, tid - 64 * CW, kGsWinBlock - 64 * CW);
      }
      __syncthreads();
    }
    __threadfence();  // this sweep's xl stores before the next sweep's window loads
    __syncthreads();
  }
}

__global__ void k_gs_b_level(const int32_t* __restrict__ rows, int64_t n,
                             const double* __restrict__ b, double* __restrict__ blvl,
                             const int32_t* done) {
  if (done && *done) return;
  const int64_t p = blockIdx.x * 256ll + threadIdx.x;
  if (p < n) blvl[p] = b[rows[p]];
}

// MLAMG_GS_NO_LDS=1 keeps small systems on the global-memory kernel (A/B runs, tests)
static bool gs_lds_disabled() {
  const char* e = std::getenv("MLAMG_GS_NO_LDS");
  return e && e[0] == '1';
}

template <int R, int K, bool BLK>
static void launch_gs_pipe(const mlamg_gs* G, double* x, const double* b, int iterations,
                           const int32_t* done, hipStream_t s) {
  const int64_t n = G->A->n_rows;
  hipLaunchKernelGGL(k_gs_b_level, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, G->rows,
                     n, b, G->b_lvl, done);
  if (R == 1 && n <= kGsLdsMax && !gs_lds_disabled()) {
    hipLaunchKernelGGL((k_gs_lds<K, BLK>), dim3(1), dim3(kGsBlock), sizeof(double) * n, s, G->rows,
                       G->d_level_ptr, G->n_levels, n, G->pk_col, G->pk_val, G->pk_diag,
                       G->b_lvl, iterations, x, done);
    return;
  }
  hipLaunchKernelGGL((k_gs_pipe<R, K, BLK>), dim3(1), dim3(kGsBlock), 0, s, G->rows, G->d_level_ptr,
                     G->n_levels, G->pk_col, G->pk_val, G->pk_diag, G->b_lvl, iterations, x,
                     done);
}

// x <- xl after the window sweeps (rows in level order: coalesced reads of xl; a zero-diagonal
// row's xl still holds its old x)
__global__ void k_gs_win_post(const int32_t* __restrict__ rows, int64_t n,
                              const double* __restrict__ xl, double* __restrict__ x,
                              const int32_t* done) {
  if (done && *done) return;
  const int64_t p = blockIdx.x * 256ll + threadIdx.x;
  if (p < n) x[rows[p]] = xl[p];
}

__global__ void k_gs_win_prep(const int32_t* __restrict__ rows, int64_t n,
                              const double* __restrict__ b, double* __restrict__ blvl,
                              const double* __restrict__ x, double* __restrict__ xl,
                              const int32_t* done) {
  if (done && *done) return;
  const int64_t p = blockIdx.x * 256ll + threadIdx.x;
  if (p < n) {
    const int32_t i = rows[p];
    blvl[p] = b[i];
    xl[p] = x[i];
  }
}

static bool gs_ring_disabled() {  // MLAMG_GS_NO_RING=1: A/B runs, tests
  const char* e = std::getenv("MLAMG_GS_NO_RING");
  return e && e[0] == '1';
}

static bool gs_wave_disabled() {  // MLAMG_GS_NO_WAVE=1: A/B runs, tests
  const char* e = std::getenv("MLAMG_GS_NO_WAVE");
  return e && e[0] == '1';
}

static bool gs_wring_disabled() {  // MLAMG_GS_NO_WRING=1: A/B runs, tests
  const char* e = std::getenv("MLAMG_GS_NO_WRING");
  return e && e[0] == '1';
}

static bool gs_win_disabled() {  // MLAMG_GS_NO_WIN=1: A/B runs, tests
  const char* e = std::getenv("MLAMG_GS_NO_WIN");
  return e && e[0] == '1';
}

template <int KM, int RW, int CW, bool BLK>
static void launch_gs_win(const mlamg_gs* G, double* x, const double* b, int iterations,
                          const int32_t* done, hipStream_t s) {
  const int64_t n = G->A->n_rows;
  hipLaunchKernelGGL(k_gs_win_prep, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, G->rows,
                     n, b, G->b_lvl, x, G->win_xl, done);
  hipLaunchKernelGGL((k_gs_win<KM, RW, CW, BLK>), dim3(1), dim3(kGsWinBlock), G->win_lds, s,
                     reinterpret_cast<const int4*>(G->d_clev), G->d_clev + 8 * G->n_chunks,
                     G->n_chunks, G->wcol, G->pk_val, G->pk_diag, G->b_lvl, G->ring_log2,
                     G->win_cap, iterations, G->win_xl, done);
  hipLaunchKernelGGL(k_gs_win_post, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, G->rows,
                     n, G->win_xl, x, done);
}

int64_t gs_rows(const mlamg_gs* G) { return G->A->n_rows; }

static size_t gs_ring_lds(const mlamg_gs* G) {
  return (sizeof(double) << G->ring_log2_r) + sizeof(double) +
         sizeof(int32_t) * (G->n_levels + 1);
}

template <bool BLK>
static int gs_sweep_one(const mlamg_gs* G, double* x, const double* b, int iterations,
                        const int32_t* done, hipStream_t s) {
  const mlamg_csr* A = G->A;
  if (A->n_rows == 0 || iterations <= 0) return MLAMG_OK;
  const bool pipe = G->pk_k > 0 && G->n_levels > 4;
  if (pipe && G->win_rw > 0 && !gs_win_disabled()) {
    // win_rw = 64-row slots per level: up to 4 sweeping waves, then 2 rows per lane
    if (G->pk_k == 4) {
      switch (G->win_rw) {
        case 1: launch_gs_win<4, 1, 1, BLK>(G, x, b, iterations, done, s); break;
        case 2: launch_gs_win<4, 1, 2, BLK>(G, x, b, iterations, done, s); break;
        case 3: launch_gs_win<4, 1, 3, BLK>(G, x, b, iterations, done, s); break;
        case 4: launch_gs_win<4, 1, 4, BLK>(G, x, b, iterations, done, s); break;
        default: launch_gs_win<4, 2, 4, BLK>(G, x, b, iterations, done, s); break;
      }
    } else {
      switch (G->win_rw) {
        case 1: launch_gs_win<8, 1, 1, BLK>(G, x, b, iterations, done, s); break;
        case 2: launch_gs_win<8, 1, 2, BLK>(G, x, b, iterations, done, s); break;
        case 3: launch_gs_win<8, 1, 3, BLK>(G, x, b, iterations, done, s); break;
        case 4: launch_gs_win<8, 1, 4, BLK>(G, x, b, iterations, done, s); break;
        default: launch_gs_win<8, 2, 4, BLK>(G, x, b, iterations, done, s); break;
      }
    }
  } else if (pipe && G->rcol && G->rpv && G->rcode && G->rxl && !gs_ring_disabled() &&
             gs_ring_lds(G) <= kGsRingLdsMax) {
    const int64_t n = A->n_rows;
    // one sweep per launch pair: the products of the old values are formed before each
    for (int it = 0; it < iterations; ++it) {
      hipLaunchKernelGGL((k_gs_ring_prep<BLK>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                         G->rows, n, G->rcol, G->pk_val, G->pk_diag, b, x, G->rpv, G->b_lvl,
                         done);
      hipLaunchKernelGGL((k_gs_ring<BLK>), dim3(1), dim3(kGsBlock), gs_ring_lds(G), s,
                         G->d_level_ptr, G->n_levels, reinterpret_cast<const uint2*>(G->rcode),
                         G->rpv, G->pk_diag, G->b_lvl, G->ring_log2_r, G->rxl, done);
      // the level-ordered values back to x (coalesced stores in the sweep, one scatter here)
      hipLaunchKernelGGL(k_gs_win_post, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                         G->rows, n, G->rxl, x, done);
    }
  } else if (pipe && G->max_level_rows <= 2 * kGsBlock) {
    const bool one = G->max_level_rows <= kGsBlock;
    if (G->pk_k == 4) {
      if (one) launch_gs_pipe<1, 4, BLK>(G, x, b, iterations, done, s);
      else launch_gs_pipe<2, 4, BLK>(G, x, b, iterations, done, s);
    } else {
      if (one) launch_gs_pipe<1, 8, BLK>(G, x, b, iterations, done, s);
      else launch_gs_pipe<2, 8, BLK>(G, x, b, iterations, done, s);
    }
  } else if (G->wr_code && G->rxl && G->b_lvl && !gs_wring_disabled()) {
    const int64_t n = A->n_rows;
    const int span = G->wr_lpr * G->wr_epl;
    auto go = [&](auto l, auto e) {
      hipLaunchKernelGGL((k_gs_wring<decltype(l)::value, decltype(e)::value, BLK>), dim3(1),
                         dim3(gs_wring_threads<decltype(e)::value>()), G->wr_lds, s, G->wr_st, G->wr_steps, (int32_t)(n - 1),
                         G->wr_code, G->wr_pv, G->wr_len, G->b_lvl, G->wr_d, G->wr_log2, G->rxl,
                         done);
    };
    using I2 = std::integral_constant<int, 2>;
    using I4 = std::integral_constant<int, 4>;
    using I8 = std::integral_constant<int, 8>;
    using I16 = std::integral_constant<int, 16>;
    for (int it = 0; it < iterations; ++it) {
      hipLaunchKernelGGL((k_gs_wring_prep<BLK>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                         s, G->rows, n, A->indptr, A->indices, A->data, G->wr_code, span, b, x,
                         G->wr_pv, G->b_lvl, G->wr_d, done);
      if (G->wr_epl == 2) {
        if (G->wr_lpr == 8) go(I8(), I2());
        else go(I16(), I2());
      } else {
        if (G->wr_lpr == 8) go(I8(), I4());
        else go(I16(), I4());
      }
      hipLaunchKernelGGL(k_gs_win_post, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                         G->rows, n, G->rxl, x, done);
    }
  } else if (G->wpos && G->max_level_rows <= kGsBlockMaxLevelRows && G->n_levels > 4 &&
             !gs_wave_disabled()) {
    auto go = [&](auto l, auto e) {
      hipLaunchKernelGGL((k_gs_wave<decltype(l)::value, decltype(e)::value, BLK>), dim3(1),
                         dim3(kGsWaveBlock), 0, s, reinterpret_cast<const int4*>(G->wpos),
                         A->indices, A->data, G->d_level_ptr, G->n_levels, iterations, x, b,
                         done);
    };
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I4 = std::integral_constant<int, 4>;
    using I8 = std::integral_constant<int, 8>;
    using I16 = std::integral_constant<int, 16>;
    const int ml = G->max_len;
    // 8 lanes per row when the levels average more than 64 rows (128 rows per pass: fewer
    // passes, each with its loads on the critical path), else 16 (fewer entries per lane)
    static const char* lpr_env = std::getenv("MLAMG_GS_WAVE_LPR");  // A/B knob: 8 or 16
    const bool wide = lpr_env ? lpr_env[0] == '8' : A->n_rows > 64 * (int64_t)G->n_levels;
    if (wide && ml <= 64) {
      if (ml <= 8) go(I8(), I1());
      else if (ml <= 16) go(I8(), I2());
      else if (ml <= 32) go(I8(), I4());
      else go(I8(), I8());
    } else {
      if (ml <= 16) go(I16(), I1());
      else if (ml <= 32) go(I16(), I2());
      else if (ml <= 64) go(I16(), I4());
      else go(I16(), I8());
    }
  } else if (G->max_level_rows <= kGsBlock && G->n_levels > 4) {
    // one row per thread per level; wider levels go one launch per level over the whole chip
    hipLaunchKernelGGL(k_gs_block<BLK>, dim3(1), dim3(kGsBlock), 0, s, A->indptr, A->indices, A->data,
                       G->rows, G->d_level_ptr, G->n_levels, iterations, x, b, done);
  } else {
    for (int it = 0; it < iterations; ++it) {
      for (int32_t l = 0; l < G->n_levels; ++l) {
        const int32_t a = G->level_ptr[l], cnt = G->level_ptr[l + 1] - a;
        hipLaunchKernelGGL(k_gs_level<BLK>, dim3((cnt + 255) / 256), dim3(256), 0, s, A->indptr,
                           A->indices, A->data, G->rows + a, cnt, x, b, done);
      }
    }
  }
  MLAMG_HIP(hipGetLastError());
  return MLAMG_OK;
}

// one iteration of a symmetric sweep = the forward schedule, then the backward one
int gs_sweep_impl(const mlamg_gs* G, double* x, const double* b, int iterations,
                  const int32_t* done, hipStream_t s) {
  auto one = [&](const mlamg_gs* H, int it) {
    return H->block ? gs_sweep_one<true>(H, x, b, it, done, s)
                    : gs_sweep_one<false>(H, x, b, it, done, s);
  };
  if (!G->bwd) return one(G, iterations);
  for (int it = 0; it < iterations; ++it) {
    MLAMG_TRY(one(G, 1));
    MLAMG_TRY(one(G->bwd, 1));
  }
  return MLAMG_OK;
}

}  // namespace mlamg

using namespace mlamg;

// The ring sweep's plan (levels of <= 1024 rows, K = 4 slots): W = the widest level distance from
// a row to an earlier-swept column; positions of levels [l - W, l] must fit the ring
// (<= 8,192 doubles). Optional: rcol stays nullptr otherwise.
static void setup_ring(mlamg_gs* G, const std::vector<int32_t>& level,
                       const std::vector<int32_t>& rows, const std::vector<int32_t>& pcol) {
  const int64_t n = G->A->n_rows;
  const int K = kGsRingK;
  if (G->max_level_rows > kGsBlock || G->n_levels <= 4 || n == 0) return;
  std::vector<int32_t> pos(n);
  for (int64_t p = 0; p < n; ++p) pos[rows[p]] = (int32_t)p;
  int W = 0;
  for (int64_t p = 0; p < n; ++p)
    for (int k = 0; k < K; ++k) {
      const int32_t c = pcol[(size_t)p * K + k];
      if (c >= 0 && level[c] < level[rows[p]]) W = std::max(W, level[rows[p]] - level[c]);
    }
  const std::vector<int32_t>& lp = G->level_ptr;
  int64_t span = 0;
  for (int l = 0; l < G->n_levels; ++l)
    span = std::max<int64_t>(span, lp[l + 1] - lp[std::max(0, l - W)]);
  int lg = 0;
  while ((int64_t(1) << lg) < span) ++lg;
  if (lg > 13) return;
  std::vector<int32_t> rc((size_t)n * K);
  for (int64_t p = 0; p < n; ++p)
    for (int k = 0; k < K; ++k) {
      const int32_t c = pcol[(size_t)p * K + k];
      rc[(size_t)p * K + k] = c < 0 ? -1 : (level[c] < level[rows[p]] ? pos[c] : -(c + 2));
    }
  if (hipMalloc(&G->rcol, sizeof(int32_t) * rc.size()) != hipSuccess) {
    G->rcol = nullptr;
    return;
  }
  (void)hipMemcpy(G->rcol, rc.data(), sizeof(int32_t) * rc.size(), hipMemcpyHostToDevice);
  std::vector<uint16_t> code(rc.size());
  const int32_t RM = (1 << lg) - 1;
  for (size_t e = 0; e < rc.size(); ++e)
    code[e] = (uint16_t)(rc[e] >= 0 ? (rc[e] & RM) : (rc[e] == -1 ? kGsRingPad : kGsRingLater));
  if (hipMalloc(&G->rpv, sizeof(double) * rc.size()) != hipSuccess) G->rpv = nullptr;
  if (hipMalloc(&G->rxl, sizeof(double) * n) != hipSuccess) G->rxl = nullptr;
  if (hipMalloc(&G->rcode, sizeof(uint16_t) * code.size()) != hipSuccess) G->rcode = nullptr;
  else
    (void)hipMemcpy(G->rcode, code.data(), sizeof(uint16_t) * code.size(), hipMemcpyHostToDevice);
  G->ring_log2_r = lg;
}

// The long-row ring sweep's plan (rows of 9..64 entries, levels swept in steps of 1024 / LPR
// rows): the slot codes in the padded level order, the row lengths, the step table and the ring
// (W levels of positions, <= 8,192 slots). Optional: wr_code stays nullptr otherwise.
static void setup_wring(mlamg_gs* G, const std::vector<int32_t>& ip,
                        const std::vector<int32_t>& ij, const std::vector<int32_t>& level,
                        const std::vector<int32_t>& rows) {
  const int64_t n = G->A->n_rows;
  const int nlev = G->n_levels;
  const int ml = G->max_len;
  if (n == 0 || nlev <= 4 || ml > 64) return;
  // 8 lanes per row when levels average more than 64 rows, else 16; two slots per lane in
  // 1024-thread workgroups, four (rows of 33..64 entries, or 17..32 on wide levels) in 512-thread
  // ones: five register sets of four slots exceed the 128 VGPRs a 1024-thread workgroup has
  // (spilled, the 3-D 128^3 level-1 sweep ran 2x slower than k_gs_wave)
  const bool wide = n > 64 * (int64_t)nlev;
  const int lpr = (wide && ml <= 32) ? 8 : 16;
  const int epl = ml <= 2 * lpr ? 2 : 4;
  if (ml > lpr * epl) return;
  const int span = lpr * epl, rows_per_step = (epl == 2 ? 1024 : 512) / lpr;
  std::vector<int32_t> pos(n);
  for (int64_t p = 0; p < n; ++p) pos[rows[p]] = (int32_t)p;
  int W = 0;
  for (int64_t i = 0; i < n; ++i)
    for (int k = ip[i]; k < ip[i + 1]; ++k)
      if (ij[k] != i && level[ij[k]] < level[i]) W = std::max(W, level[i] - level[ij[k]]);
  const std::vector<int32_t>& lp = G->level_ptr;
  std::vector<int2> st;
  for (int l = 0; l < nlev; ++l)
    for (int32_t a = lp[l]; a < lp[l + 1]; a += rows_per_step)
      st.push_back(make_int2(a, std::min<int32_t>(rows_per_step, lp[l + 1] - a)));
  // a step costs about what one of k_gs_wave's level passes does: levels much wider than a step
  // stay there (3-D 128^3 level 1, 14 steps a level: V-cycle 63 -> 137 ms through this kernel)
  if (st.size() > 2 * (size_t)nlev) return;
  const size_t rest = sizeof(double) * 3 +
                      (sizeof(double) + sizeof(uint16_t)) * rows_per_step * span + 8 +
                      sizeof(int2) * st.size() + 16;
  if (rest >= kGsWringLdsMax) return;
  int64_t cap = 8192;  // ring slots: at most 8,192 and what the LDS budget leaves
  while (cap > 1 && rest + sizeof(double) * cap > kGsWringLdsMax) cap >>= 1;
  // the ring horizon Wr: the most levels back whose positions fit the ring; couplings further
  // back are read from xl two steps ahead, which needs Wr >= 2 (a step advances <= 1 level)
  auto span_of = [&](int w) {
    int64_t sp = 0;
    for (int l = 0; l < nlev; ++l) sp = std::max<int64_t>(sp, lp[l + 1] - lp[std::max(0, l - w)]);
    return sp;
  };
  int Wr = W;
  while (Wr > 2 && span_of(Wr) > cap) Wr = std::max(2, Wr * 7 / 8);
  if (span_of(Wr) > cap || (Wr < W && Wr < 2)) return;
  const int64_t spanp = span_of(Wr);
  int lg = 0;
  while ((int64_t(1) << lg) < spanp) ++lg;
  if (lg > 13 || (int64_t(1) << lg) > cap) return;
  const size_t lds = rest + (sizeof(double) << lg);
  const int32_t RM = (1 << lg) - 1;
  std::vector<int32_t> code((size_t)n * span, kGsWringPad);
  std::vector<int32_t> len(n);
  for (int64_t p = 0; p < n; ++p) {
    const int32_t i = rows[p];
    len[p] = ip[i + 1] - ip[i];
    for (int k = ip[i]; k < ip[i + 1]; ++k) {
      const int32_t j = ij[k];
      int32_t c = kGsWringLater;
      if (j == i) c = kGsWringDiag;
      else if (level[j] < level[i]) c = level[i] - level[j] <= Wr ? (pos[j] & RM) : kGsWringFar - pos[j];
      code[(size_t)p * span + (k - ip[i])] = c;
    }
  }
  const size_t m = (size_t)n * span;
  bool ok = hipMalloc(&G->wr_code, sizeof(int32_t) * m) == hipSuccess;
  ok = ok && hipMalloc(&G->wr_pv, sizeof(double) * m) == hipSuccess;
  ok = ok && hipMalloc(&G->wr_len, sizeof(int32_t) * n) == hipSuccess;
  ok = ok && hipMalloc(&G->wr_d, sizeof(double) * n) == hipSuccess;
  ok = ok && hipMalloc(&G->wr_st, sizeof(int2) * st.size()) == hipSuccess;
  if (!G->rxl) ok = ok && hipMalloc(&G->rxl, sizeof(double) * n) == hipSuccess;
  if (!G->b_lvl) ok = ok && hipMalloc(&G->b_lvl, sizeof(double) * n) == hipSuccess;
  if (!ok) {
    for (void* q : {(void*)G->wr_code, (void*)G->wr_pv, (void*)G->wr_len, (void*)G->wr_d,
                    (void*)G->wr_st})
      if (q) (void)hipFree(q);
    G->wr_code = nullptr;
    G->wr_pv = G->wr_d = nullptr;
    G->wr_len = nullptr;
    G->wr_st = nullptr;
    return;
  }
  (void)hipMemcpy(G->wr_code, code.data(), sizeof(int32_t) * m, hipMemcpyHostToDevice);
  (void)hipMemset(G->wr_pv, 0, sizeof(double) * m);
  (void)hipMemcpy(G->wr_len, len.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice);
  (void)hipMemcpy(G->wr_st, st.data(), sizeof(int2) * st.size(), hipMemcpyHostToDevice);
  G->wr_lpr = lpr;
  G->wr_epl = epl;
  G->wr_steps = (int32_t)st.size();
  G->wr_log2 = lg;
  G->wr_lds = lds;
}

// The windowed one-wave sweep's plan: W = the widest level distance of a coupling, chunks of
// levels that fit a staging buffer, and the ring that holds every position a step and the
// concurrent staging of the next chunk touch. Optional: win_rw stays 0 when levels are wider
// than 64 * RW rows or the ring and buffers do not fit the LDS budget.
static void setup_window(mlamg_gs* G, const std::vector<int32_t>& ip,
                         const std::vector<int32_t>& ij, const std::vector<int32_t>& level,
                         const std::vector<int32_t>& rows, const std::vector<int32_t>& pcol,
                         int K) {
  const int64_t n = G->A->n_rows;
  const int nlev = G->n_levels;
  const int rw = (G->max_level_rows + 63) / 64;  // 64-row slots: <= 4 waves x 2 rows per lane
  if (rw < 1 || rw > 8 || nlev <= 4) return;
  int W = 0;
  for (int64_t i = 0; i < n; ++i)
    for (int k = ip[i]; k < ip[i + 1]; ++k)
      if (ij[k] != i) W = std::max(W, std::abs(level[ij[k]] - level[i]));
  const std::vector<int32_t>& lp = G->level_ptr;
  const size_t budget = 150 * 1024;
  for (int cap = 4096; cap >= G->max_level_rows; cap = cap * 7 / 8) {
    std::vector<int32_t> clev{0};
    for (int l = 0; l < nlev;) {
      const int start = l;
      while (l < nlev && (l == start || lp[l + 1] - lp[start] <= cap)) ++l;
      clev.push_back(l);
    }
    const int nch = (int)clev.size() - 1;
    int64_t span = 0;
    for (int ch = 0; ch < nch; ++ch) {
      const int lo = std::max(0, clev[ch] - W);
      const int hi = std::min(nlev, clev[std::min(ch + 2, nch)] + W);
      span = std::max<int64_t>(span, lp[hi] - lp[lo]);
    }
    int lg = 0;
    while ((int64_t(1) << lg) < span) ++lg;
    const size_t ring = ((size_t(1) << lg) + 4) * 8;
    const size_t bufs = 2 * (size_t)win_buf_bytes(cap, K);
    if (ring + bufs > budget) continue;
    // per chunk: {levels, first position, positions, old-x start} {old-x count, level-start
    // offset, -, -}, then every chunk's level starts relative to its first position
    std::vector<int32_t> plan(8 * (size_t)nch);
    for (int ch = 0; ch < nch; ++ch) {
      const int l0 = clev[ch], l1 = clev[ch + 1];
      const int la = ch == 0 ? 0 : std::min(nlev, l0 + W), lb = std::min(nlev, l1 + W);
      int32_t* d = plan.data() + 8 * (size_t)ch;
      d[0] = l1 - l0;
      d[1] = lp[l0];
      d[2] = lp[l1] - lp[l0];
      d[3] = lp[la];
      d[4] = lp[lb] - lp[la];
      d[5] = (int32_t)plan.size() - 8 * nch;
      for (int l = l0; l <= l1; ++l) plan.push_back(lp[l] - lp[l0]);
    }
    std::vector<int32_t> pos(n), wcol((size_t)n * K, -1);
    for (int64_t p = 0; p < n; ++p) pos[rows[p]] = (int32_t)p;
    for (size_t q = 0; q < (size_t)n * K; ++q)
      if (pcol[q] >= 0) wcol[q] = pos[pcol[q]];
    if (hipMalloc(&G->wcol, sizeof(int32_t) * std::max<size_t>((size_t)n * K, 1)) != hipSuccess ||
        hipMalloc(&G->d_clev, sizeof(int32_t) * plan.size()) != hipSuccess ||
        hipMalloc(&G->win_xl, sizeof(double) * std::max<int64_t>(n, 1)) != hipSuccess) {
      for (void* q : {(void*)G->wcol, (void*)G->d_clev, (void*)G->win_xl})
        if (q) (void)hipFree(q);
      G->wcol = nullptr;
      G->d_clev = nullptr;
      G->win_xl = nullptr;
      return;
    }
    (void)hipMemcpy(G->wcol, wcol.data(), sizeof(int32_t) * (size_t)n * K, hipMemcpyHostToDevice);
    (void)hipMemcpy(G->d_clev, plan.data(), sizeof(int32_t) * plan.size(), hipMemcpyHostToDevice);
    G->win_w = W;
    G->win_cap = cap;
    G->ring_log2 = lg;
    G->n_chunks = nch;
    G->win_lds = ring + bufs + 64;
    G->win_rw = rw;
    return;
  }
}

// one sweep direction's schedule and packed copies
static int gs_build(const mlamg_csr* A, bool backward, bool block, mlamg_gs** out,
                    hipStream_t s) {
  const int64_t n = A->n_rows;
  // MLAMG_TIMING=1: host phase times of the schedule analysis on stderr
  static const bool timing = std::getenv("MLAMG_TIMING") != nullptr;
  auto t_prev = std::chrono::steady_clock::now();
  auto phase = [&](const char* name) {
    if (!timing) return;
    const auto t = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[gs_create] %s %.3f ms\n", name,
                 std::chrono::duration<double, std::milli>(t - t_prev).count());
    t_prev = t;
  };
  std::vector<int32_t> ip(n + 1), ij(A->nnz);
  MLAMG_HIP(hipMemcpyAsync(ip.data(), A->indptr, sizeof(int32_t) * (n + 1), hipMemcpyDeviceToHost, s));
  if (A->nnz)
    MLAMG_HIP(hipMemcpyAsync(ij.data(), A->indices, sizeof(int32_t) * A->nnz, hipMemcpyDeviceToHost, s));
  MLAMG_HIP(hipStreamSynchronize(s));
  phase("copy_in");
  std::vector<int32_t> level(n, 0), req(n, 0);
  int32_t nlev = 0;
  // rows in sweep order; `before(j, i)`: row j is swept before row i
  auto before = [backward](int64_t j, int64_t i) { return backward ? j > i : j < i; };
  for (int64_t t = 0; t < n; ++t) {
    const int64_t i = backward ? n - 1 - t : t;
    int32_t L = req[i];
    for (int k = ip[i]; k < ip[i + 1]; ++k) {
      const int32_t j = ij[k];
      if (j != i && before(j, i)) L = std::max(L, level[j] + 1);
    }
    level[i] = L;
    for (int k = ip[i]; k < ip[i + 1]; ++k) {
      const int32_t j = ij[k];
      if (j != i && before(i, j)) req[j] = std::max(req[j], L + 1);
    }
    nlev = std::max(nlev, L + 1);
  }
  auto* G = new mlamg_gs();
  G->A = A;
  G->block = block;
  G->backward = backward;
  G->n_levels = nlev;
  G->level_ptr.assign(nlev + 1, 0);
  for (int64_t i = 0; i < n; ++i) G->level_ptr[level[i] + 1]++;
  for (int32_t l = 0; l < nlev; ++l) G->level_ptr[l + 1] += G->level_ptr[l];
  std::vector<int32_t> rows(n), fill(G->level_ptr.begin(), G->level_ptr.end() - 1);
  for (int64_t i = 0; i < n; ++i) rows[fill[level[i]]++] = (int32_t)i;
  if (hipMalloc(&G->rows, sizeof(int32_t) * std::max<int64_t>(n, 1)) != hipSuccess) {
    delete G;
    set_error("gs_create: hipMalloc failed");
    return MLAMG_ENOMEM;
  }
  if (n) (void)hipMemcpy(G->rows, rows.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice);
  for (int32_t l = 0; l < nlev; ++l)
    G->max_level_rows = std::max(G->max_level_rows, G->level_ptr[l + 1] - G->level_ptr[l]);
  phase("levels");
  if (hipMalloc(&G->d_level_ptr, sizeof(int32_t) * (nlev + 1)) != hipSuccess) {
    (void)hipFree(G->rows);
    delete G;
    set_error("gs_create: hipMalloc failed");
    return MLAMG_ENOMEM;
  }
  (void)hipMemcpy(G->d_level_ptr, G->level_ptr.data(), sizeof(int32_t) * (nlev + 1),
                  hipMemcpyHostToDevice);
  // level-ordered packed copy for k_gs_pipe (rows with <= 8 off-diagonals)
  {
    int32_t mo = 0;
    for (int64_t i = 0; i < n; ++i) {
      int32_t c = 0;
      for (int k = ip[i]; k < ip[i + 1]; ++k) c += ij[k] != i;
      mo = std::max(mo, c);
    }
    G->max_off = mo;
    const int K = mo <= 4 ? 4 : (mo <= 8 ? 8 : 0);
    int32_t ml = 0;
    for (int64_t i = 0; i < n; ++i) ml = std::max(ml, ip[i + 1] - ip[i]);
    G->max_len = ml;
    // the copies below serve one-workgroup sweeps only: levels wider than they take are swept
    // one launch per level straight from the CSR arrays, so such schedules skip them (C4-size
    // operators: ~1 GB of host packing and upload per sweep direction)
    if (!K && ml <= 8 * kGsWaveMaxLPR && G->max_level_rows <= kGsBlockMaxLevelRows) {
      std::vector<int32_t> wp((size_t)n * 4);
      for (int64_t p = 0; p < n; ++p) {
        const int32_t i = rows[p];
        wp[4 * p] = i;
        wp[4 * p + 1] = ip[i];
        wp[4 * p + 2] = ip[i + 1] - ip[i];
        wp[4 * p + 3] = 0;
      }
      if (hipMalloc(&G->wpos, sizeof(int32_t) * std::max<size_t>(wp.size(), 4)) == hipSuccess) {
        if (n) (void)hipMemcpy(G->wpos, wp.data(), sizeof(int32_t) * wp.size(), hipMemcpyHostToDevice);
      } else {
        G->wpos = nullptr;  // optional: the plain one-workgroup kernel takes these rows
      }
      setup_wring(G, ip, ij, level, rows);
    }
    if (K && G->max_level_rows <= 2 * kGsBlock) {
      std::vector<double> ax(A->nnz);
      if (A->nnz)
        MLAMG_HIP(hipMemcpy(ax.data(), A->data, sizeof(double) * A->nnz, hipMemcpyDeviceToHost));
      std::vector<int32_t> pcol((size_t)n * K, -1);
      std::vector<double> pval((size_t)n * K, 0.0), pdiag(n, 0.0);
      for (int64_t p = 0; p < n; ++p) {
        const int32_t i = rows[p];
        int c = 0;
        for (int k = ip[i]; k < ip[i + 1]; ++k) {
          if (ij[k] == i) {
            pdiag[p] = ax[k];  // the last stored diagonal entry counts, as in the sweep
          } else {
            pcol[(size_t)p * K + c] = ij[k];
            pval[(size_t)p * K + c] = ax[k];
            ++c;
          }
        }
        if (block) pdiag[p] = pdiag[p] != 0.0 ? 1.0 / pdiag[p] : 0.0;  // Dinv = pinv(A_ii)
      }
      phase("pack");
      const size_t m = std::max<size_t>((size_t)n * K, 1), nn = std::max<int64_t>(n, 1);
      if (hipMalloc(&G->pk_col, sizeof(int32_t) * m) == hipSuccess &&
          hipMalloc(&G->pk_val, sizeof(double) * m) == hipSuccess &&
          hipMalloc(&G->pk_diag, sizeof(double) * nn) == hipSuccess &&
          hipMalloc(&G->b_lvl, sizeof(double) * nn) == hipSuccess) {
        if (n) {
          (void)hipMemcpy(G->pk_col, pcol.data(), sizeof(int32_t) * n * K, hipMemcpyHostToDevice);
          (void)hipMemcpy(G->pk_val, pval.data(), sizeof(double) * n * K, hipMemcpyHostToDevice);
          (void)hipMemcpy(G->pk_diag, pdiag.data(), sizeof(double) * n, hipMemcpyHostToDevice);
        }
        G->pk_k = K;
        phase("pack_upload");
        static const char* prefer_ring = std::getenv("MLAMG_GS_PREFER_RING");  // A/B knob
        if (!(prefer_ring && prefer_ring[0] == '1')) setup_window(G, ip, ij, level, rows, pcol, K);
        phase("window");
        if (K == kGsRingK && G->win_rw == 0) setup_ring(G, level, rows, pcol);
      } else {  // optional: the sweep falls back to the plain kernels
        for (void* q : {(void*)G->pk_col, (void*)G->pk_val, (void*)G->pk_diag, (void*)G->b_lvl})
          if (q) (void)hipFree(q);
        G->pk_col = nullptr;
        G->pk_val = G->pk_diag = G->b_lvl = nullptr;
      }
    }
  }
  *out = G;
  return MLAMG_OK;
}

extern "C" {

int mlamg_gs_create_ex(const mlamg_csr* A, int sweep, int block, mlamg_gs** out, void* stream) {
  MLAMG_REQUIRE(A && out, "NULL argument");
  MLAMG_REQUIRE(A->n_rows == A->n_cols, "square matrix required");
  MLAMG_REQUIRE(sweep >= 0 && sweep <= 2, "sweep must be 0 forward, 1 backward, 2 symmetric");
  MLAMG_REQUIRE(block == 0 || block == 1, "block must be 0 or 1");
  hipStream_t s = S(stream);
  mlamg_gs* G = nullptr;
  MLAMG_TRY(gs_build(A, sweep == 1, block == 1, &G, s));
  if (sweep == 2) {
    int rc = gs_build(A, true, block == 1, &G->bwd, s);
    if (rc != MLAMG_OK) {
      mlamg_gs_destroy(G);
      return rc;
    }
  }
  *out = G;
  return MLAMG_OK;
}

int mlamg_gs_create(const mlamg_csr* A, mlamg_gs** out, void* stream) {
  return mlamg_gs_create_ex(A, 0, 0, out, stream);
}

int mlamg_gs_destroy(mlamg_gs* G) {
  if (G) {
    if (G->bwd) mlamg_gs_destroy(G->bwd);
    for (void* q : {(void*)G->rows, (void*)G->d_level_ptr, (void*)G->pk_col, (void*)G->pk_val,
                    (void*)G->pk_diag, (void*)G->b_lvl, (void*)G->wcol, (void*)G->d_clev,
                    (void*)G->win_xl, (void*)G->wpos, (void*)G->rcol, (void*)G->rpv,
                    (void*)G->rcode, (void*)G->rxl, (void*)G->wr_code, (void*)G->wr_pv,
                    (void*)G->wr_len, (void*)G->wr_d, (void*)G->wr_st})
      if (q) (void)hipFree(q);
    delete G;
  }
  return MLAMG_OK;
}

int mlamg_gs_levels(const mlamg_gs* G, int32_t* n_levels) {
  MLAMG_REQUIRE(G && n_levels, "NULL argument");
  *n_levels = G->n_levels;
  return MLAMG_OK;
}

int mlamg_gs_sweep(const mlamg_gs* G, double* x, const double* b, int iterations, void* stream) {
  MLAMG_REQUIRE(G && (G->A->n_rows == 0 || (x && b)), "NULL argument");
  return gs_sweep_impl(G, x, b, iterations, nullptr, S(stream));
}

}  // extern "C"
