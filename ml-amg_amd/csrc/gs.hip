// Forward lexicographic Gauss-Seidel, pyamg relaxation.gauss_seidel semantics (the smoother of
// the reference driver, ns/lib/multigrid.py:175,184):
//     for i in 0..n-1: rsum = sum_{j != i} A_ij x_j (stored order); diag = A_ii (last one);
//                      if diag != 0: x_i = (b_i - rsum) / diag
// Row i reads x_j (j < i) after their update and x_j (j > i) before theirs. Level scheduling
// keeps exactly that order on the GPU: level(i) = 1 + max level(j) over j < i coupled to i in
// either direction (a_ij or a_ji nonzero), so every row of a level sees final values of all
// earlier-coupled rows and old values of all later-coupled rows; rows inside a level are
// independent. Results are therefore bit for bit those of the sequential sweep.
#include "common.hpp"

struct mlamg_gs {
  const mlamg_csr* A = nullptr;
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
  // windowed one-wave sweep (k_gs_win): x by level-order position in an LDS ring of 2^ring_log2
  // slots; wcol = the packed columns as positions (pads -1); chunks of levels staged into two
  // LDS buffers of win_cap + 1 positions; win_w = the widest level distance of a coupling
  int32_t win_rw = 0;  // rows per lane (0: no windowed sweep)
  int32_t ring_log2 = 0, win_cap = 0, win_w = 0, n_chunks = 0;
  int32_t* wcol = nullptr;
  int32_t* d_clev = nullptr;
  size_t win_lds = 0;
};

namespace mlamg {

__device__ __forceinline__ void gs_row(const int32_t* __restrict__ ip,
                                       const int32_t* __restrict__ ij,
                                       const double* __restrict__ ax, int32_t i, double* x,
                                       const double* __restrict__ b) {
  double rsum = 0.0, diag = 0.0;
  for (int k = ip[i]; k < ip[i + 1]; ++k) {
    const int32_t j = ij[k];
    if (j == i) diag = ax[k];
    else rsum += ax[k] * x[j];
  }
  if (diag != 0.0) x[i] = (b[i] - rsum) / diag;
}

__global__ __launch_bounds__(256) void k_gs_level(const int32_t* __restrict__ ip,
                                                  const int32_t* __restrict__ ij,
                                                  const double* __restrict__ ax,
                                                  const int32_t* __restrict__ rows, int32_t cnt,
                                                  double* x, const double* __restrict__ b,
                                                  const int32_t* done) {
  if (done && *done) return;
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= cnt) return;
  gs_row(ip, ij, ax, rows[t], x, b);
}

// The whole sweep in one workgroup: levels in order, a barrier between consecutive levels
// (workgroup-scope visibility of the x updates). For operators whose levels are narrow, where
// one launch per level would make the sweep launch-bound.
constexpr int kGsBlock = 1024;
constexpr int kGsBlockMaxLevelRows = 8 * kGsBlock;

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
      for (int32_t t = a + (int32_t)threadIdx.x; t < z; t += kGsBlock) gs_row(ip, ij, ax, rows[t], x, b);
      __syncthreads();
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

template <int R, int K>
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
        double rsum = 0.0;
#pragma unroll
        for (int k = 0; k < K; ++k)
          if (cur.col[u][k] >= 0) rsum += cur.val[u][k] * xv[u][k];
        if (cur.diag[u] != 0.0) x[cur.row[u]] = (cur.bi[u] - rsum) / cur.diag[u];
      }
      __syncthreads();
      if (l + 1 < n_levels) cur = nxt;
    }
  }
}

// Small systems (n <= kGsLdsMax): the same pipelined walk with x held in LDS for the whole sweep
// (x loaded once, written back once): a level's gathers and its updates are LDS accesses, so a
// level costs an LDS round trip and a barrier instead of a global-memory round trip.
constexpr int kGsLdsMax = 8192;  // 64 KB of x: within the default dynamic-LDS limit

template <int K>
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
        double rsum = 0.0;
#pragma unroll
        for (int k = 0; k < K; ++k)
          if (cur.col[0][k] >= 0) rsum += cur.val[0][k] * xv[k];
        if (cur.diag[0] != 0.0) xs[cur.row[0]] = (cur.bi[0] - rsum) / cur.diag[0];
      }
      __syncthreads();
      if (l + 1 < n_levels) cur = nxt;
    }
  }
  for (int64_t i = threadIdx.x; i < n; i += kGsBlock) x[i] = xs[i];
}

// Windowed one-wave sweep for levels of <= 64 * RW rows: wave 0 walks the levels with x held by
// level-order position in an LDS ring (a level's rows read positions at most W levels away, so
// levels [l - W, l + W] are all a step needs); waves 1-15 meanwhile stage the next chunk of
// levels (structure + the old x of the levels entering the window, loaded past L1) into the other
// buffer. Consecutive levels need only a wavefront fence; a chunk ends with a workgroup barrier.
// Pads point at the ring's zero slot (+0.0 products: the sum starts at +0.0 and never becomes
// -0.0, so bitwise neutral); a zero-diagonal row is left alone, as the sequential sweep does.
// Updated values go to the ring and to x. Same products, order and division: bitwise gs_row.
// 256 lanes: wave 0 gets the registers of RW rows x KM slots (+ the next level's) without spills;
// the 3 other waves stage
constexpr int kGsWinBlock = 256;

template <int KM, int RW>
__global__ __launch_bounds__(kGsWinBlock) void k_gs_win(const int32_t* __restrict__ rows,
                                                     const int32_t* __restrict__ lptr,
                                                     int32_t nlev,
                                                     const int32_t* __restrict__ clev,
                                                     int32_t nchunks,
                                                     const int32_t* __restrict__ wcol,
                                                     const double* __restrict__ pval,
                                                     const double* __restrict__ pdiag,
                                                     const double* __restrict__ blvl,
                                                     int ring_log2, int cap, int W,
                                                     int iterations, double* x,
                                                     const int32_t* done) {
  extern __shared__ double lds[];
  if (done && *done) return;
  const int tid = threadIdx.x, lane = tid & 63;
  const int RS = 1 << ring_log2, RM = RS - 1;
  double* ring = lds;  // RS slots + the zero slot (RS) + the sink slot (RS + 1)
  // per buffer (position-major, 16-byte aligned): vals cap+1 x KM | diag | b | cols (ring slots)
  // cap+1 x KM | target slot | row | level starts
  // (cap + 1) x (2 KM + 4) words of doubles + (cap + 1) x (KM + 4) words of ints, in doubles
  const int64_t buf = (((int64_t)(cap + 1) * (3 * KM + 8) + 1) / 2 + 1) & ~int64_t(1);
  double* bufs = lds + ((RS + 2 + 1) & ~1);
  if (tid == 0) ring[RS] = 0.0;
  auto stage = [&](int ch, double* wv, int t0, int nt) {
    double* wd = wv + (int64_t)(cap + 1) * KM;
    double* wb = wd + (cap + 1);
    int32_t* wc = reinterpret_cast<int32_t*>(wb + (cap + 1));
    int32_t* wt = wc + (int64_t)(cap + 1) * KM;
    int32_t* wr = wt + (cap + 1);
    int32_t* wl = wr + (cap + 1);
    const int l0 = clev[ch], l1 = clev[ch + 1];
    const int P0 = lptr[l0], cnt = lptr[l1] - P0;
    for (int q = t0; q < cnt * KM; q += nt) {
      const int32_t c = wcol[(int64_t)P0 * KM + q];
      wc[q] = c >= 0 ? (c & RM) : RS;
      wv[q] = pval[(int64_t)P0 * KM + q];
    }
    for (int q = t0; q < cnt; q += nt) {
      const double d = pdiag[P0 + q];
      wd[q] = d != 0.0 ? d : 1.0;
      wb[q] = blvl[P0 + q];
      wt[q] = d != 0.0 ? ((P0 + q) & RM) : RS + 1;  // zero diagonal: left alone (sink)
      wr[q] = d != 0.0 ? rows[P0 + q] : -1;
    }
    for (int q = t0; q <= l1 - l0; q += nt) wl[q] = lptr[l0 + q] - P0;
    if (t0 < KM) {  // the dummy position of lanes past a level's end
      wc[cnt * KM + t0] = RS;
      wv[cnt * KM + t0] = 0.0;
    }
    if (t0 == 0) {
      wd[cnt] = 1.0;
      wb[cnt] = 0.0;
      wt[cnt] = RS + 1;
      wr[cnt] = -1;
    }
    // the old x of the levels entering the window with this chunk (past L1: the previous
    // sweep of this launch wrote them from wave 0)
    const int la = ch == 0 ? 0 : min(nlev, l0 + W), lb = min(nlev, l1 + W);
    for (int p = lptr[la] + t0; p < lptr[lb]; p += nt)
      ring[p & RM] = __hip_atomic_load(x + rows[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  for (int it = 0; it < iterations; ++it) {
    stage(0, bufs, tid, kGsWinBlock);
    __syncthreads();
    for (int ch = 0; ch < nchunks; ++ch) {
      double* cur = bufs + (ch & 1) * buf;
      if (tid < 64) {
        const double* sv = cur;
        const double* sd = sv + (int64_t)(cap + 1) * KM;
        const double* sb = sd + (cap + 1);
        const int32_t* sc = reinterpret_cast<const int32_t*>(sb + (cap + 1));
        const int32_t* st = sc + (int64_t)(cap + 1) * KM;
        const int32_t* sr = st + (cap + 1);
        const int32_t* sl = sr + (cap + 1);
        const int nl = clev[ch + 1] - clev[ch];
        const int cnt = sl[nl];
        int c[RW][KM], tg[RW], rw[RW];
        double v[RW][KM], d[RW], bv[RW];
        auto load = [&](int l, int (&cc)[RW][KM], double (&vv)[RW][KM], double* dd, double* bb,
                        int* tt, int* rr) {
          const int a = sl[l], z = sl[l + 1];
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
            tt[u] = st[p];
            rr[u] = sr[p];
          }
        };
        load(0, c, v, d, bv, tg, rw);
        #pragma unroll 1
        for (int l = 0; l < nl; ++l) {
          double g[RW][KM];
#pragma unroll
          for (int u = 0; u < RW; ++u)
#pragma unroll
            for (int k = 0; k < KM; ++k) g[u][k] = ring[c[u][k]];
          int c2[RW][KM], tg2[RW], rw2[RW];
          double v2[RW][KM], d2[RW], bv2[RW];
          load(l + 1 < nl ? l + 1 : l, c2, v2, d2, bv2, tg2, rw2);
#pragma unroll
          for (int u = 0; u < RW; ++u) {
            double y = 0.0;
#pragma unroll
            for (int k = 0; k < KM; ++k) y += v[u][k] * g[u][k];
            const double xi = (bv[u] - y) / d[u];
            ring[tg[u]] = xi;
            if (rw[u] >= 0) x[rw[u]] = xi;
          }
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
            tg[u] = tg2[u];
            rw[u] = rw2[u];
          }
        }
      } else if (ch + 1 < nchunks) {
        stage(ch + 1, bufs + ((ch + 1) & 1) * buf, tid - 64, kGsWinBlock - 64);
      }
      __syncthreads();
    }
    __threadfence();  // this sweep's x stores before the next sweep's window loads
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

template <int R, int K>
static void launch_gs_pipe(const mlamg_gs* G, double* x, const double* b, int iterations,
                           const int32_t* done, hipStream_t s) {
  const int64_t n = G->A->n_rows;
  hipLaunchKernelGGL(k_gs_b_level, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, G->rows,
                     n, b, G->b_lvl, done);
  if (R == 1 && n <= kGsLdsMax && !gs_lds_disabled()) {
    hipLaunchKernelGGL((k_gs_lds<K>), dim3(1), dim3(kGsBlock), sizeof(double) * n, s, G->rows,
                       G->d_level_ptr, G->n_levels, n, G->pk_col, G->pk_val, G->pk_diag,
                       G->b_lvl, iterations, x, done);
    return;
  }
  hipLaunchKernelGGL((k_gs_pipe<R, K>), dim3(1), dim3(kGsBlock), 0, s, G->rows, G->d_level_ptr,
                     G->n_levels, G->pk_col, G->pk_val, G->pk_diag, G->b_lvl, iterations, x,
                     done);
}

static bool gs_win_disabled() {  // MLAMG_GS_NO_WIN=1: A/B runs, tests
  const char* e = std::getenv("MLAMG_GS_NO_WIN");
  return e && e[0] == '1';
}

template <int KM, int RW>
static void launch_gs_win(const mlamg_gs* G, double* x, const double* b, int iterations,
                          const int32_t* done, hipStream_t s) {
  const int64_t n = G->A->n_rows;
  hipLaunchKernelGGL(k_gs_b_level, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, G->rows,
                     n, b, G->b_lvl, done);
  hipLaunchKernelGGL((k_gs_win<KM, RW>), dim3(1), dim3(kGsWinBlock), G->win_lds, s, G->rows,
                     G->d_level_ptr, G->n_levels, G->d_clev, G->n_chunks, G->wcol, G->pk_val,
                     G->pk_diag, G->b_lvl, G->ring_log2, G->win_cap, G->win_w, iterations, x,
                     done);
}

int64_t gs_rows(const mlamg_gs* G) { return G->A->n_rows; }

int gs_sweep_impl(const mlamg_gs* G, double* x, const double* b, int iterations,
                  const int32_t* done, hipStream_t s) {
  const mlamg_csr* A = G->A;
  if (A->n_rows == 0 || iterations <= 0) return MLAMG_OK;
  const bool pipe = G->pk_k > 0 && G->n_levels > 4;
  if (pipe && G->win_rw > 0 && !gs_win_disabled()) {
    if (G->pk_k == 4) {
      switch (G->win_rw) {
        case 1: launch_gs_win<4, 1>(G, x, b, iterations, done, s); break;
        case 2: launch_gs_win<4, 2>(G, x, b, iterations, done, s); break;
        case 3: launch_gs_win<4, 3>(G, x, b, iterations, done, s); break;
        default: launch_gs_win<4, 4>(G, x, b, iterations, done, s); break;
      }
    } else {
      if (G->win_rw == 1) launch_gs_win<8, 1>(G, x, b, iterations, done, s);
      else launch_gs_win<8, 2>(G, x, b, iterations, done, s);
    }
  } else if (pipe && G->max_level_rows <= 2 * kGsBlock) {
    const bool one = G->max_level_rows <= kGsBlock;
    if (G->pk_k == 4) {
      if (one) launch_gs_pipe<1, 4>(G, x, b, iterations, done, s);
      else launch_gs_pipe<2, 4>(G, x, b, iterations, done, s);
    } else {
      if (one) launch_gs_pipe<1, 8>(G, x, b, iterations, done, s);
      else launch_gs_pipe<2, 8>(G, x, b, iterations, done, s);
    }
  } else if (G->max_level_rows <= kGsBlockMaxLevelRows && G->n_levels > 4) {
    hipLaunchKernelGGL(k_gs_block, dim3(1), dim3(kGsBlock), 0, s, A->indptr, A->indices, A->data,
                       G->rows, G->d_level_ptr, G->n_levels, iterations, x, b, done);
  } else {
    for (int it = 0; it < iterations; ++it) {
      for (int32_t l = 0; l < G->n_levels; ++l) {
        const int32_t a = G->level_ptr[l], cnt = G->level_ptr[l + 1] - a;
        hipLaunchKernelGGL(k_gs_level, dim3((cnt + 255) / 256), dim3(256), 0, s, A->indptr,
                           A->indices, A->data, G->rows + a, cnt, x, b, done);
      }
    }
  }
  MLAMG_HIP(hipGetLastError());
  return MLAMG_OK;
}

}  // namespace mlamg

using namespace mlamg;

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
  const int rw_max = K == 4 ? 4 : 2;
  const int rw = (G->max_level_rows + 63) / 64;
  if (rw < 1 || rw > rw_max || nlev <= 4) return;
  int W = 0;
  for (int64_t i = 0; i < n; ++i)
    for (int k = ip[i]; k < ip[i + 1]; ++k)
      if (ij[k] != i) W = std::max(W, std::abs(level[ij[k]] - level[i]));
  const std::vector<int32_t>& lp = G->level_ptr;
  const size_t budget = 150 * 1024;
  const size_t per_pos = (size_t)(12 * K + 32);
  for (int cap = 4096; cap >= G->max_level_rows; cap = cap * 3 / 4) {
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
    const size_t bufs = 2 * ((size_t)(cap + 1) * per_pos + 32);
    if (ring + bufs > budget) continue;
    std::vector<int32_t> pos(n), wcol((size_t)n * K, -1);
    for (int64_t p = 0; p < n; ++p) pos[rows[p]] = (int32_t)p;
    for (size_t q = 0; q < (size_t)n * K; ++q)
      if (pcol[q] >= 0) wcol[q] = pos[pcol[q]];
    if (hipMalloc(&G->wcol, sizeof(int32_t) * std::max<size_t>((size_t)n * K, 1)) != hipSuccess ||
        hipMalloc(&G->d_clev, sizeof(int32_t) * clev.size()) != hipSuccess) {
      if (G->wcol) (void)hipFree(G->wcol);
      G->wcol = nullptr;
      return;
    }
    (void)hipMemcpy(G->wcol, wcol.data(), sizeof(int32_t) * (size_t)n * K, hipMemcpyHostToDevice);
    (void)hipMemcpy(G->d_clev, clev.data(), sizeof(int32_t) * clev.size(), hipMemcpyHostToDevice);
    G->win_w = W;
    G->win_cap = cap;
    G->ring_log2 = lg;
    G->n_chunks = nch;
    G->win_lds = ring + bufs + 64;
    G->win_rw = rw;
    return;
  }
}

extern "C" {

int mlamg_gs_create(const mlamg_csr* A, mlamg_gs** out, void* stream) {
  MLAMG_REQUIRE(A && out, "NULL argument");
  MLAMG_REQUIRE(A->n_rows == A->n_cols, "square matrix required");
  hipStream_t s = S(stream);
  const int64_t n = A->n_rows;
  std::vector<int32_t> ip(n + 1), ij(A->nnz);
  MLAMG_HIP(hipMemcpyAsync(ip.data(), A->indptr, sizeof(int32_t) * (n + 1), hipMemcpyDeviceToHost, s));
  if (A->nnz)
    MLAMG_HIP(hipMemcpyAsync(ij.data(), A->indices, sizeof(int32_t) * A->nnz, hipMemcpyDeviceToHost, s));
  MLAMG_HIP(hipStreamSynchronize(s));
  std::vector<int32_t> level(n, 0), req(n, 0);
  int32_t nlev = 0;
  for (int64_t i = 0; i < n; ++i) {
    int32_t L = req[i];
    for (int k = ip[i]; k < ip[i + 1]; ++k) {
      const int32_t j = ij[k];
      if (j < i) L = std::max(L, level[j] + 1);
    }
    level[i] = L;
    for (int k = ip[i]; k < ip[i + 1]; ++k) {
      const int32_t j = ij[k];
      if (j > i) req[j] = std::max(req[j], L + 1);
    }
    nlev = std::max(nlev, L + 1);
  }
  auto* G = new mlamg_gs();
  G->A = A;
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
    if (K) {
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
      }
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
        setup_window(G, ip, ij, level, rows, pcol, K);
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

int mlamg_gs_destroy(mlamg_gs* G) {
  if (G) {
    for (void* q : {(void*)G->rows, (void*)G->d_level_ptr, (void*)G->pk_col, (void*)G->pk_val,
                    (void*)G->pk_diag, (void*)G->b_lvl, (void*)G->wcol, (void*)G->d_clev})
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
