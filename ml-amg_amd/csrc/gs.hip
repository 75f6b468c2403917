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

int64_t gs_rows(const mlamg_gs* G) { return G->A->n_rows; }

int gs_sweep_impl(const mlamg_gs* G, double* x, const double* b, int iterations,
                  const int32_t* done, hipStream_t s) {
  const mlamg_csr* A = G->A;
  if (A->n_rows == 0 || iterations <= 0) return MLAMG_OK;
  const bool pipe = G->pk_k > 0 && G->n_levels > 4;
  if (pipe && G->max_level_rows <= 2 * kGsBlock) {
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
                    (void*)G->pk_diag, (void*)G->b_lvl})
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
