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

int64_t gs_rows(const mlamg_gs* G) { return G->A->n_rows; }

int gs_sweep_impl(const mlamg_gs* G, double* x, const double* b, int iterations,
                  const int32_t* done, hipStream_t s) {
  const mlamg_csr* A = G->A;
  if (A->n_rows == 0 || iterations <= 0) return MLAMG_OK;
  if (G->max_level_rows <= kGsBlockMaxLevelRows && G->n_levels > 4) {
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
  *out = G;
  return MLAMG_OK;
}

int mlamg_gs_destroy(mlamg_gs* G) {
  if (G) {
    if (G->rows) (void)hipFree(G->rows);
    if (G->d_level_ptr) (void)hipFree(G->d_level_ptr);
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
