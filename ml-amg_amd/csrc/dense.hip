// Coarsest-level direct solve. Replaces spla.factorized / splu (ns/lib/multigrid.py:168,
// ns/preconditioner/MLAMG.py:122): the coarse operator (n_c up to a few thousand) is expanded
// to a dense row-major matrix and inverted in place by Gauss-Jordan elimination with partial
// pivoting (fp64) once at setup; each V-cycle's coarse solve is then one dense GEMV
// (n_c^2 * 8 bytes, HBM/L2-bound) instead of two sequential triangular solves.
#include "common.hpp"

#include <cmath>

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
  // loop is otherwise a chain of dependent memory round trips: ~10 us for n = 1008)
  int64_t j = lane;
  for (; j + 7 * 64 < n; j += 8 * 64) {
    double m[8], v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      m[u] = r[j + u * 64];
      v[u] = b[j + u * 64];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) s += m[u] * v[u];
  }
  for (; j < n; j += 64) s += r[j] * b[j];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (lane == 0) x[row] = s;
}

int dense_solve_impl(const mlamg_dense* D, const double* b, double* x, const int32_t* done,
                     hipStream_t s) {
  if (D->n == 0) return MLAMG_OK;
  hipLaunchKernelGGL(k_gemv, dim3((D->n + 3) / 4), dim3(256), 0, s, D->inv, D->n, b, x, done);
  MLAMG_HIP(hipGetLastError());
  return MLAMG_OK;
}

}  // namespace mlamg

using namespace mlamg;

extern "C" {

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

int mlamg_dense_destroy(mlamg_dense* D) {
  if (D) {
    if (D->inv) (void)hipFree(D->inv);
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
