// Vector kernels of the V-cycle and device-wide scans.
//   norm2      ||x||_2, deterministic two-pass reduction      (multigrid.py:191,193 la.norm)
//   diag_inv   dinv_w[i] = (1.0/a_ii)*omega                    (MLAMG.py:104; multigrid.py:41)
//   jacobi_r   x[i] += dinv_w[i]*r[i]   (Jacobi sweep from a residual already formed, used when
//              the end-of-cycle residual b - A@x is reused by the next pre-smoothing sweep)
//   scale      x[i] = dinv_w[i]*b[i]    (first sweep from a zero initial guess: 0 + d*(b - A@0))
#include "common.hpp"

#include <rocprim/rocprim.hpp>

namespace mlamg {

__device__ __forceinline__ double wave_sum_v(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// pass 1: per-block partial sums of x^2 over a fixed grid (grid-stride, fixed order)
__global__ __launch_bounds__(256) void k_sumsq_partial(const double* __restrict__ x, int64_t n,
                                                       double* __restrict__ partial,
                                                       const int32_t* done) {
  __shared__ double red[4];
  if (done && *done) return;
  double s = 0.0;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    s += x[i] * x[i];
  s = wave_sum_v(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
}

__global__ __launch_bounds__(1024) void k_sum_sqrt(const double* __restrict__ partial, int n,
                                                   double* out, const int32_t* done) {
  __shared__ double red[16];
  if (done && *done) return;
  double s = 0.0;
  s = strided_sum(partial, n, threadIdx.x, 1024);
  s = wave_sum_v(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int i = 0; i < 16; ++i) t += red[i];
    *out = sqrt(t);
  }
}

constexpr int kNormBlocks = 1024;

int norm2_impl(const double* x, int64_t n, double* out, double* partial, const int32_t* done,
               hipStream_t s) {
  if (!partial) partial = static_cast<double*>(scratch(sizeof(double) * kNormBlocks, 1));
  MLAMG_REQUIRE(partial, "scratch allocation failed");
  int nb = (int)std::min<int64_t>(kNormBlocks, std::max<int64_t>(1, (n + 255) / 256));
  hipLaunchKernelGGL(k_sumsq_partial, dim3(nb), dim3(256), 0, s, x, n, partial, done);
  hipLaunchKernelGGL(k_sum_sqrt, dim3(1), dim3(1024), 0, s, partial, nb, out, done);
  MLAMG_HIP(hipGetLastError());
  return MLAMG_OK;
}

__global__ __launch_bounds__(1024) void k_sum_hist(const double* __restrict__ partial, int n,
                                                   double* hist, int32_t* counter, int32_t* done,
                                                   double tol) {
  __shared__ double red[16];
  if (done && *done) return;
  double s = strided_sum(partial, n, threadIdx.x, 1024);
  s = wave_sum_v(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int i = 0; i < 16; ++i) t += red[i];
    const double nrm = sqrt(t);
    const int c = *counter;
    if (hist) hist[c] = nrm;
    *counter = c + 1;
    if (tol >= 0.0 && nrm <= tol) *done = 1;
  }
}

int norm_hist_impl(const double* x, int64_t n, double* partial, double* hist, int32_t* counter,
                   int32_t* done, double tol, hipStream_t s) {
  const int nb = (int)std::min<int64_t>(kNormBlocks, std::max<int64_t>(1, (n + 255) / 256));
  hipLaunchKernelGGL(k_sumsq_partial, dim3(nb), dim3(256), 0, s, x, n, partial, done);
  hipLaunchKernelGGL(k_sum_hist, dim3(1), dim3(1024), 0, s, partial, nb, hist, counter, done, tol);
  MLAMG_HIP(hipGetLastError());
  return MLAMG_OK;
}

__global__ __launch_bounds__(256) void k_diag_inv(const int32_t* __restrict__ indptr,
                                                  const int32_t* __restrict__ indices,
                                                  const double* __restrict__ vals, int64_t n,
                                                  double omega, double* __restrict__ dinv) {
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  // scipy csr_diagonal: sum of duplicate diagonal entries, 0 if absent
  double d = 0.0;
  for (int k = indptr[i]; k < indptr[i + 1]; ++k)
    if (indices[k] == (int32_t)i) d += vals[k];
  const double inv = 1.0 / d;
  dinv[i] = inv * omega;
}

__global__ __launch_bounds__(256) void k_axpy_diag(double* __restrict__ x,
                                                   const double* __restrict__ d,
                                                   const double* __restrict__ r, int64_t n,
                                                   const int32_t* done) {
  if (done && *done) return;
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i < n) x[i] = x[i] + d[i] * r[i];
}

__global__ __launch_bounds__(256) void k_mul_diag(double* __restrict__ x,
                                                  const double* __restrict__ d,
                                                  const double* __restrict__ b, int64_t n,
                                                  const int32_t* done) {
  if (done && *done) return;
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  // 0 + d*(b - 0): equals d*b bit for bit (b - 0 = b; 0 + y = y)
  if (i < n) x[i] = d[i] * b[i];
}

int jacobi_from_residual(double* x, const double* dinv, const double* r, int64_t n,
                         const int32_t* done, hipStream_t s) {
  if (n == 0) return MLAMG_OK;
  hipLaunchKernelGGL(k_axpy_diag, dim3((n + 255) / 256), dim3(256), 0, s, x, dinv, r, n, done);
  MLAMG_HIP(hipGetLastError());
  return MLAMG_OK;
}

int jacobi_from_zero(double* x, const double* dinv, const double* b, int64_t n,
                     const int32_t* done, hipStream_t s) {
  if (n == 0) return MLAMG_OK;
  hipLaunchKernelGGL(k_mul_diag, dim3((n + 255) / 256), dim3(256), 0, s, x, dinv, b, n, done);
  MLAMG_HIP(hipGetLastError());
  return MLAMG_OK;
}

// ---------------------------------------------------------------- scans (rocPRIM)
template <class T>
static int exclusive_scan_t(const T* in, T* out, int64_t n, hipStream_t s) {
  // out has n+1 entries; out[n] = total
  size_t tmp_bytes = 0;
  MLAMG_HIP(rocprim::exclusive_scan(nullptr, tmp_bytes, in, out, T(0), (size_t)n,
                                    rocprim::plus<T>(), s));
  void* tmp = scratch(tmp_bytes + 16, 2);
  MLAMG_REQUIRE(tmp, "scratch allocation failed");
  if (n > 0)
    MLAMG_HIP(rocprim::exclusive_scan(tmp, tmp_bytes, in, out, T(0), (size_t)n,
                                      rocprim::plus<T>(), s));
  // total = out[n-1] + in[n-1]
  return MLAMG_OK;
}

template <class T>
__global__ void k_scan_total(const T* in, T* out, int64_t n) {
  out[n] = n > 0 ? out[n - 1] + in[n - 1] : T(0);
}

int exclusive_scan_i64(const int64_t* in, int64_t* out, int64_t n, hipStream_t s) {
  MLAMG_TRY(exclusive_scan_t<int64_t>(in, out, n, s));
  hipLaunchKernelGGL(k_scan_total<int64_t>, dim3(1), dim3(1), 0, s, in, out, n);
  MLAMG_HIP(hipGetLastError());
  return MLAMG_OK;
}

int exclusive_scan_i32(const int32_t* in, int32_t* out, int64_t n, hipStream_t s) {
  MLAMG_TRY(exclusive_scan_t<int32_t>(in, out, n, s));
  hipLaunchKernelGGL(k_scan_total<int32_t>, dim3(1), dim3(1), 0, s, in, out, n);
  MLAMG_HIP(hipGetLastError());
  return MLAMG_OK;
}

}  // namespace mlamg

using namespace mlamg;

extern "C" {

int mlamg_norm2(const double* x, int64_t n, double* out, void* stream) {
  MLAMG_REQUIRE(out && (n == 0 || x), "NULL argument");
  MLAMG_REQUIRE(n >= 0, "n < 0");
  return norm2_impl(x, n, out, nullptr, nullptr, S(stream));
}

int mlamg_diag_inv(const mlamg_csr* A, double omega, double* dinv_w, void* stream) {
  MLAMG_REQUIRE(A && (A->n_rows == 0 || dinv_w), "NULL argument");
  MLAMG_REQUIRE(A->n_rows == A->n_cols, "diag_inv needs a square matrix");
  if (A->n_rows == 0) return MLAMG_OK;
  hipLaunchKernelGGL(k_diag_inv, dim3((A->n_rows + 255) / 256), dim3(256), 0, S(stream),
                     A->indptr, A->indices, A->data, A->n_rows, omega, dinv_w);
  MLAMG_HIP(hipGetLastError());
  return MLAMG_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- index validation
namespace mlamg {
__global__ void k_count_out_of_range(const int32_t* __restrict__ a, int64_t n, int64_t lo,
                                     int64_t hi, unsigned long long* bad) {
  unsigned long long c = 0;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t v = a[i];
    c += (v < lo || v >= hi) ? 1ull : 0ull;
  }
  if (c) atomicAdd(bad, c);
}

// number of entries of a[0..n) outside [lo, hi); syncs `s`
int count_out_of_range(const int32_t* a, int64_t n, int64_t lo, int64_t hi, hipStream_t s,
                       int64_t* bad_out) {
  *bad_out = 0;
  if (n <= 0) return MLAMG_OK;
  unsigned long long* d = static_cast<unsigned long long*>(scratch(sizeof(unsigned long long), 3));
  MLAMG_REQUIRE(d, "scratch allocation failed");
  MLAMG_HIP(hipMemsetAsync(d, 0, sizeof(unsigned long long), s));
  const int nb = (int)std::min<int64_t>(2048, (n + 255) / 256);
  hipLaunchKernelGGL(k_count_out_of_range, dim3(nb), dim3(256), 0, s, a, n, lo, hi, d);
  MLAMG_HIP(hipGetLastError());
  unsigned long long h = 0;
  MLAMG_HIP(hipMemcpyAsync(&h, d, sizeof(h), hipMemcpyDeviceToHost, s));
  MLAMG_HIP(hipStreamSynchronize(s));
  *bad_out = (int64_t)h;
  return MLAMG_OK;
}
}  // namespace mlamg

// ---------------------------------------------------------------- operator fingerprint
// 64-bit fingerprint of a CSR operator (rows, columns, value bits, per-entry position): the sum
// mod 2^64 of a splitmix64 mix of every (row, row length) and (entry, column, value bits) —
// addition commutes, so the result does not depend on the launch geometry. Keys the format
// autotune's cache (mlamg/hierarchy.py): an operator rebuilt with the same entries reuses its
// timing decision.
namespace mlamg {
__device__ __forceinline__ uint64_t fp_mix(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__global__ __launch_bounds__(256) void k_csr_fp(const int32_t* __restrict__ ip,
                                                const int32_t* __restrict__ ij,
                                                const double* __restrict__ v, int64_t n,
                                                int64_t nnz, unsigned long long* __restrict__ out) {
  uint64_t h = 0;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
    h += fp_mix(((uint64_t)i << 32) ^ (uint64_t)(uint32_t)(ip[i + 1] - ip[i]) ^ 0x5555ull);
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < nnz; e += stride)
    h += fp_mix(fp_mix(((uint64_t)e << 32) ^ (uint64_t)(uint32_t)ij[e]) ^
                (uint64_t)__double_as_longlong(v[e]));
  for (int o = 32; o > 0; o >>= 1) h += __shfl_xor(h, o);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, (unsigned long long)h);
}
}  // namespace mlamg

extern "C" int mlamg_csr_fingerprint(const mlamg_csr* A, uint64_t* fp_host, void* stream) {
  using namespace mlamg;
  MLAMG_REQUIRE(A && fp_host, "NULL argument");
  hipStream_t s = S(stream);
  unsigned long long* d = nullptr;
  MLAMG_HIP(hipMalloc(&d, sizeof(unsigned long long)));
  unsigned long long h = 0;
  hipError_t e = hipMemsetAsync(d, 0, sizeof(unsigned long long), s);
  if (e == hipSuccess) {
    const int64_t m = std::max<int64_t>(A->n_rows, A->nnz);
    const unsigned g = (unsigned)std::min<int64_t>(std::max<int64_t>((m + 255) / 256, 1), 4096);
    hipLaunchKernelGGL(k_csr_fp, dim3(g), dim3(256), 0, s, A->indptr, A->indices, A->data,
                       A->n_rows, A->nnz, d);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(&h, d, sizeof(h), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  (void)hipFree(d);
  MLAMG_HIP(e);
  *fp_host = (uint64_t)h ^ ((uint64_t)A->n_cols * 0x9e3779b97f4a7c15ull);
  return MLAMG_OK;
}
