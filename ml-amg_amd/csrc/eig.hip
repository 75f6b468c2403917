// lambda_max(D^-1 A) for the smoothed-aggregation weight omega = (4/3)/lambda_max
// (ns/lib/multigrid.py:105: ARPACK eigs(Dinv@A, k=1, which='LM')).
//
// D^-1 A is similar to the symmetric B = D^-1/2 A D^-1/2 (A symmetric, positive diagonal), so
// plain Lanczos on B converges to the same extreme eigenvalue. Every iteration is one CSR-stream
// SpMV (with the D^-1/2 scaling and the Rayleigh dot fused into its epilogue) plus one fused
// update/norm kernel; alpha_j and beta_j stay on the device and the host only reads them every
// kCheck iterations to bisect the tridiagonal T_j for its largest eigenvalue. Reductions use a
// fixed order, so the result is deterministic.
#include "common.hpp"

#include <cmath>

namespace mlamg {

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ double block_sum256(double v, double* red) {
  v = wsum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double t = ((red[0] + red[1]) + red[2]) + red[3];
  __syncthreads();
  return t;
}

// w = h .* (A u), partial[b] = sum over the block of w_i * v_i
__global__ __launch_bounds__(kThreads) void k_lanczos_spmv(
    const int32_t* __restrict__ indptr, const int32_t* __restrict__ indices,
    const double* __restrict__ vals, const int32_t* __restrict__ blk,
    const double* __restrict__ u, const double* __restrict__ h, const double* __restrict__ v,
    double* __restrict__ w, double* __restrict__ partial) {
  __shared__ double prod[kBlockNnz];
  __shared__ int32_t rp[kBlockRows + 1];
  __shared__ double red[4];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int r0 = blk[b], r1 = blk[b + 1], nr = r1 - r0;
  const int e0 = indptr[r0], ne = indptr[r1] - e0;
  double acc = 0.0;
  if (ne <= kBlockNnz) {
    for (int t = tid; t <= nr; t += kThreads) rp[t] = indptr[r0 + t] - e0;
    for (int e = tid; e < ne; e += kThreads) prod[e] = vals[e0 + e] * u[indices[e0 + e]];
    __syncthreads();
    for (int t = tid; t < nr; t += kThreads) {
      double s = 0.0;
      for (int k = rp[t]; k < rp[t + 1]; ++k) s += prod[k];
      const int i = r0 + t;
      const double wi = h[i] * s;
      w[i] = wi;
      acc += wi * v[i];
    }
  } else {
    double s = 0.0;
    for (int c = 0; c < ne; c += kBlockNnz) {
      const int m = min(kBlockNnz, ne - c);
      for (int e = tid; e < m; e += kThreads) prod[e] = vals[e0 + c + e] * u[indices[e0 + c + e]];
      __syncthreads();
      if (tid == 0)
        for (int k = 0; k < m; ++k) s += prod[k];
      __syncthreads();
    }
    if (tid == 0) {
      const double wi = h[r0] * s;
      w[r0] = wi;
      acc = wi * v[r0];
    }
  }
  const double t = block_sum256(acc, red);
  if (tid == 0) partial[b] = t;
}

__global__ __launch_bounds__(1024) void k_reduce_to(const double* __restrict__ partial, int n,
                                                    double* __restrict__ out, int take_sqrt) {
  __shared__ double red[16];
  double s = 0.0;
  s = strided_sum(partial, n, threadIdx.x, 1024);
  s = wsum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int i = 0; i < 16; ++i) t += red[i];
    *out = take_sqrt ? sqrt(t) : t;
  }
}

// w -= alpha*v + beta*vprev ; partial = sum w^2
__global__ __launch_bounds__(256) void k_lanczos_update(double* __restrict__ w,
                                                        const double* __restrict__ v,
                                                        const double* __restrict__ vprev,
                                                        const double* __restrict__ alpha,
                                                        const double* __restrict__ beta,
                                                        int64_t n, double* __restrict__ partial) {
  __shared__ double red[4];
  const double a = *alpha, bt = *beta;
  double acc = 0.0;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const double wi = (w[i] - a * v[i]) - bt * vprev[i];
    w[i] = wi;
    acc += wi * wi;
  }
  const double t = block_sum256(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = t;
}

// vprev <- v ; v <- w / beta ; u <- h .* v
__global__ __launch_bounds__(256) void k_lanczos_next(double* __restrict__ vprev,
                                                      double* __restrict__ v,
                                                      const double* __restrict__ w,
                                                      const double* __restrict__ h,
                                                      double* __restrict__ u,
                                                      const double* __restrict__ beta, int64_t n) {
  const double bt = *beta;
  const double inv = bt > 0.0 ? 1.0 / bt : 0.0;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    vprev[i] = v[i];
    const double vi = w[i] * inv;
    v[i] = vi;
    u[i] = h[i] * vi;
  }
}

__device__ __forceinline__ uint64_t splitmix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// h_i = 1/sqrt(a_ii); v = random; partial = sum v^2
__global__ __launch_bounds__(256) void k_lanczos_init(const int32_t* __restrict__ indptr,
                                                      const int32_t* __restrict__ indices,
                                                      const double* __restrict__ vals,
                                                      int64_t n, uint64_t seed,
                                                      double* __restrict__ h,
                                                      double* __restrict__ w,
                                                      double* __restrict__ partial) {
  __shared__ double red[4];
  double acc = 0.0;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    double d = 0.0;
    for (int k = indptr[i]; k < indptr[i + 1]; ++k)
      if (indices[k] == (int32_t)i) d += vals[k];
    h[i] = 1.0 / sqrt(d);
    const uint64_t r = splitmix(seed * 0x100000001B3ull + (uint64_t)i);
    const double x = (double)(r >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0;
    w[i] = x;
    acc += x * x;
  }
  const double t = block_sum256(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = t;
}

// number of eigenvalues of the symmetric tridiagonal (a[0..m), b[1..m)) smaller than x
static int sturm_count(const std::vector<double>& a, const std::vector<double>& b, int m, double x) {
  int cnt = 0;
  double q = 1.0;
  for (int i = 0; i < m; ++i) {
    const double bb = i > 0 ? b[i] * b[i] : 0.0;
    q = (a[i] - x) - (i > 0 ? bb / q : 0.0);
    if (q == 0.0) q = -1e-300;
    if (q < 0.0) ++cnt;
  }
  return cnt;
}

static double tridiag_max_eig(const std::vector<double>& a, const std::vector<double>& b, int m) {
  double lo = a[0], hi = a[0];
  for (int i = 0; i < m; ++i) {
    const double r = (i > 0 ? std::fabs(b[i]) : 0.0) + (i + 1 < m ? std::fabs(b[i + 1]) : 0.0);
    lo = std::min(lo, a[i] - r);
    hi = std::max(hi, a[i] + r);
  }
  for (int it = 0; it < 200; ++it) {
    const double mid = 0.5 * (lo + hi);
    if (mid <= lo || mid >= hi) break;
    if (sturm_count(a, b, m, mid) == m) hi = mid;  // all eigenvalues < mid
    else lo = mid;
  }
  return hi;
}

int launch_spmv_plain(const mlamg_csr* A, const double* x, double* y, hipStream_t s);

}  // namespace mlamg

using namespace mlamg;

extern "C" int mlamg_lambda_max_dinvA(const mlamg_csr* A, int max_iter, double tol, uint64_t seed,
                                      double* lam_host, int* iters_host, void* stream) {
  MLAMG_REQUIRE(A && lam_host, "NULL argument");
  MLAMG_REQUIRE(A->n_rows == A->n_cols, "square matrix required");
  MLAMG_REQUIRE(max_iter > 0, "max_iter must be positive");
  hipStream_t s = S(stream);
  const int64_t n = A->n_rows;
  if (n == 0) {
    *lam_host = 0.0;
    if (iters_host) *iters_host = 0;
    return MLAMG_OK;
  }
  const int nbv = (int)std::min<int64_t>(1024, (n + 255) / 256);
  const int npart = std::max<int>(A->n_blocks, nbv);
  const int m_max = (int)std::min<int64_t>(max_iter, n);
  double *h, *u, *v, *vprev, *w, *partial, *alpha, *beta;
  MLAMG_HIP(hipMalloc(&h, sizeof(double) * n * 5 + sizeof(double) * (npart + 2 * (m_max + 2))));
  u = h + n;
  v = u + n;
  vprev = v + n;
  w = vprev + n;
  partial = w + n;
  alpha = partial + npart;
  beta = alpha + (m_max + 2);
  struct Free {
    double* p;
    ~Free() { (void)hipFree(p); }
  } guard{h};
  MLAMG_HIP(hipMemsetAsync(vprev, 0, sizeof(double) * n, s));
  MLAMG_HIP(hipMemsetAsync(beta, 0, sizeof(double) * (m_max + 2), s));
  hipLaunchKernelGGL(k_lanczos_init, dim3(nbv), dim3(256), 0, s, A->indptr, A->indices, A->data,
                     n, seed, h, w, partial);
  hipLaunchKernelGGL(k_reduce_to, dim3(1), dim3(1024), 0, s, partial, nbv, beta + 0, 1);
  // v1 = w / ||w||  (beta[0] is reset to 0 after use)
  hipLaunchKernelGGL(k_lanczos_next, dim3(nbv), dim3(256), 0, s, vprev, v, w, h, u, beta + 0, n);
  MLAMG_HIP(hipMemsetAsync(vprev, 0, sizeof(double) * n, s));
  MLAMG_HIP(hipMemsetAsync(beta, 0, sizeof(double), s));
  MLAMG_HIP(hipGetLastError());

  const int kCheck = 32;
  std::vector<double> ha(m_max + 2), hb(m_max + 2);
  double theta_prev = -1.0, theta = 0.0;
  int j = 0;
  bool done = false;
  while (!done) {
    const int jend = std::min(m_max, j + kCheck);
    for (; j < jend; ++j) {
      hipLaunchKernelGGL(k_lanczos_spmv, dim3(A->n_blocks), dim3(kThreads), 0, s, A->indptr,
                         A->indices, A->data, A->blk, u, h, v, w, partial);
      hipLaunchKernelGGL(k_reduce_to, dim3(1), dim3(1024), 0, s, partial, A->n_blocks, alpha + j,
                         0);
      // beta[j] couples v_j and v_{j-1}; beta[j+1] is the new norm
      hipLaunchKernelGGL(k_lanczos_update, dim3(nbv), dim3(256), 0, s, w, v, vprev, alpha + j,
                         beta + j, n, partial);
      hipLaunchKernelGGL(k_reduce_to, dim3(1), dim3(1024), 0, s, partial, nbv, beta + j + 1, 1);
      hipLaunchKernelGGL(k_lanczos_next, dim3(nbv), dim3(256), 0, s, vprev, v, w, h, u,
                         beta + j + 1, n);
    }
    MLAMG_HIP(hipGetLastError());
    MLAMG_HIP(hipMemcpyAsync(ha.data(), alpha, sizeof(double) * j, hipMemcpyDeviceToHost, s));
    MLAMG_HIP(hipMemcpyAsync(hb.data(), beta, sizeof(double) * (j + 1), hipMemcpyDeviceToHost, s));
    MLAMG_HIP(hipStreamSynchronize(s));
    // T_j: diagonal ha[0..j), off-diagonal hb[1..j)
    int m = j;
    bool breakdown = false;
    for (int i = 1; i <= j; ++i) {
      if (!(hb[i] > 1e-14 * std::fabs(ha[i - 1]) + 1e-300)) {
        m = i;
        breakdown = true;
        break;
      }
    }
    theta = tridiag_max_eig(ha, hb, m);
    if (breakdown || j >= m_max) done = true;
    if (theta_prev > 0.0 && std::fabs(theta - theta_prev) <= tol * std::fabs(theta)) done = true;
    theta_prev = theta;
  }
  *lam_host = theta;
  if (iters_host) *iters_host = j;
  return MLAMG_OK;
}
