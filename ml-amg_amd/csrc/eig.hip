// lambda_max(D^-1 A) for the smoothed-aggregation weight omega = (4/3)/lambda_max
// (ns/lib/multigrid.py:105: ARPACK eigs(Dinv@A, k=1, which='LM')).
//
// D^-1 A is self-adjoint in the D inner product <x, y>_D = x^T D y (A symmetric, positive
// diagonal), so Lanczos in that inner product converges to its extreme eigenvalue with plain
// products by A: q_j D-orthonormal, z = A q_j, alpha_j = z . q_j,
// w = D^-1 z - alpha_j q_j - beta_j q_{j-1}, beta_{j+1} = ||w||_D, q_{j+1} = w / beta_{j+1}.
// The product z = A q is the operator's own SpMV kernel in whatever format it carries (the C4
// fine level in the row-pair format: 37 us instead of 250 us for a CSR pass with the scaling
// fused), the vector work is three streaming kernels and the three Lanczos vectors rotate by
// pointer. alpha_j and beta_j stay on the device; the host reads them every kCheck iterations
// to bisect the tridiagonal T_j for its largest eigenvalue. Reductions use a fixed order, so
// the result is deterministic.
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

// partial[b] = sum over the block's entries of z_i q_i
__global__ __launch_bounds__(256) void k_lz_dot(const double* __restrict__ z,
                                                const double* __restrict__ q, int64_t n,
                                                double* __restrict__ partial) {
  __shared__ double red[4];
  double acc = 0.0;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    acc += z[i] * q[i];
  const double t = block_sum256(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = t;
}

// w = D^-1 z - alpha q - beta q_prev ; partial = sum d_i w_i^2 (the D-norm)
__global__ __launch_bounds__(256) void k_lz_update(const double* __restrict__ z,
                                                   const double* __restrict__ dinv,
                                                   const double* __restrict__ d,
                                                   const double* __restrict__ q,
                                                   const double* __restrict__ qprev,
                                                   const double* __restrict__ alpha,
                                                   const double* __restrict__ beta, int64_t n,
                                                   double* __restrict__ w,
                                                   double* __restrict__ partial) {
  __shared__ double red[4];
  const double a = *alpha, bt = *beta;
  double acc = 0.0;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const double wi = (dinv[i] * z[i] - a * q[i]) - bt * qprev[i];
    w[i] = wi;
    acc += d[i] * (wi * wi);
  }
  const double t = block_sum256(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = t;
}

// w <- w / beta (beta = 0: breakdown, w = 0)
__global__ __launch_bounds__(256) void k_lz_scale(double* __restrict__ w,
                                                  const double* __restrict__ beta, int64_t n) {
  const double bt = *beta;
  const double inv = bt > 0.0 ? 1.0 / bt : 0.0;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    w[i] = w[i] * inv;
}

__device__ __forceinline__ uint64_t splitmix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// d_i = a_ii (sum of the stored diagonal entries), dinv = 1/d; q = random; partial = sum d q^2
__global__ __launch_bounds__(256) void k_lz_init(const int32_t* __restrict__ indptr,
                                                 const int32_t* __restrict__ indices,
                                                 const double* __restrict__ vals, int64_t n,
                                                 uint64_t seed, double* __restrict__ d,
                                                 double* __restrict__ dinv,
                                                 double* __restrict__ q,
                                                 double* __restrict__ partial) {
  __shared__ double red[4];
  double acc = 0.0;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    double di = 0.0;
    for (int k = indptr[i]; k < indptr[i + 1]; ++k)
      if (indices[k] == (int32_t)i) di += vals[k];
    d[i] = di;
    dinv[i] = 1.0 / di;
    const uint64_t r = splitmix(seed * 0x100000001B3ull + (uint64_t)i);
    const double x = (double)(r >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0;
    q[i] = x;
    acc += di * (x * x);
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
  const int m_max = (int)std::min<int64_t>(max_iter, n);
  double* base = nullptr;
  MLAMG_HIP(hipMalloc(&base, sizeof(double) * (n * 6 + nbv + 2 * (m_max + 2) + 1)));
  struct Free {
    double* p;
    ~Free() { (void)hipFree(p); }
  } guard{base};
  double* z = base;
  double* d = z + n;
  double* dinv = d + n;
  double* Q[3] = {dinv + n, dinv + 2 * n, dinv + 3 * n};  // q_prev, q, w
  double* partial = dinv + 4 * n;
  double* alpha = partial + nbv;
  double* beta = alpha + (m_max + 2);
  double* nrm0 = beta + (m_max + 2);
  MLAMG_HIP(hipMemsetAsync(Q[0], 0, sizeof(double) * n, s));
  MLAMG_HIP(hipMemsetAsync(beta, 0, sizeof(double) * (m_max + 2), s));
  hipLaunchKernelGGL(k_lz_init, dim3(nbv), dim3(256), 0, s, A->indptr, A->indices, A->data, n,
                     seed, d, dinv, Q[1], partial);
  hipLaunchKernelGGL(k_reduce_to, dim3(1), dim3(1024), 0, s, partial, nbv, nrm0, 1);
  hipLaunchKernelGGL(k_lz_scale, dim3(nbv), dim3(256), 0, s, Q[1], nrm0, n);
  MLAMG_HIP(hipGetLastError());

  const int kCheck = 32;
  std::vector<double> ha(m_max + 2), hb(m_max + 2);
  double theta_prev = -1.0, theta = 0.0;
  int j = 0;
  bool done = false;
  while (!done) {
    const int jend = std::min(m_max, j + kCheck);
    for (; j < jend; ++j) {
      MLAMG_TRY(launch_spmv_plain(A, Q[1], z, s));
      hipLaunchKernelGGL(k_lz_dot, dim3(nbv), dim3(256), 0, s, z, Q[1], n, partial);
      hipLaunchKernelGGL(k_reduce_to, dim3(1), dim3(1024), 0, s, partial, nbv, alpha + j, 0);
      // beta[j] couples q_j and q_{j-1}; beta[j+1] is the new norm
      hipLaunchKernelGGL(k_lz_update, dim3(nbv), dim3(256), 0, s, z, dinv, d, Q[1], Q[0],
                         alpha + j, beta + j, n, Q[2], partial);
      hipLaunchKernelGGL(k_reduce_to, dim3(1), dim3(1024), 0, s, partial, nbv, beta + j + 1, 1);
      hipLaunchKernelGGL(k_lz_scale, dim3(nbv), dim3(256), 0, s, Q[2], beta + j + 1, n);
      double* old = Q[0];  // q_prev <- q, q <- w, w <- (old q_prev)
      Q[0] = Q[1];
      Q[1] = Q[2];
      Q[2] = old;
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
