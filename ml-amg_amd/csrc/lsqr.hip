// LSQR (Paige & Saunders) on the device: the coarse solve of the reference's singular two-level
// cycle, x += P @ spla.lsqr(P.T@A@P, P.T@(b - A@x))[0] (ns/lib/multigrid.py:178-179), with
// scipy's defaults (damp = 0, atol = btol = 1e-6, conlim = 1e8, iter_lim = 2 n, x0 = 0).
//
// Third-party algorithm restated: scipy.sparse.linalg.lsqr (scipy 1.15, the version in this
// image; the reference pins none). Every elementwise update is scipy's expression with the same
// roundings ((1/beta)*u, t - alfa*u, x + t1*w, ...); the scalar recurrences (Givens rotation
// _sym_ortho, norm / condition estimates, stopping tests istop 1..7 in scipy's order) run in one
// device thread, so the iteration needs no host round trip. Norms are fixed-order device
// reductions where scipy calls BLAS ddot: iterates agree to fp64 rounding, not bitwise.
//
// Per iteration, all on one stream, every kernel a no-op once the done flag is up:
//   t = A v | u = t - alfa u, sum u^2 | beta, anorm | u /= beta | t = A^T u | v = t - beta v,
//   sum v^2 | alfa, rotation, x-norm estimates | v /= alfa, x += t1 w, w = v + t2 w, sum dk^2 |
//   ddnorm, tests, istop
// The host checks the flag every kLsqrChunk iterations.
#include "common.hpp"

#include <cmath>
#include <limits>

namespace mlamg {

namespace {
constexpr int kLsqrChunk = 8;
constexpr int kLsqrBlocks = 512;  // fixed grid of the vector kernels: fixed reduction order

struct LsqrState {
  double alfa, beta, anorm, ddnorm, xnorm, xxnorm, z, cs2, sn2, rhobar, phibar, bnorm, res2;
  double rnorm, arnorm, t1, t2, rinv, binv, ainv;
  double atol, btol, ctol;
  int32_t done, istop, itn, iter_lim;
};

__device__ __forceinline__ double block_sum(double v, double* red) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x == 0)
    for (int i = 0; i < 4; ++i) t += red[i];
  return t;
}

// single-workgroup fixed-order sum of the kLsqrBlocks partials (thread 0 gets it)
__device__ __forceinline__ double partial_total(const double* __restrict__ p, double* red) {
  double s = strided_sum(p, kLsqrBlocks, threadIdx.x, 256);
  return block_sum(s, red);
}

// u = t - alfa*u; partial sums of u^2
__global__ __launch_bounds__(256) void k_ls_u(const double* __restrict__ t, double* __restrict__ u,
                                              int64_t n, const LsqrState* st, double* partial) {
  __shared__ double red[4];
  if (st->done) return;
  const double a = st->alfa;
  double sq = 0.0;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const double ui = t[i] - a * u[i];
    u[i] = ui;
    sq += ui * ui;
  }
  const double b = block_sum(sq, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = b;
}

// beta = ||u||; if beta > 0: anorm = sqrt(anorm^2 + alfa^2 + beta^2 + dampsq), 1/beta
__global__ __launch_bounds__(256) void k_ls_beta(const double* __restrict__ partial, LsqrState* st) {
  __shared__ double red[4];
  if (st->done) return;
  const double s = partial_total(partial, red);
  if (threadIdx.x == 0) {
    const double beta = sqrt(s);
    st->beta = beta;
    if (beta > 0.0) {
      const double a = st->anorm, al = st->alfa;
      st->anorm = sqrt(a * a + al * al + beta * beta + 0.0);
      st->binv = 1.0 / beta;
    }
  }
}

// u = (1/beta)*u (beta > 0)
__global__ __launch_bounds__(256) void k_ls_scale_u(double* __restrict__ u, int64_t n,
                                                    const LsqrState* st) {
  if (st->done || !(st->beta > 0.0)) return;
  const double bi = st->binv;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    u[i] = bi * u[i];
}

// v = t - beta*v (beta > 0); partial sums of v^2
__global__ __launch_bounds__(256) void k_ls_v(const double* __restrict__ t, double* __restrict__ v,
                                              int64_t n, const LsqrState* st, double* partial) {
  __shared__ double red[4];
  if (st->done || !(st->beta > 0.0)) return;
  const double b = st->beta;
  double sq = 0.0;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const double vi = t[i] - b * v[i];
    v[i] = vi;
    sq += vi * vi;
  }
  const double s = block_sum(sq, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

__device__ __forceinline__ double sgn(double a) { return a > 0.0 ? 1.0 : (a < 0.0 ? -1.0 : 0.0); }

// scipy _sym_ortho: stable Givens rotation (c, s, r) with [c s; -s c] [a; b] = [r; 0]
__device__ void sym_ortho(double a, double b, double& c, double& s, double& r) {
  if (b == 0.0) {
    c = sgn(a);
    s = 0.0;
    r = fabs(a);
  } else if (a == 0.0) {
    c = 0.0;
    s = sgn(b);
    r = fabs(b);
  } else if (fabs(b) > fabs(a)) {
    const double tau = a / b;
    s = sgn(b) / sqrt(1.0 + tau * tau);
    c = s * tau;
    r = b / s;
  } else {
    const double tau = b / a;
    c = sgn(a) / sqrt(1.0 + tau * tau);
    s = c * tau;
    r = a / c;
  }
}

// alfa = ||v|| (beta > 0), then the rotation and the x-norm estimate recurrences
__global__ __launch_bounds__(256) void k_ls_step(const double* __restrict__ partial, LsqrState* st) {
  __shared__ double red[4];
  if (st->done) return;
  const bool bpos = st->beta > 0.0;
  const double s = bpos ? partial_total(partial, red) : 0.0;
  if (threadIdx.x != 0) return;
  st->itn += 1;
  double alfa = st->alfa;
  if (bpos) {
    alfa = sqrt(s);
    st->alfa = alfa;
    st->ainv = alfa > 0.0 ? 1.0 / alfa : 1.0;
  }
  const double beta = st->beta;
  const double rhobar1 = st->rhobar;  // damp = 0: psi = 0
  double cs, sn, rho;
  sym_ortho(rhobar1, beta, cs, sn, rho);
  const double theta = sn * alfa;
  st->rhobar = -cs * alfa;
  const double phi = cs * st->phibar;
  const double phibar = sn * st->phibar;
  st->phibar = phibar;
  const double tau = sn * phi;
  st->t1 = phi / rho;
  st->t2 = -theta / rho;
  st->rinv = 1.0 / rho;
  const double delta = st->sn2 * rho;
  const double gambar = -st->cs2 * rho;
  const double rhs = phi - delta * st->z;
  const double zbar = rhs / gambar;
  st->xnorm = sqrt(st->xxnorm + zbar * zbar);
  const double gamma = sqrt(gambar * gambar + theta * theta);
  st->cs2 = gambar / gamma;
  st->sn2 = theta / gamma;
  st->z = rhs / gamma;
  st->xxnorm = st->xxnorm + st->z * st->z;
  const double res1 = phibar * phibar;
  st->res2 = st->res2 + 0.0;
  st->rnorm = sqrt(res1 + st->res2);
  st->arnorm = alfa * fabs(tau);
}

// v = (1/alfa)*v (beta, alfa > 0); dk = (1/rho)*w; x = x + t1*w; w = v + t2*w; sum dk^2
__global__ __launch_bounds__(256) void k_ls_update(double* __restrict__ v, double* __restrict__ w,
                                                   double* __restrict__ x, int64_t n,
                                                   const LsqrState* st, double* partial) {
  __shared__ double red[4];
  if (st->done) return;
  const bool sv = st->beta > 0.0 && st->alfa > 0.0;
  const double ai = st->ainv, ri = st->rinv, t1 = st->t1, t2 = st->t2;
  double sq = 0.0;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    double vi = v[i];
    if (sv) {
      vi = ai * vi;
      v[i] = vi;
    }
    const double wi = w[i];
    const double dk = ri * wi;
    sq += dk * dk;
    x[i] = x[i] + t1 * wi;
    w[i] = vi + t2 * wi;
  }
  const double s = block_sum(sq, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

// ddnorm += ||dk||^2, then scipy's stopping tests (later tests override earlier ones)
__global__ __launch_bounds__(256) void k_ls_test(const double* __restrict__ partial, LsqrState* st) {
  __shared__ double red[4];
  if (st->done) return;
  const double s = partial_total(partial, red);
  if (threadIdx.x != 0) return;
  const double eps = std::numeric_limits<double>::epsilon();
  const double dkn = sqrt(s);
  st->ddnorm = st->ddnorm + dkn * dkn;
  const double anorm = st->anorm, rnorm = st->rnorm, bnorm = st->bnorm, xnorm = st->xnorm;
  const double acond = anorm * sqrt(st->ddnorm);
  const double test1 = rnorm / bnorm;
  const double test2 = st->arnorm / (anorm * rnorm + eps);
  const double test3 = 1.0 / (acond + eps);
  const double t1 = test1 / (1.0 + anorm * xnorm / bnorm);
  const double rtol = st->btol + st->atol * anorm * xnorm / bnorm;
  int istop = 0;
  if (st->itn >= st->iter_lim) istop = 7;
  if (1.0 + test3 <= 1.0) istop = 6;
  if (1.0 + test2 <= 1.0) istop = 5;
  if (1.0 + t1 <= 1.0) istop = 4;
  if (test3 <= st->ctol) istop = 3;
  if (test2 <= st->atol) istop = 2;
  if (test1 <= rtol) istop = 1;
  st->istop = istop;
  if (istop != 0) st->done = 1;
}

// sum of squares of a vector into partial[0..kLsqrBlocks)
__global__ __launch_bounds__(256) void k_ls_sq(const double* __restrict__ a, int64_t n,
                                               double* partial) {
  __shared__ double red[4];
  double sq = 0.0;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    sq += a[i] * a[i];
  const double s = block_sum(sq, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_ls_total(const double* __restrict__ partial, double* out) {
  __shared__ double red[4];
  const double s = partial_total(partial, red);
  if (threadIdx.x == 0) *out = s;
}

// x -= sum(x) / n with the sum from k_ls_sum / k_ls_total (fixed order)
__global__ __launch_bounds__(256) void k_ls_sum(const double* __restrict__ a, int64_t n,
                                                double* partial) {
  __shared__ double red[4];
  double acc = 0.0;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    acc += a[i];
  const double s = block_sum(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

__global__ void k_ls_sub_mean(double* __restrict__ a, int64_t n, const double* __restrict__ sum) {
  const double mean = *sum / (double)n;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    a[i] = a[i] - mean;
}

__global__ void k_ls_scale(double* __restrict__ a, int64_t n, double f) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    a[i] = f * a[i];
}
}  // namespace

}  // namespace mlamg

using namespace mlamg;

extern "C" {

int mlamg_lsqr(const mlamg_csr* A, const mlamg_csr* AT, const double* b, double* x, double atol,
               double btol, double conlim, int iter_lim, int* istop_out, int* itn_out,
               void* stream) {
  MLAMG_REQUIRE(A && AT && b && x, "NULL argument");
  MLAMG_REQUIRE(AT->n_rows == A->n_cols && AT->n_cols == A->n_rows, "AT must be A's transpose");
  hipStream_t s = S(stream);
  const int64_t m = A->n_rows, n = A->n_cols;
  if (iter_lim <= 0) iter_lim = (int)std::min<int64_t>(2 * n, (int64_t)1 << 30);
  const int nb = kLsqrBlocks;
  const unsigned gm = (unsigned)nb;
  double *u = nullptr, *v = nullptr, *w = nullptr, *t = nullptr, *partial = nullptr;
  LsqrState* st = nullptr;
  const size_t big = (size_t)std::max<int64_t>(std::max(m, n), 1);
  auto cleanup = [&]() {
    for (void* p : {(void*)u, (void*)v, (void*)w, (void*)t, (void*)partial, (void*)st})
      if (p) (void)hipFree(p);
  };
  if (hipMalloc(&u, sizeof(double) * big) != hipSuccess ||
      hipMalloc(&v, sizeof(double) * big) != hipSuccess ||
      hipMalloc(&w, sizeof(double) * big) != hipSuccess ||
      hipMalloc(&t, sizeof(double) * big) != hipSuccess ||
      hipMalloc(&partial, sizeof(double) * (nb + 1)) != hipSuccess ||
      hipMalloc(&st, sizeof(LsqrState)) != hipSuccess) {
    cleanup();
    set_error("lsqr: out of device memory");
    return MLAMG_ENOMEM;
  }
  int rc = MLAMG_OK;
  auto hip = [&](hipError_t e, const char* what) {
    if (rc == MLAMG_OK && e != hipSuccess) {
      set_error(std::string("lsqr: ") + what + ": " + hipGetErrorString(e));
      rc = MLAMG_EHIP;
    }
  };
  auto norm_sq = [&](const double* a, int64_t len) {
    double r = 0.0;
    hipLaunchKernelGGL(k_ls_sq, dim3(gm), dim3(256), 0, s, a, len, partial);
    hipLaunchKernelGGL(k_ls_total, dim3(1), dim3(256), 0, s, partial, partial + nb);
    hip(hipGetLastError(), "launch");
    hip(hipMemcpyAsync(&r, partial + nb, sizeof(double), hipMemcpyDeviceToHost, s), "copy");
    hip(hipStreamSynchronize(s), "sync");
    return r;
  };
  // x = 0, u = b, beta = bnorm = ||b||
  hip(hipMemsetAsync(x, 0, sizeof(double) * std::max<int64_t>(n, 1), s), "memset");
  hip(hipMemcpyAsync(u, b, sizeof(double) * m, hipMemcpyDeviceToDevice, s), "copy");
  const double bnorm = sqrt(norm_sq(u, m));
  const double beta = bnorm;
  double alfa = 0.0;
  if (rc == MLAMG_OK && beta > 0.0) {
    hipLaunchKernelGGL(k_ls_scale, dim3(gm), dim3(256), 0, s, u, m, 1.0 / beta);
    hip(hipGetLastError(), "launch");
    if (rc == MLAMG_OK) rc = launch_spmv_plain(AT, u, v, s);  // v = A^T u
    if (rc == MLAMG_OK) alfa = sqrt(norm_sq(v, n));
  } else if (rc == MLAMG_OK) {
    hip(hipMemsetAsync(v, 0, sizeof(double) * std::max<int64_t>(n, 1), s), "memset");
  }
  if (rc == MLAMG_OK && alfa > 0.0) {
    hipLaunchKernelGGL(k_ls_scale, dim3(gm), dim3(256), 0, s, v, n, 1.0 / alfa);
    hip(hipGetLastError(), "launch");
  }
  hip(hipMemcpyAsync(w, v, sizeof(double) * std::max<int64_t>(n, 1), hipMemcpyDeviceToDevice, s),
      "copy");
  LsqrState h{};
  h.alfa = alfa;
  h.beta = beta;
  h.anorm = 0.0;
  h.ddnorm = 0.0;
  h.xnorm = 0.0;
  h.xxnorm = 0.0;
  h.z = 0.0;
  h.cs2 = -1.0;
  h.sn2 = 0.0;
  h.rhobar = alfa;
  h.phibar = beta;
  h.bnorm = bnorm;
  h.res2 = 0.0;
  h.atol = atol;
  h.btol = btol;
  h.ctol = conlim > 0.0 ? 1.0 / conlim : 0.0;
  h.iter_lim = iter_lim;
  h.done = (alfa * beta == 0.0) ? 1 : 0;  // arnorm == 0: x = 0 is the answer (istop 0)
  hip(hipMemcpyAsync(st, &h, sizeof(h), hipMemcpyHostToDevice, s), "copy");
  const int32_t* done = &st->done;
  while (rc == MLAMG_OK) {
    hip(hipStreamSynchronize(s), "sync");
    hip(hipMemcpy(&h, st, sizeof(h), hipMemcpyDeviceToHost), "copy");
    if (rc != MLAMG_OK || h.done || h.itn >= iter_lim) break;
    for (int c = 0; c < kLsqrChunk && rc == MLAMG_OK; ++c) {
      rc = spmv_set(A, v, t, done, s);  // t = A v
      if (rc != MLAMG_OK) break;
      hipLaunchKernelGGL(k_ls_u, dim3(gm), dim3(256), 0, s, t, u, m, st, partial);
      hipLaunchKernelGGL(k_ls_beta, dim3(1), dim3(256), 0, s, partial, st);
      hipLaunchKernelGGL(k_ls_scale_u, dim3(gm), dim3(256), 0, s, u, m, st);
      hip(hipGetLastError(), "launch");
      if (rc == MLAMG_OK) rc = spmv_set(AT, u, t, done, s);  // t = A^T u
      if (rc != MLAMG_OK) break;
      hipLaunchKernelGGL(k_ls_v, dim3(gm), dim3(256), 0, s, t, v, n, st, partial);
      hipLaunchKernelGGL(k_ls_step, dim3(1), dim3(256), 0, s, partial, st);
      hipLaunchKernelGGL(k_ls_update, dim3(gm), dim3(256), 0, s, v, w, x, n, st, partial);
      hipLaunchKernelGGL(k_ls_test, dim3(1), dim3(256), 0, s, partial, st);
      hip(hipGetLastError(), "launch");
    }
  }
  if (rc == MLAMG_OK) {
    if (istop_out) *istop_out = h.istop;
    if (itn_out) *itn_out = h.itn;
  }
  hip(hipStreamSynchronize(s), "sync");
  cleanup();
  return rc;
}

int mlamg_remove_mean(double* x, int64_t n, void* stream) {
  MLAMG_REQUIRE(n >= 0 && (n == 0 || x), "NULL argument");
  if (n == 0) return MLAMG_OK;
  hipStream_t s = S(stream);
  double* partial = static_cast<double*>(scratch(sizeof(double) * (kLsqrBlocks + 1), 1));
  MLAMG_REQUIRE(partial, "scratch allocation failed");
  hipLaunchKernelGGL(k_ls_sum, dim3(kLsqrBlocks), dim3(256), 0, s, x, n, partial);
  hipLaunchKernelGGL(k_ls_total, dim3(1), dim3(256), 0, s, partial, partial + kLsqrBlocks);
  hipLaunchKernelGGL(k_ls_sub_mean, dim3(kLsqrBlocks), dim3(256), 0, s, x, n,
                     partial + kLsqrBlocks);
  MLAMG_HIP(hipGetLastError());
  return MLAMG_OK;
}

}  // extern "C"
