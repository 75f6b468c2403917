// Preconditioned GMRES around the V-cycle: the Krylov acceleration of the reference's PyAMG
// preconditioner, `Amg.solve(X.array_r, tol=amg_rtol, accel='gmres')` (ns/preconditioner/
// PyAMG.py:119, the default `amg_precondition_with_gmres` of :54): zero initial guess, a
// residual tolerance relative to ||b||, one V-cycle of the hierarchy as preconditioner.
//
// The algorithm is scipy.sparse.linalg.gmres (scipy 1.15, the library in this image): restarted,
// LEFT-preconditioned (w = M A v), modified Gram-Schmidt, Givens rotations on the Hessenberg
// column, inner stop on the preconditioned residual estimate with the gh-8400 tolerance control
// (ptol adapted between restarts), outer stop ||b - A x||_2 <= atol = rtol ||b||_2. pyamg's own
// krylov.gmres, which the reference calls, is absent here (parity unpinned); scipy's is the
// pinned restatement of the same method.
//
// Everything n-sized runs on the device: the SpMV (the operator's exact-order format), the
// preconditioner (hier_coarse_cycle: one V-cycle from a zero guess, replayed from a captured
// graph), and the Gram-Schmidt dots / updates (fixed-order reductions finished by the
// last-arriving workgroup, so a solve is deterministic). The (restart+1)-sized Hessenberg work —
// rotations and the inner stop test — runs on the device in one thread (k_gm_arnoldi, the same
// operations as scipy's numpy code), so an inner iteration costs one status read; the
// triangular solve and the restart logic stay on the host, once per restart cycle.
#include "common.hpp"

#include <cmath>

namespace mlamg {

constexpr int kGmThreads = 256;
constexpr int kGmMaxBlocks = 1024;

__device__ __forceinline__ double gm_wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// out[0] = a . b, fixed order: per-workgroup partials, summed in order by the last-arriving
// workgroup (agent-scope acquire/release on the arrival counter)
__global__ __launch_bounds__(kGmThreads) void k_gm_dot(const double* __restrict__ a,
                                                      const double* __restrict__ b, int64_t n,
                                                      double* __restrict__ partial, int32_t* ctr,
                                                      double* out, const int32_t* done) {
  __shared__ double red[kGmThreads / 64];
  __shared__ int last;
  if (done && *done) return;  // uniform: no workgroup arrives, the counter stays 0
  double s = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)kGmThreads + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kGmThreads)
    s += a[i] * b[i];
  s = gm_wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    partial[blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
    __threadfence();
    const int prev = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    last = prev == (int)gridDim.x - 1;
    if (last) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  double t = strided_sum(partial, gridDim.x, threadIdx.x, kGmThreads);
  t = gm_wave_sum(t);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x == 0) *out = ((red[0] + red[1]) + red[2]) + red[3];
}

// The inner loop's dots without the arrival counter: k_gm_part writes k_gm_dot's per-workgroup
// partials, and the consumer sums them with gm_total — k_gm_dot's last-workgroup sum, the same
// order — so no workgroup needs the agent-scope fence before arriving (on MI355X that fence
// writes back the XCD's L2, once per workgroup).
__global__ __launch_bounds__(kGmThreads) void k_gm_part(const double* __restrict__ a,
                                                       const double* __restrict__ b, int64_t n,
                                                       double* __restrict__ partial,
                                                       const int32_t* done) {
  __shared__ double red[kGmThreads / 64];
  if (done && *done) return;
  double s = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)kGmThreads + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kGmThreads)
    s += a[i] * b[i];
  s = gm_wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
}

// sum of np partials by a whole workgroup of kGmThreads, k_gm_dot's order; every thread gets it
__device__ double gm_total(const double* __restrict__ partial, int np, double* red) {
  double t = strided_sum(partial, np, threadIdx.x, kGmThreads);
  t = gm_wave_sum(t);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = t;
  __syncthreads();
  return ((red[0] + red[1]) + red[2]) + red[3];
}

// w -= c v with c = the dot k_gm_part left in partial (every workgroup sums it; workgroup 0
// also stores it, the Hessenberg entry)
__global__ __launch_bounds__(kGmThreads) void k_gm_axmy_p(double* __restrict__ w,
                                                         const double* __restrict__ v, int64_t n,
                                                         const double* __restrict__ partial,
                                                         int np, double* coef,
                                                         const int32_t* done) {
  __shared__ double red[kGmThreads / 64];
  if (done && *done) return;
  const double c = gm_total(partial, np, red);
  if (blockIdx.x == 0 && threadIdx.x == 0) *coef = c;
  for (int64_t i = blockIdx.x * (int64_t)kGmThreads + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kGmThreads)
    w[i] = w[i] - c * v[i];
}

// w -= (*coef) * v   (numpy's `w -= tmp * v[k, :]`: one product, one subtraction per entry)
__global__ __launch_bounds__(kGmThreads) void k_gm_axmy(double* __restrict__ w,
                                                       const double* __restrict__ v, int64_t n,
                                                       const double* coef, const int32_t* done) {
  if (done && *done) return;
  const double c = *coef;
  for (int64_t i = blockIdx.x * (int64_t)kGmThreads + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kGmThreads)
    w[i] = w[i] - c * v[i];
}

// y = x * (1 / d)  with d = sqrt(*dd) (numpy: v *= (1 / norm))
__global__ __launch_bounds__(kGmThreads) void k_gm_scale(double* __restrict__ y,
                                                        const double* __restrict__ x, int64_t n,
                                                        double d) {
  const double inv = 1.0 / d;
  for (int64_t i = blockIdx.x * (int64_t)kGmThreads + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kGmThreads)
    y[i] = x[i] * inv;
}

// y = x * (1 / d) with d read on the device (the Arnoldi step's h1), skipped once done
__global__ __launch_bounds__(kGmThreads) void k_gm_scale_dev(double* __restrict__ y,
                                                            const double* __restrict__ x,
                                                            int64_t n, const double* d,
                                                            const int32_t* done) {
  if (*done) return;
  const double inv = 1.0 / *d;
  for (int64_t i = blockIdx.x * (int64_t)kGmThreads + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kGmThreads)
    y[i] = x[i] * inv;
}

// x += sum_k y[k] v_k (k ascending: numpy's `x += y @ v[:m, :]`)
__global__ __launch_bounds__(kGmThreads) void k_gm_update(double* __restrict__ x,
                                                         const double* __restrict__ V,
                                                         int64_t n, int64_t ld,
                                                         const double* __restrict__ y, int m) {
  for (int64_t i = blockIdx.x * (int64_t)kGmThreads + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kGmThreads) {
    double t = 0.0;
    for (int k = 0; k < m; ++k) t += y[k] * V[k * ld + i];
    x[i] = x[i] + t;
  }
}

static int gm_grid(int64_t n) {
  return (int)std::min<int64_t>(kGmMaxBlocks, std::max<int64_t>(1, (n + kGmThreads - 1) /
                                                                       kGmThreads));
}

// LAPACK dlartg (3.10+, the safe-scaling version scipy's get_lapack_funcs('lartg') binds):
// c f + s g = r, -s f + c g = 0
__host__ __device__ static void lartg(double f, double g, double* c, double* s, double* r) {
  if (g == 0.0) {
    *c = 1.0;
    *s = 0.0;
    *r = f;
  } else if (f == 0.0) {
    *c = 0.0;
    *s = g > 0 ? 1.0 : -1.0;
    *r = fabs(g);
  } else {
    const double d = sqrt(f * f + g * g);
    *c = fabs(f) / d;
    *r = f > 0 ? d : -d;
    *s = g / *r;
  }
}

// One Arnoldi step's small-matrix work on the device, by one thread — what the host did with
// the read-back column, the same operations in the same order (so the same bits): Hessenberg
// column from the MGS coefficients and norms, exact-solution test, the past rotations, a new
// rotation (lartg), the rotated right-hand side and the preconditioned residual estimate; then
// the inner stop (presid <= ptol or breakdown) raises `done`, which the next iteration's kernels
// and V-cycle (the hierarchy's own flag) read, so the host needs one status read per iteration.
// st: [0] presid, [1] h1 (the scale of v_{col+1}), [2] breakdown, [3] last column, [4] steps,
// [5] ||w||^2 before the projections (h0^2).
__global__ __launch_bounds__(kGmThreads) void k_gm_arnoldi(
    int col, int ldh, const double* __restrict__ scal, const double* __restrict__ p_h0,
    const double* __restrict__ p_h1, int np, double* __restrict__ Hd, double* __restrict__ giv,
    double* __restrict__ S, double* __restrict__ st, double eps, double ptol, double bnrm2,
    double* __restrict__ hist, int hist_cap, int32_t* done) {
  __shared__ double red[kGmThreads / 64];
  if (*done) return;
  // ||w||^2 before and after the projections, from k_gm_part's partials (k_gm_dot's sums)
  const double w0 = gm_total(p_h0, np, red);
  __syncthreads();
  const double w1 = gm_total(p_h1, np, red);
  if (threadIdx.x != 0) return;
  st[5] = w0;
  auto H = [&](int c, int k) -> double& { return Hd[(size_t)c * ldh + k]; };
  const double h0 = sqrt(w0);
  for (int k = 0; k <= col; ++k) H(col, k) = scal[k];
  const double h1 = sqrt(w1);
  H(col, col + 1) = h1;
  bool breakdown = false;
  if (h1 <= eps * h0) {  // exact solution indicator
    H(col, col + 1) = 0.0;
    breakdown = true;
  }
  st[1] = h1;
  for (int k = 0; k < col; ++k) {  // past rotations
    const double c = giv[2 * k], sn = giv[2 * k + 1];
    const double n0 = H(col, k), n1 = H(col, k + 1);
    H(col, k) = c * n0 + sn * n1;
    H(col, k + 1) = -sn * n0 + c * n1;
  }
  double c, sn, mag;
  lartg(H(col, col), H(col, col + 1), &c, &sn, &mag);
  giv[2 * col] = c;
  giv[2 * col + 1] = sn;
  H(col, col) = mag;
  H(col, col + 1) = 0.0;
  const double t2 = -sn * S[col];
  S[col] = c * S[col];
  S[col + 1] = t2;
  const double presid = fabs(t2);
  const int steps = (int)st[4];
  if (hist && steps < hist_cap) hist[steps] = presid / bnrm2;
  st[0] = presid;
  st[2] = breakdown ? 1.0 : 0.0;
  st[3] = (double)col;
  st[4] = (double)(steps + 1);
  if (presid <= ptol || breakdown) *done = 1;
}

struct GmWork {
  double* V = nullptr;    // (restart + 1) x ld
  double* w = nullptr;
  double* r = nullptr;
  double* pb = nullptr;   // staging right-hand side of the preconditioner (fixed address)
  double* partial = nullptr;
  double* p_h0 = nullptr;  // k_gm_part partials of ||w||^2 before / after the projections
  double* p_h1 = nullptr;
  double* scal = nullptr;  // dot results: [0..restart+1) MGS coefficients, [restart+1] norm^2
  double* y = nullptr;     // solution of the small triangular system
  int32_t* ctr = nullptr;
  double* Hd = nullptr;    // restart x (restart + 1) Hessenberg columns (device copy)
  double* giv = nullptr;   // 2 restart Givens coefficients
  double* S = nullptr;     // restart + 1 rotated right-hand side
  double* st = nullptr;    // Arnoldi status (k_gm_arnoldi)
  double* hist = nullptr;  // presid / ||b|| per inner step
  void* mem = nullptr;
  int64_t ld = 0;
};

int gmres_impl(const mlamg_csr* A, mlamg_hier* M, const double* b, double* x, double rtol,
               int restart, int maxiter, bool x_zero, int* info_out, int* iters_out,
               double* presid_hist, int hist_cap, hipStream_t s, double* rel_out) {
  const int64_t n = A->n_rows;
  if (rel_out) *rel_out = 0.0;
  if (restart <= 0) restart = 20;
  restart = (int)std::min<int64_t>(restart, std::max<int64_t>(n, 1));
  if (maxiter <= 0) maxiter = (int)std::min<int64_t>(INT32_MAX, 10 * std::max<int64_t>(n, 1));
  GmWork W;
  W.ld = ((std::max<int64_t>(n, 1) + 31) / 32) * 32;
  const size_t vec = sizeof(double) * W.ld;
  const size_t small = sizeof(double) * ((size_t)restart * (restart + 1) + 2 * restart +
                                         (restart + 1) + 8 + std::max(hist_cap, 1));
  const size_t total = vec * (restart + 1) + 3 * vec + 3 * sizeof(double) * kGmMaxBlocks +
                       sizeof(double) * (2 * restart + 6) + 256 + small;
  // the preconditioner hierarchy keeps the workspace across calls (a restart-100
  // solve on a 10M-row grid would map and unmap 8 GB per call)
  MLAMG_TRY(hier_workspace(M, total, &W.mem));
  char* p = static_cast<char*>(W.mem);
  W.V = reinterpret_cast<double*>(p);
  p += vec * (restart + 1);
  W.w = reinterpret_cast<double*>(p);
  p += vec;
  W.r = reinterpret_cast<double*>(p);
  p += vec;
  W.pb = reinterpret_cast<double*>(p);
  p += vec;
  W.partial = reinterpret_cast<double*>(p);
  p += sizeof(double) * kGmMaxBlocks;
  W.p_h0 = reinterpret_cast<double*>(p);
  p += sizeof(double) * kGmMaxBlocks;
  W.p_h1 = reinterpret_cast<double*>(p);
  p += sizeof(double) * kGmMaxBlocks;
  W.scal = reinterpret_cast<double*>(p);
  W.y = W.scal + restart + 2;
  W.ctr = reinterpret_cast<int32_t*>(W.y + restart + 2);
  W.Hd = reinterpret_cast<double*>(reinterpret_cast<char*>(W.ctr) + 64);
  W.giv = W.Hd + (size_t)restart * (restart + 1);
  W.S = W.giv + 2 * restart;
  W.st = W.S + restart + 1;
  W.hist = W.st + 8;
  MLAMG_HIP(hipMemsetAsync(W.ctr, 0, 64, s));
  MLAMG_TRY(hier_prepare_ext(M));  // allocates the hierarchy's flags and work buffers
  MLAMG_HIP(hipMemsetAsync(hier_done_flag(M), 0, sizeof(int32_t), s));
  const int nb = gm_grid(n);
  const int norm_slot = restart + 1;

  auto dot = [&](const double* a, const double* c, int slot) -> int {
    hipLaunchKernelGGL(k_gm_dot, dim3(nb), dim3(kGmThreads), 0, s, a, c, n, W.partial, W.ctr,
                       W.scal + slot, nullptr);
    MLAMG_HIP(hipGetLastError());
    return MLAMG_OK;
  };
  auto read = [&](int slot, int count, double* dst) -> int {
    MLAMG_HIP(hipMemcpyAsync(dst, W.scal + slot, sizeof(double) * count, hipMemcpyDeviceToHost,
                             s));
    MLAMG_HIP(hipStreamSynchronize(s));
    return MLAMG_OK;
  };
  auto norm = [&](const double* a, double* out) -> int {  // np.linalg.norm: sqrt(a . a)
    MLAMG_TRY(dot(a, a, norm_slot));
    double t = 0.0;
    MLAMG_TRY(read(norm_slot, 1, &t));
    *out = std::sqrt(t);
    return MLAMG_OK;
  };
  auto psolve = [&](const double* in, double* out) -> int {  // one V-cycle from x = 0
    MLAMG_HIP(hipMemcpyAsync(W.pb, in, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
    double* z = nullptr;
    MLAMG_TRY(hier_coarse_cycle(M, W.pb, &z, 1, s));
    MLAMG_HIP(hipMemcpyAsync(out, z, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
    return MLAMG_OK;
  };
  auto resid = [&](const double* xv, double* rv) -> int {  // r = b - A x
    return residual_impl(A, b, xv, rv, nullptr, nullptr, nullptr, nullptr, kNoTol, nullptr,
                         nullptr, nullptr, s);
  };

  int iters = 0;
  *info_out = 0;
  double bnrm2 = 0.0;
  MLAMG_TRY(norm(b, &bnrm2));
  const double atol = rtol * bnrm2;  // _get_atol_rtol: max(atol = 0, rtol * ||b||)
  if (bnrm2 == 0.0) {  // scipy returns postprocess(b)
    MLAMG_HIP(hipMemcpyAsync(x, b, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
    *iters_out = 0;
    return MLAMG_OK;
  }
  const double eps = 2.220446049250313e-16;
  MLAMG_TRY(psolve(b, W.w));
  double Mb_nrm2 = 0.0;
  MLAMG_TRY(norm(W.w, &Mb_nrm2));
  double ptol_max_factor = 1.0;
  double ptol = Mb_nrm2 * std::min(ptol_max_factor, atol / bnrm2);
  double presid = 0.0, rnorm = 0.0;
  std::vector<double> h((size_t)restart * (restart + 1), 0.0), S(restart + 1, 0.0),
      y(restart + 1, 0.0);
  auto H = [&](int c, int k) -> double& { return h[(size_t)c * (restart + 1) + k]; };
  double* V0 = W.V;
  auto Vk = [&](int k) { return W.V + (int64_t)k * W.ld; };
  for (int iteration = 0; iteration < maxiter; ++iteration) {
    if (iteration == 0) {
      if (x_zero) {
        MLAMG_HIP(hipMemcpyAsync(W.r, b, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
      } else {
        MLAMG_TRY(resid(x, W.r));
      }
      double r0 = 0.0;
      MLAMG_TRY(norm(W.r, &r0));
      if (r0 < atol) {
        rnorm = r0;
        break;
      }
    }
    MLAMG_TRY(psolve(W.r, V0));
    double tmp = 0.0;
    MLAMG_TRY(norm(V0, &tmp));
    hipLaunchKernelGGL(k_gm_scale, dim3(nb), dim3(kGmThreads), 0, s, V0, V0, n, tmp);
    MLAMG_HIP(hipGetLastError());
    std::fill(S.begin(), S.end(), 0.0);
    S[0] = tmp;
    // the cycle's small state on the device: rotated right-hand side, step count; the inner
    // stop is the hierarchy's done flag (k_gm_arnoldi raises it; the V-cycle and the Krylov
    // kernels of later steps then do nothing), one status read per step
    int32_t* done = hier_done_flag(M);
    double st_h[8] = {0.0, 0.0, 0.0, 0.0, (double)iters, 0.0, 0.0, 0.0};
    MLAMG_HIP(hipMemcpyAsync(W.S, S.data(), sizeof(double) * (restart + 1),
                             hipMemcpyHostToDevice, s));
    MLAMG_HIP(hipMemcpyAsync(W.st, st_h, sizeof(st_h), hipMemcpyHostToDevice, s));
    bool breakdown = false;
    int col = 0;
    for (col = 0; col < restart; ++col) {
      MLAMG_TRY(spmv_set(A, Vk(col), W.r, done, s));  // av (W.r is free until the update)
      MLAMG_TRY(psolve(W.r, W.w));                    // w = M av
      hipLaunchKernelGGL(k_gm_part, dim3(nb), dim3(kGmThreads), 0, s, W.w, W.w, n, W.p_h0,
                         done);  // h0^2
      for (int k = 0; k <= col; ++k) {  // modified Gram-Schmidt, coefficient on the device
        hipLaunchKernelGGL(k_gm_part, dim3(nb), dim3(kGmThreads), 0, s, Vk(k), W.w, n,
                           W.partial, done);
        hipLaunchKernelGGL(k_gm_axmy_p, dim3(nb), dim3(kGmThreads), 0, s, W.w, Vk(k), n,
                           W.partial, nb, W.scal + k, done);
        MLAMG_HIP(hipGetLastError());
      }
      hipLaunchKernelGGL(k_gm_part, dim3(nb), dim3(kGmThreads), 0, s, W.w, W.w, n, W.p_h1, done);
      hipLaunchKernelGGL(k_gm_arnoldi, dim3(1), dim3(kGmThreads), 0, s, col, restart + 1,
                         W.scal, W.p_h0, W.p_h1, nb, W.Hd, W.giv, W.S, W.st, eps, ptol, bnrm2,
                         presid_hist ? W.hist : nullptr, hist_cap, done);
      MLAMG_HIP(hipGetLastError());
      hipLaunchKernelGGL(k_gm_scale_dev, dim3(nb), dim3(kGmThreads), 0, s, Vk(col + 1), W.w, n,
                         W.st + 1, done);
      MLAMG_HIP(hipGetLastError());
      int32_t dn = 0;
      MLAMG_HIP(hipMemcpyAsync(&dn, done, sizeof(int32_t), hipMemcpyDeviceToHost, s));
      MLAMG_HIP(hipStreamSynchronize(s));
      if (dn) break;
    }
    MLAMG_HIP(hipMemcpyAsync(st_h, W.st, sizeof(st_h), hipMemcpyDeviceToHost, s));
    MLAMG_HIP(hipMemcpyAsync(h.data(), W.Hd, sizeof(double) * h.size(), hipMemcpyDeviceToHost,
                             s));
    MLAMG_HIP(hipMemcpyAsync(S.data(), W.S, sizeof(double) * (restart + 1),
                             hipMemcpyDeviceToHost, s));
    MLAMG_HIP(hipMemsetAsync(done, 0, sizeof(int32_t), s));  // the update's V-cycles run again
    MLAMG_HIP(hipStreamSynchronize(s));
    presid = st_h[0];
    breakdown = st_h[2] != 0.0;
    iters = (int)st_h[4];
    if (col == restart) col = restart - 1;
    if (H(col, col) == 0.0) S[col] = 0.0;
    for (int k = 0; k <= col; ++k) y[k] = S[k];
    for (int k = col; k > 0; --k) {
      if (y[k] != 0.0) {
        y[k] /= H(k, k);
        const double t = y[k];
        for (int j = 0; j < k; ++j) y[j] -= t * H(k, j);
      }
    }
    if (y[0] != 0.0) y[0] /= H(0, 0);
    MLAMG_HIP(hipMemcpyAsync(W.y, y.data(), sizeof(double) * (col + 1), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_gm_update, dim3(nb), dim3(kGmThreads), 0, s, x, W.V, n, W.ld, W.y,
                       col + 1);
    MLAMG_HIP(hipGetLastError());
    MLAMG_TRY(resid(x, W.r));
    MLAMG_TRY(norm(W.r, &rnorm));
    if (rnorm <= atol) break;
    if (breakdown) break;
    if (presid <= ptol)
      ptol_max_factor = std::max(eps, 0.25 * ptol_max_factor);
    else
      ptol_max_factor = std::min(1.0, 1.5 * ptol_max_factor);
    ptol = presid * std::min(ptol_max_factor, atol / rnorm);
  }
  *info_out = rnorm <= atol ? 0 : maxiter;
  *iters_out = iters;
  if (rel_out) *rel_out = rnorm / bnrm2;
  if (presid_hist && iters > 0)
    MLAMG_HIP(hipMemcpyAsync(presid_hist, W.hist, sizeof(double) * std::min(iters, hist_cap),
                             hipMemcpyDeviceToHost, s));
  MLAMG_HIP(hipStreamSynchronize(s));
  return MLAMG_OK;
}

// ---------------------------------------------------------------- Householder GMRES
// pyamg.krylov.gmres with its default orthog='householder' (pyamg 4.x _gmres_householder; the
// Krylov loop of `Amg.solve(b, accel='gmres')`, ns/preconditioner/PyAMG.py:119). pyamg is absent:
// restated from its published algorithm, parity unpinned (bitwise nothing: the device dots are
// fixed-order tree reductions where amg_core sums serially; oracle/restated.py
// pyamg_gmres_householder is the same algorithm in numpy). Left preconditioned: r0 = M(b - A x0);
// return at once if ||r0|| < tol ||b|| (||b|| = 0 counts as 1); else the inner stop is
// |g_{k+1}| < tol ||r0||, one outer cycle of at most min(maxiter, n) steps (restrt=None).
// Reflectors P_j = I - 2 w_j w_j^T, Krylov vector k = P_0 .. P_k e_k, new column
// P_k .. P_0 M A v, next reflector from its tail, Givens rotations on the head (host, O(k)).

// v = P_k e_k = e_k - 2 w_k[k] w_k
__global__ __launch_bounds__(kGmThreads) void k_hh_unit(double* __restrict__ v,
                                                       const double* __restrict__ w, int64_t n,
                                                       int64_t k) {
  const double c = -2.0 * w[k];
  for (int64_t i = blockIdx.x * (int64_t)kGmThreads + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kGmThreads)
    v[i] = c * w[i] + (i == k ? 1.0 : 0.0);
}

// v += (-2 (w . v)) w with the dot k_gm_part left in partial (amg_core apply_householders)
__global__ __launch_bounds__(kGmThreads) void k_hh_apply(double* __restrict__ v,
                                                        const double* __restrict__ w, int64_t n,
                                                        const double* __restrict__ partial,
                                                        int np) {
  __shared__ double red[kGmThreads / 64];
  const double a = -2.0 * gm_total(partial, np, red);
  for (int64_t i = blockIdx.x * (int64_t)kGmThreads + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kGmThreads)
    v[i] = v[i] + a * w[i];
}

// w = (0 .. 0, v[k1] + alpha, v[k1+1], ..) (the next reflector before its normalisation), and
// v[k1] = -alpha, v[k1+1:] = 0
__global__ __launch_bounds__(kGmThreads) void k_hh_next(double* __restrict__ w,
                                                       double* __restrict__ v, int64_t n,
                                                       int64_t k1, double alpha, int make_w) {
  for (int64_t i = blockIdx.x * (int64_t)kGmThreads + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kGmThreads) {
    const double vi = v[i];
    if (make_w) w[i] = i < k1 ? 0.0 : (i == k1 ? vi + alpha : vi);
    if (i == k1) v[i] = -alpha;
    else if (i > k1) v[i] = 0.0;
  }
}

// u[j] += y  (the Horner step's coefficient)
__global__ void k_hh_addat(double* u, int64_t j, double y) { u[j] = u[j] + y; }

// x = x + u
__global__ __launch_bounds__(kGmThreads) void k_hh_axpy1(double* __restrict__ x,
                                                        const double* __restrict__ u,
                                                        int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)kGmThreads + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kGmThreads)
    x[i] = x[i] + u[i];
}

static double hh_sign(double v) { return v == 0.0 ? 1.0 : (v > 0.0 ? 1.0 : -1.0); }

int gmres_householder_impl(const mlamg_csr* A, mlamg_hier* M, const double* b, double* x,
                           double tol, int maxiter, bool x_zero, int* info_out, int* iters_out,
                           double* resid_hist, int hist_cap, hipStream_t s) {
  const int64_t n = A->n_rows;
  if (maxiter <= 0) maxiter = (int)std::min<int64_t>(n, 40);
  const int max_inner = (int)std::min<int64_t>(maxiter, n);
  const int64_t ld = ((std::max<int64_t>(n, 1) + 31) / 32) * 32;
  const size_t vec = sizeof(double) * ld;
  const size_t total = vec * (max_inner + 1) + 4 * vec + sizeof(double) * kGmMaxBlocks + 256;
  void* mem = nullptr;
  MLAMG_TRY(hier_workspace(M, total, &mem));
  char* p = static_cast<char*>(mem);
  double* Wv = reinterpret_cast<double*>(p);  // reflectors w_0 .. w_max_inner
  p += vec * (max_inner + 1);
  double* v = reinterpret_cast<double*>(p);
  p += vec;
  double* r = reinterpret_cast<double*>(p);
  p += vec;
  double* pb = reinterpret_cast<double*>(p);
  p += vec;
  double* u = reinterpret_cast<double*>(p);
  p += vec;
  double* partial = reinterpret_cast<double*>(p);
  p += sizeof(double) * kGmMaxBlocks;
  double* scal = reinterpret_cast<double*>(p);  // 16 doubles
  int32_t* ctr = reinterpret_cast<int32_t*>(scal + 16);
  MLAMG_HIP(hipMemsetAsync(ctr, 0, 64, s));
  MLAMG_TRY(hier_prepare_ext(M));
  MLAMG_HIP(hipMemsetAsync(hier_done_flag(M), 0, sizeof(int32_t), s));
  const int nb = gm_grid(n);
  auto Wk = [&](int k) { return Wv + (int64_t)k * ld; };
  auto dotv = [&](const double* a, const double* c, int64_t len, double* out) -> int {
    hipLaunchKernelGGL(k_gm_dot, dim3(gm_grid(len)), dim3(kGmThreads), 0, s, a, c, len, partial,
                       ctr, scal, nullptr);
    MLAMG_HIP(hipGetLastError());
    MLAMG_HIP(hipMemcpyAsync(out, scal, sizeof(double), hipMemcpyDeviceToHost, s));
    MLAMG_HIP(hipStreamSynchronize(s));
    return MLAMG_OK;
  };
  auto nrm = [&](const double* a, int64_t len, double* out) -> int {
    double t = 0.0;
    MLAMG_TRY(dotv(a, a, len, &t));
    *out = std::sqrt(t);
    return MLAMG_OK;
  };
  auto at = [&](const double* a, int64_t i, double* out) -> int {
    MLAMG_HIP(hipMemcpyAsync(out, a + i, sizeof(double), hipMemcpyDeviceToHost, s));
    MLAMG_HIP(hipStreamSynchronize(s));
    return MLAMG_OK;
  };
  auto apply = [&](double* z, int j) -> int {  // z = P_j z
    hipLaunchKernelGGL(k_gm_part, dim3(nb), dim3(kGmThreads), 0, s, Wk(j), z, n, partial,
                       nullptr);
    hipLaunchKernelGGL(k_hh_apply, dim3(nb), dim3(kGmThreads), 0, s, z, Wk(j), n, partial, nb);
    MLAMG_HIP(hipGetLastError());
    return MLAMG_OK;
  };
  auto psolve = [&](const double* in, double* out) -> int {  // one V-cycle from x = 0
    MLAMG_HIP(hipMemcpyAsync(pb, in, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
    double* z = nullptr;
    MLAMG_TRY(hier_coarse_cycle(M, pb, &z, 1, s));
    MLAMG_HIP(hipMemcpyAsync(out, z, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
    return MLAMG_OK;
  };
  auto pres = [&](double* out_norm) -> int {  // r = M (b - A x), ||r||
    if (x_zero) {
      MLAMG_HIP(hipMemcpyAsync(v, b, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
    } else {
      MLAMG_TRY(residual_impl(A, b, x, v, nullptr, nullptr, nullptr, nullptr, kNoTol, nullptr,
                              nullptr, nullptr, s));
    }
    MLAMG_TRY(psolve(v, r));
    return nrm(r, n, out_norm);
  };
  *info_out = 0;
  *iters_out = 0;
  int nh = 0;
  double normr = 0.0, normb = 0.0;
  MLAMG_TRY(pres(&normr));
  x_zero = false;  // from here on x holds the iterate
  if (resid_hist && nh < hist_cap) resid_hist[nh++] = normr;
  MLAMG_TRY(nrm(b, n, &normb));
  if (normb == 0.0) normb = 1.0;
  if (normr < tol * normb) return MLAMG_OK;
  if (normr != 0.0) tol = tol * normr;
  // first reflector: w = r + sign(r_0) ||r|| e_0, normalised; g_0 = -sign(r_0) ||r||
  double r0 = 0.0;
  MLAMG_TRY(at(r, 0, &r0));
  hipLaunchKernelGGL(k_hh_next, dim3(nb), dim3(kGmThreads), 0, s, Wk(0), r, n, (int64_t)0,
                     hh_sign(r0) * normr, 1);
  MLAMG_HIP(hipGetLastError());
  double wn = 0.0;
  MLAMG_TRY(nrm(Wk(0), n, &wn));
  hipLaunchKernelGGL(k_gm_scale, dim3(nb), dim3(kGmThreads), 0, s, Wk(0), Wk(0), n, wn);
  std::vector<double> g(max_inner + 1, 0.0), H((size_t)max_inner * max_inner, 0.0);
  std::vector<double> Qc(max_inner, 1.0), Qs(max_inner, 0.0), head(max_inner + 2, 0.0);
  g[0] = -hh_sign(r0) * normr;
  int inner = 0, niter = 0;
  for (inner = 0; inner < max_inner; ++inner) {
    // v = P_0 .. P_inner e_inner
    hipLaunchKernelGGL(k_hh_unit, dim3(nb), dim3(kGmThreads), 0, s, v, Wk(inner), n,
                       (int64_t)inner);
    for (int j = inner - 1; j >= 0; --j) MLAMG_TRY(apply(v, j));
    // v = M A v
    MLAMG_TRY(spmv_set(A, v, u, nullptr, s));
    MLAMG_TRY(psolve(u, v));
    for (int j = 0; j <= inner; ++j) MLAMG_TRY(apply(v, j));
    if (inner != n - 1) {
      double alpha = 0.0;
      MLAMG_TRY(nrm(v + inner + 1, n - inner - 1, &alpha));
      if (alpha == 0.0 && inner < max_inner - 1) {
        // pyamg's reflector storage starts zeroed: an unused reflector is the identity
        MLAMG_HIP(hipMemsetAsync(Wk(inner + 1), 0, sizeof(double) * n, s));
      }
      if (alpha != 0.0) {
        double v1 = 0.0;
        MLAMG_TRY(at(v, inner + 1, &v1));
        alpha = hh_sign(v1) * alpha;
        const int make_w = inner < max_inner - 1;
        hipLaunchKernelGGL(k_hh_next, dim3(nb), dim3(kGmThreads), 0, s,
                           make_w ? Wk(inner + 1) : u, v, n, (int64_t)(inner + 1), alpha,
                           make_w);
        MLAMG_HIP(hipGetLastError());
        if (make_w) {
          MLAMG_TRY(nrm(Wk(inner + 1), n, &wn));
          hipLaunchKernelGGL(k_gm_scale, dim3(nb), dim3(kGmThreads), 0, s, Wk(inner + 1),
                             Wk(inner + 1), n, wn);
        }
      }
    }
    const int hl = (int)std::min<int64_t>(inner + 2, n);
    MLAMG_HIP(hipMemcpyAsync(head.data(), v, sizeof(double) * hl, hipMemcpyDeviceToHost, s));
    MLAMG_HIP(hipStreamSynchronize(s));
    for (int j = 0; j < inner; ++j) {  // the previous rotations on the head
      const double a0 = head[j], a1 = head[j + 1];
      head[j] = Qc[j] * a0 + Qs[j] * a1;
      head[j + 1] = -Qs[j] * a0 + Qc[j] * a1;
    }
    if (inner != n - 1 && head[inner + 1] != 0.0) {
      double c = 1.0, sn = 0.0, rr = 0.0;
      lartg(head[inner], head[inner + 1], &c, &sn, &rr);
      Qc[inner] = c;
      Qs[inner] = sn;
      const double g0 = g[inner], g1 = g[inner + 1];
      g[inner] = c * g0 + sn * g1;
      g[inner + 1] = -sn * g0 + c * g1;
      head[inner] = c * head[inner] + sn * head[inner + 1];
      head[inner + 1] = 0.0;
    }
    for (int j = 0; j <= inner && j < max_inner; ++j) H[(size_t)inner * max_inner + j] = head[j];
    ++niter;
    if (inner < max_inner - 1) {
      normr = std::fabs(g[inner + 1]);
      if (normr < tol) break;  // pyamg breaks before recording the estimate
      if (resid_hist && nh < hist_cap) resid_hist[nh++] = normr;
    }
  }
  if (inner == max_inner) inner = max_inner - 1;
  // y = R^-1 g (R upper triangular: column c of R is H[c][0 .. c])
  std::vector<double> y(inner + 1, 0.0);
  for (int k = inner; k >= 0; --k) {
    double t = g[k];
    for (int c = k + 1; c <= inner; ++c) t -= H[(size_t)c * max_inner + k] * y[c];
    y[k] = t / H[(size_t)k * max_inner + k];
  }
  // update = P_0 (y_0 e_0 + P_1 (y_1 e_1 + .. P_inner (y_inner e_inner))) (Horner)
  MLAMG_HIP(hipMemsetAsync(u, 0, sizeof(double) * n, s));
  for (int j = inner; j >= 0; --j) {
    hipLaunchKernelGGL(k_hh_addat, dim3(1), dim3(1), 0, s, u, (int64_t)j, y[j]);
    MLAMG_TRY(apply(u, j));
  }
  hipLaunchKernelGGL(k_hh_axpy1, dim3(nb), dim3(kGmThreads), 0, s, x, u, n);
  MLAMG_HIP(hipGetLastError());
  MLAMG_TRY(pres(&normr));
  if (resid_hist && nh < hist_cap) resid_hist[nh++] = normr;
  *iters_out = niter;
  *info_out = normr < tol ? 0 : niter;
  return MLAMG_OK;
}

}  // namespace mlamg

using namespace mlamg;

extern "C" {

int mlamg_gmres_householder(const mlamg_csr* A, mlamg_hier* M, const double* b, double* x,
                            double tol, int maxiter, int x_is_zero, int* info, int* inner_iters,
                            double* resid_hist_host, int hist_cap, void* stream) {
  MLAMG_REQUIRE(A && M && info && inner_iters, "NULL argument");
  MLAMG_REQUIRE(A->n_rows == A->n_cols, "square matrix required");
  MLAMG_REQUIRE(hier_fine_rows(M) == A->n_rows, "preconditioner hierarchy does not match A");
  MLAMG_REQUIRE(A->n_rows == 0 || (b && x && b != x), "b and x must be distinct device vectors");
  MLAMG_REQUIRE(tol >= 0.0, "tol >= 0 required");
  if (A->n_rows == 0) {
    *info = 0;
    *inner_iters = 0;
    return MLAMG_OK;
  }
  if (x_is_zero) MLAMG_HIP(hipMemsetAsync(x, 0, sizeof(double) * A->n_rows, S(stream)));
  return gmres_householder_impl(A, M, b, x, tol, maxiter, x_is_zero != 0, info, inner_iters,
                                resid_hist_host, resid_hist_host ? hist_cap : 0, S(stream));
}

int mlamg_gmres(const mlamg_csr* A, mlamg_hier* M, const double* b, double* x, double rtol,
                int restart, int maxiter, int x_is_zero, int* info, int* inner_iters,
                double* presid_hist_host, int hist_cap, void* stream) {
  MLAMG_REQUIRE(A && M && info && inner_iters, "NULL argument");
  MLAMG_REQUIRE(A->n_rows == A->n_cols, "square matrix required");
  MLAMG_REQUIRE(hier_fine_rows(M) == A->n_rows, "preconditioner hierarchy does not match A");
  MLAMG_REQUIRE(A->n_rows == 0 || (b && x && b != x), "b and x must be distinct device vectors");
  MLAMG_REQUIRE(rtol >= 0.0, "rtol >= 0 required");
  if (A->n_rows == 0) {
    *info = 0;
    *inner_iters = 0;
    return MLAMG_OK;
  }
  return gmres_impl(A, M, b, x, rtol, restart, maxiter, x_is_zero != 0, info, inner_iters,
                    presid_hist_host, presid_hist_host ? hist_cap : 0, S(stream));
}

}  // extern "C"
