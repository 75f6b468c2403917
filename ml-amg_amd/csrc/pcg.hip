// Coarsest-level solve without a size cap: the reference factorises
// the Galerkin operator with SuperLU at any size (`spla.factorized(A_H)`, ns/lib/multigrid.py:168;
// `splu(A_H, COLAMD)`, ns/preconditioner/MLAMG.py:122). A dense inverse (dense.hip) stops being
// an option once n_c^2 doubles no longer fit or its O(n_c^3) setup dominates, so above that the
// coarse system A_c x = b is solved by preconditioned conjugate gradients, the preconditioner
// being one V-cycle (zero guess) of an inner multilevel hierarchy built on A_c itself — setup
// O(nnz), a handful of V-cycles per solve. The solve runs to a relative residual
// ||b - A_c x||_2 <= rtol * ||b||_2 (default 1e-12), i.e. it replaces an exact factorisation by
// a solve accurate far beyond the outer cycle's own convergence (parity: tolerance, stated in
// the tests). A_c must be symmetric positive definite (P^T A P of an SPD A, the reference's
// use); the V(nu,nu) weighted-Jacobi cycle with R = P^T is then a symmetric preconditioner.
//
// Every kernel checks the solver's done flag (shared with the inner hierarchy, whose kernels
// check it too), so once the tolerance is met the remaining launches of the solve return at
// once. Eagerly launched solves poll the flag every few iterations and stop launching; inside a
// stream capture every iteration up to maxit is recorded (the V-cycle executor therefore runs
// hierarchies with a PCG coarse solver eagerly). Reductions are fixed-order (partials over a
// fixed grid, summed in order by the kernel that consumes the scalar), so a solve is
// deterministic.
#include "common.hpp"

#include <cmath>

struct mlamg_pcg {
  const mlamg_csr* A = nullptr;
  mlamg_hier* M = nullptr;
  int64_t n = 0;
  double rtol = 1e-12;
  int maxit = 200;
  int poll = 2;
  void* mem = nullptr;
  double *r = nullptr, *p = nullptr, *q = nullptr, *partial = nullptr;
  double* scal = nullptr;     // [0] rho, [1] alpha, [2] beta, [3] ||b||^2, [4] ||r||^2 (last),
                              // [5] largest final ||r||/||b|| over solves, [6], [7] rho by
                              // iteration parity
  int32_t* flags = nullptr;   // [0] iterations of the last solve, [1] solves not converged,
                              // [2] total iterations, [3] solves ended by a breakdown
                              // (p.Ap <= 0, r.z <= 0 or a NaN: A_c or the preconditioner
                              // not positive definite)
  int32_t* ctr = nullptr;     // arrival counter of the reduction kernels (re-armed to 0)
  int32_t* done_host = nullptr;  // two pinned slots of the polled done flag
  hipEvent_t ev[2] = {nullptr, nullptr};
  int nb = 1;
};

namespace mlamg {

constexpr int kPcgThreads = 256;
constexpr int kPcgMaxBlocks = 1024;

__device__ __forceinline__ double pcg_wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ void block_partial(double s, double* partial) {
  __shared__ double red[kPcgThreads / 64];
  s = pcg_wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
}

// Each reduction kernel finishes its own scalar step: every workgroup writes its partial, and the
// workgroup that arrives last at the solver's counter (release / acquire at agent scope, so the
// other XCDs' partials are visible to it) sums the partials in fixed order and updates the
// scalars — one launch per dot product instead of a partials launch plus a one-workgroup
// finalisation launch. The counter is re-armed by that same workgroup.
__device__ __forceinline__ bool arrive_last(int32_t* ctr) {
  __shared__ int last;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const int prev = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    last = prev == (int)gridDim.x - 1;
    if (last) {
      __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __threadfence();
    }
  }
  __syncthreads();
  return last != 0;
}

// fixed-order sum of nb partials by one kPcgThreads workgroup (all threads get the total)
__device__ __forceinline__ double last_total(const double* __restrict__ partial, int nb) {
  __shared__ double red[kPcgThreads / 64];
  double s = strided_sum(partial, nb, threadIdx.x, kPcgThreads);
  s = pcg_wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  return ((red[0] + red[1]) + red[2]) + red[3];
}

// x = 0, r = b, ||b||^2; done := outer done (a finished outer iteration skips the solve); a zero
// right-hand side is solved by x = 0
__global__ __launch_bounds__(kPcgThreads) void k_pcg_init(const double* __restrict__ b,
                                                          double* __restrict__ x,
                                                          double* __restrict__ r, int64_t n,
                                                          double* __restrict__ partial,
                                                          int32_t* ctr, double* scal,
                                                          int32_t* done, const int32_t* outer,
                                                          int32_t* flags) {
  const bool skip = outer && *outer;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    *done = skip ? 1 : 0;
    flags[0] = 0;
  }
  if (skip) return;
  double s = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)kPcgThreads + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kPcgThreads) {
    const double v = b[i];
    x[i] = 0.0;
    r[i] = v;
    s += v * v;
  }
  block_partial(s, partial);
  if (!arrive_last(ctr)) return;
  const double t = last_total(partial, gridDim.x);
  if (threadIdx.x == 0) {
    scal[3] = t;
    if (!(t > 0.0)) *done = 1;
  }
}

// a breakdown ends the solve (done) and is counted; the iterate stays as it was
__device__ __forceinline__ void breakdown(int32_t* done, int32_t* flags) {
  *done = 1;
  flags[3] += 1;
}

// The iteration's dot products without the arrival counter: a reduction kernel only writes
// its per-workgroup partials, and the kernel that consumes the scalar sums them itself (every
// workgroup, last_total's fixed order, so every workgroup gets the same bits). An arrival counter
// needs an agent-scope release fence in every workgroup, and on MI355X that fence writes back the
// XCD's L2 (GMRES, the same change: 1.6-2.7x per solve). rho alternates between scal[6] and
// scal[7] by iteration parity, so no workgroup overwrites a value another one still reads.

// partials of p.q (the alpha step's denominator)
__global__ __launch_bounds__(kPcgThreads) void k_pcg_pq(const double* __restrict__ p,
                                                        const double* __restrict__ q, int64_t n,
                                                        double* __restrict__ partial,
                                                        const int32_t* done) {
  if (*done) return;
  double s = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)kPcgThreads + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kPcgThreads)
    s += p[i] * q[i];
  block_partial(s, partial);
}

// alpha = rho / (p.q); x += alpha p, r -= alpha q; partials of r.r
__global__ __launch_bounds__(kPcgThreads) void k_pcg_update(double* __restrict__ x,
                                                            double* __restrict__ r,
                                                            const double* __restrict__ p,
                                                            const double* __restrict__ q,
                                                            int64_t n, double* scal,
                                                            const double* __restrict__ pq,
                                                            double* __restrict__ partial,
                                                            int np, int32_t* done,
                                                            int32_t* flags, int it) {
  if (*done) return;
  const double t = last_total(pq, np);
  const double alpha = scal[6 + (it & 1)] / t;
  if (!(t > 0.0)) {  // p.Ap <= 0 or NaN: A_c not positive definite
    if (blockIdx.x == 0 && threadIdx.x == 0) breakdown(done, flags);
    return;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) scal[1] = alpha;
  double s = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)kPcgThreads + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kPcgThreads) {
    x[i] += alpha * p[i];
    const double v = r[i] - alpha * q[i];
    r[i] = v;
    s += v * v;
  }
  block_partial(s, partial);
}

// ||r||^2 <= rtol^2 ||b||^2 -> done (before the V-cycle, which then does nothing); iteration
// count; one workgroup
__global__ __launch_bounds__(kPcgThreads) void k_pcg_check(const double* __restrict__ partial,
                                                           int np, double* scal, int32_t* done,
                                                           int32_t* flags, double rtol) {
  if (*done) return;
  const double t = last_total(partial, np);
  if (threadIdx.x == 0) {
    scal[4] = t;
    flags[0] += 1;
    flags[2] += 1;
    if (t <= rtol * rtol * scal[3]) {
      *done = 1;
      const double rel = sqrt(t / scal[3]);
      if (rel > scal[5]) scal[5] = rel;
    } else if (!(t >= 0.0)) {
      breakdown(done, flags);  // NaN residual
    }
  }
}

// partials of r.z
__global__ __launch_bounds__(kPcgThreads) void k_pcg_rz(const double* __restrict__ r,
                                                        const double* __restrict__ z, int64_t n,
                                                        double* __restrict__ partial,
                                                        const int32_t* done) {
  if (*done) return;
  double s = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)kPcgThreads + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kPcgThreads)
    s += r[i] * z[i];
  block_partial(s, partial);
}

// rho = r.z (into scal[6 + (it + 1) % 2], the next iteration's), beta = rho / rho_old (first:
// beta = 0, so p = z); p = z + beta p
__global__ __launch_bounds__(kPcgThreads) void k_pcg_p(const double* __restrict__ z,
                                                       double* __restrict__ p, int64_t n,
                                                       const double* __restrict__ rz, int np,
                                                       double* scal, int32_t* done,
                                                       int32_t* flags, int first, int it) {
  if (*done) return;
  const double t = last_total(rz, np);
  // r != 0 here (a zero residual ended the solve), so r.z <= 0 means the preconditioner is not
  // positive definite
  if (!(t > 0.0)) {
    if (blockIdx.x == 0 && threadIdx.x == 0) breakdown(done, flags);
    return;
  }
  const double beta = first ? 0.0 : t / scal[6 + (it & 1)];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    scal[6 + ((it + 1) & 1)] = t;
    scal[0] = t;
    scal[2] = beta;
  }
  for (int64_t i = blockIdx.x * (int64_t)kPcgThreads + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kPcgThreads)
    p[i] = z[i] + beta * p[i];
}

// after the last launched iteration: a solve that did not reach the tolerance is counted
__global__ void k_pcg_end(double* scal, int32_t* done, int32_t* flags, const int32_t* outer) {
  if (threadIdx.x != 0 || *done || (outer && *outer)) return;
  flags[1] += 1;
  const double rel = sqrt(scal[4] / scal[3]);
  if (rel > scal[5]) scal[5] = rel;
  *done = 1;
}

static int pcg_grid(int64_t n) {
  return (int)std::min<int64_t>(kPcgMaxBlocks, std::max<int64_t>(1, (n + kPcgThreads - 1) /
                                                                        kPcgThreads));
}

static int pcg_iteration(mlamg_pcg* C, double* x, int32_t* done, int it, hipStream_t s) {
  const int nb = C->nb;
  const int64_t n = C->n;
  double* pa = C->partial;             // p.q partials
  double* pb = C->partial + kPcgMaxBlocks;  // r.r, then r.z partials
  MLAMG_TRY(spmv_set(C->A, C->p, C->q, done, s));
  hipLaunchKernelGGL(k_pcg_pq, dim3(nb), dim3(kPcgThreads), 0, s, C->p, C->q, n, pa, done);
  hipLaunchKernelGGL(k_pcg_update, dim3(nb), dim3(kPcgThreads), 0, s, x, C->r, C->p, C->q, n,
                     C->scal, pa, pb, nb, done, C->flags, it);
  hipLaunchKernelGGL(k_pcg_check, dim3(1), dim3(kPcgThreads), 0, s, pb, nb, C->scal, done,
                     C->flags, C->rtol);
  double* z = nullptr;
  MLAMG_TRY(hier_coarse_cycle(C->M, C->r, &z, 0, s));
  hipLaunchKernelGGL(k_pcg_rz, dim3(nb), dim3(kPcgThreads), 0, s, C->r, z, n, pa, done);
  hipLaunchKernelGGL(k_pcg_p, dim3(nb), dim3(kPcgThreads), 0, s, z, C->p, n, pa, nb, C->scal,
                     done, C->flags, 0, it);
  MLAMG_HIP(hipGetLastError());
  return MLAMG_OK;
}

int pcg_solve_impl(mlamg_pcg* C, const double* b, double* x, const int32_t* outer_done,
                   hipStream_t s) {
  if (C->n == 0) return MLAMG_OK;
  MLAMG_TRY(hier_prepare_ext(C->M));
  int32_t* done = hier_done_flag(C->M);
  const int nb = C->nb;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  MLAMG_HIP(hipStreamIsCapturing(s, &cap));
  const bool poll = cap == hipStreamCaptureStatusNone && C->done_host;
  hipLaunchKernelGGL(k_pcg_init, dim3(nb), dim3(kPcgThreads), 0, s, b, x, C->r, C->n, C->partial,
                     C->ctr, C->scal, done, outer_done, C->flags);
  double* z = nullptr;
  MLAMG_TRY(hier_coarse_cycle(C->M, C->r, &z, 0, s));
  // rho_0 = r.z into scal[6] (iteration 0 reads it), p = z
  hipLaunchKernelGGL(k_pcg_rz, dim3(nb), dim3(kPcgThreads), 0, s, C->r, z, C->n, C->partial,
                     done);
  hipLaunchKernelGGL(k_pcg_p, dim3(nb), dim3(kPcgThreads), 0, s, z, C->p, C->n, C->partial, nb,
                     C->scal, done, C->flags, 1, -1);
  // The host polls the done flag without draining the queue: after queueing group g of `poll`
  // iterations it copies the flag into pinned slot g % 2 and then waits for group g - 1's copy,
  // so the device always has the next group queued while the host reads the previous one.
  int g = 0;
  for (int it = 0; it < C->maxit; ++it) {
    MLAMG_TRY(pcg_iteration(C, x, done, it, s));
    if (poll && (it + 1) % C->poll == 0 && it + 1 < C->maxit) {
      const int slot = g & 1;
      MLAMG_HIP(hipMemcpyAsync(C->done_host + slot, done, sizeof(int32_t), hipMemcpyDeviceToHost,
                               s));
      MLAMG_HIP(hipEventRecord(C->ev[slot], s));
      if (g > 0) {
        MLAMG_HIP(hipEventSynchronize(C->ev[slot ^ 1]));
        if (C->done_host[slot ^ 1]) break;
      }
      ++g;
    }
  }
  hipLaunchKernelGGL(k_pcg_end, dim3(1), dim3(64), 0, s, C->scal, done, C->flags, outer_done);
  MLAMG_HIP(hipGetLastError());
  return MLAMG_OK;
}

// Symmetry to rounding of a square CSR (any column order, no duplicates): thread per row i,
// every stored a_ij is looked up in row j (linear scan: Galerkin rows are short and unsorted);
// a missing a_ji counts as 0. Violation: |a_ij - a_ji| > rtol * max(|a_ii|, |a_jj|) (rtol = 0:
// exact symmetry). bad[0] is set by plain stores (benign race, any violation wins).
__device__ __forceinline__ double row_entry(const int32_t* __restrict__ ip,
                                            const int32_t* __restrict__ ij,
                                            const double* __restrict__ v, int r, int c) {
  for (int k = ip[r]; k < ip[r + 1]; ++k)
    if (ij[k] == c) return v[k];
  return 0.0;
}

__global__ __launch_bounds__(256) void k_sym_check(const int32_t* __restrict__ ip,
                                                   const int32_t* __restrict__ ij,
                                                   const double* __restrict__ v, int64_t n,
                                                   double rtol, int32_t* bad) {
  const int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x;
  if (i >= n) return;
  const double dii = fabs(row_entry(ip, ij, v, (int)i, (int)i));
  bool ok = true;
  for (int k = ip[i]; k < ip[i + 1] && ok; ++k) {
    const int j = ij[k];
    if (j == (int)i) continue;
    const double a = v[k], b = row_entry(ip, ij, v, j, (int)i);
    const double scale = fmax(dii, fabs(row_entry(ip, ij, v, j, j)));
    ok = fabs(a - b) <= rtol * scale;
  }
  if (!ok) bad[0] = 1;
}

int64_t pcg_rows(const mlamg_pcg* C) { return C->n; }
mlamg_hier* pcg_inner(mlamg_pcg* C) { return C->M; }

}  // namespace mlamg

using namespace mlamg;

extern "C" {

int mlamg_pcg_create(const mlamg_csr* A, mlamg_hier* M, double rtol, int maxit,
                     mlamg_pcg** out) {
  MLAMG_REQUIRE(A && M && out, "NULL argument");
  MLAMG_REQUIRE(A->n_rows == A->n_cols, "square matrix required");
  MLAMG_REQUIRE(hier_fine_rows(M) == A->n_rows, "inner hierarchy does not match A");
  MLAMG_REQUIRE(rtol > 0.0 && maxit >= 1, "rtol > 0 and maxit >= 1 required");
  auto* C = new mlamg_pcg();
  C->A = A;
  C->M = M;
  C->n = A->n_rows;
  C->rtol = rtol;
  C->maxit = maxit;
  C->nb = pcg_grid(C->n);
  const size_t vec = ((sizeof(double) * (size_t)std::max<int64_t>(C->n, 1)) + 255) & ~size_t(255);
  const size_t total = 3 * vec + 2 * sizeof(double) * kPcgMaxBlocks + 256 + 256;
  if (hipMalloc(&C->mem, total) != hipSuccess) {
    delete C;
    set_error("pcg_create: hipMalloc failed");
    return MLAMG_ENOMEM;
  }
  char* p = static_cast<char*>(C->mem);
  C->r = reinterpret_cast<double*>(p);
  C->p = reinterpret_cast<double*>(p + vec);
  C->q = reinterpret_cast<double*>(p + 2 * vec);
  C->partial = reinterpret_cast<double*>(p + 3 * vec);
  C->scal = reinterpret_cast<double*>(p + 3 * vec + 2 * sizeof(double) * kPcgMaxBlocks);
  C->flags = reinterpret_cast<int32_t*>(p + 3 * vec + 2 * sizeof(double) * kPcgMaxBlocks + 256);
  C->ctr = C->flags + 8;
  if (hipMemset(C->mem, 0, total) != hipSuccess ||
      hipHostMalloc(&C->done_host, 2 * sizeof(int32_t), hipHostMallocDefault) != hipSuccess ||
      hipEventCreateWithFlags(&C->ev[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&C->ev[1], hipEventDisableTiming) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess) {
    if (C->done_host) (void)hipHostFree(C->done_host);
    for (hipEvent_t e : C->ev)
      if (e) (void)hipEventDestroy(e);
    (void)hipFree(C->mem);
    delete C;
    set_error("pcg_create: allocation failed");
    return MLAMG_ENOMEM;
  }
  *out = C;
  return MLAMG_OK;
}

int mlamg_pcg_destroy(mlamg_pcg* C) {
  if (C) {
    if (C->mem) (void)hipFree(C->mem);
    if (C->done_host) (void)hipHostFree(C->done_host);
    for (hipEvent_t e : C->ev)
      if (e) (void)hipEventDestroy(e);
    delete C;
  }
  return MLAMG_OK;
}

int mlamg_pcg_solve(mlamg_pcg* C, const double* b, double* x, void* stream) {
  MLAMG_REQUIRE(C && (C->n == 0 || (b && x)), "NULL argument");
  MLAMG_REQUIRE(b != x, "b and x must differ");
  return pcg_solve_impl(C, b, x, nullptr, S(stream));
}

int mlamg_pcg_breakdowns(const mlamg_pcg* C, int32_t* breakdowns, void* stream) {
  MLAMG_REQUIRE(C && breakdowns, "NULL argument");
  int32_t f[4] = {0, 0, 0, 0};
  hipStream_t s = S(stream);
  MLAMG_HIP(hipMemcpyAsync(f, C->flags, sizeof(f), hipMemcpyDeviceToHost, s));
  MLAMG_HIP(hipStreamSynchronize(s));
  *breakdowns = f[3];
  return MLAMG_OK;
}

int mlamg_csr_symmetric(const mlamg_csr* A, double rtol, int* symmetric, void* stream) {
  MLAMG_REQUIRE(A && symmetric, "NULL argument");
  MLAMG_REQUIRE(rtol >= 0.0, "rtol >= 0 required");
  if (A->n_rows != A->n_cols) {
    *symmetric = 0;
    return MLAMG_OK;
  }
  hipStream_t s = S(stream);
  int32_t* bad = static_cast<int32_t*>(scratch(sizeof(int32_t), 14));
  MLAMG_REQUIRE(bad, "csr_symmetric: scratch allocation failed");
  MLAMG_HIP(hipMemsetAsync(bad, 0, sizeof(int32_t), s));
  if (A->n_rows > 0) {
    const unsigned nb = (unsigned)((A->n_rows + 255) / 256);
    hipLaunchKernelGGL(k_sym_check, dim3(nb), dim3(256), 0, s, A->indptr, A->indices, A->data,
                       A->n_rows, rtol, bad);
    MLAMG_HIP(hipGetLastError());
  }
  int32_t h = 0;
  MLAMG_HIP(hipMemcpyAsync(&h, bad, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  MLAMG_HIP(hipStreamSynchronize(s));
  *symmetric = h == 0;
  return MLAMG_OK;
}

int mlamg_pcg_stats(const mlamg_pcg* C, int32_t* last_iters, int32_t* not_converged,
                    int32_t* total_iters, double* max_rel_residual, void* stream) {
  MLAMG_REQUIRE(C, "NULL argument");
  int32_t f[3] = {0, 0, 0};
  double sc[6] = {0, 0, 0, 0, 0, 0};
  hipStream_t s = S(stream);
  MLAMG_HIP(hipMemcpyAsync(f, C->flags, sizeof(f), hipMemcpyDeviceToHost, s));
  MLAMG_HIP(hipMemcpyAsync(sc, C->scal, sizeof(sc), hipMemcpyDeviceToHost, s));
  MLAMG_HIP(hipStreamSynchronize(s));
  if (last_iters) *last_iters = f[0];
  if (not_converged) *not_converged = f[1];
  if (total_iters) *total_iters = f[2];
  if (max_rel_residual) *max_rel_residual = sc[5];
  return MLAMG_OK;
}

}  // extern "C"
