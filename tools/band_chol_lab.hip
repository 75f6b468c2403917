// Band factor latency lab: band_chol (csrc/batch.hip) on one wave for a 484 x 484 SPD operator
// of half-bandwidth 23 (the 64^2 farm problem's coarse operator shape).
#include "common.hpp"
#include <cstdio>
#include <vector>
namespace mlamg {
constexpr int kBT = 1024;
constexpr int kBandMax = 63;  // half-bandwidth limit: rows (j, j + b] within the 64 lanes
// coarse size limit: the substitutions run on one wave, ~45 ns per row and direction; a single
// call with a larger coarse operator is faster with the device-wide dense factor and its coarse
// solve spread over the CUs (128^2: 13 vs 26 ms). Every batch-eligible size (n_c <= 1024, the
// Python engine's FUSED_BATCH_MAX_NC) is below it, so batches and single calls choose alike.
constexpr int kBandMaxNc = 1024;

__device__ __forceinline__ double readlane_d(double v, int l) {
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)x, l);
  const int hi = __builtin_amdgcn_readlane((int)(x >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// pointers in a given address space (1 global, 3 LDS): loads through them are global / LDS
// instructions, not flat ones, so the compiler counts them on their own counters and a
// prefetch stays in flight (a flat load in a non-inlined function waits on every counter)
template <int AS>
using as_ptr = __attribute__((address_space(AS))) double*;
template <int AS>
using as_cptr = const __attribute__((address_space(AS))) double*;

// Right-looking banded Cholesky of AH (dense n_c x n_c, only |i - k| <= b read) over a sliding
// window of the b + 1 active rows in LDS (row i in slot i mod (b + 1), its entries k in
// [i - b, i) in column slots k mod (b + 1); diagonals in their own ring, slot i mod (b + 2)).
// Column j: l_i = a_ij / l_jj for i in (j, j + b], a_ik -= l_i l_k for j < k <= i <= j + b,
// and row j + b + 1 enters the slots row j leaves: one barrier per column (the entering row and
// every update touch slots column j does not read). The entering rows are loaded from AH two
// columns ahead. Out, in the band solve's lane layout (step j's 64 lane values contiguous, steps
// padded by kBandPad zero steps on either side, see band_solve): F[j][i mod 64] = L[i][j] / L[j][j]
// for i in (j, j + b], G[i][j mod 64] = L[i][j], RI[j] = 1 / L[j][j]. Returns false
// (uniformly) on a non-positive pivot.
constexpr int kBandPad = 32;  // zero steps before and after the band solve's lane layout
__device__ __forceinline__ int64_t band_at(int j, int l) { return (int64_t)(j + kBandPad) * 64 + l; }

// LDS ordering between the lanes of one wave: its LDS operations complete in issue order, so a
// wavefront-scope fence (no wait on global memory: prefetches and stores stay in flight) only
// keeps the compiler from moving LDS accesses across it
__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One workgroup, a (row, column) pair of column j's update per thread: rings of power-of-two
// sizes (slot = index & mask, no integer division), >= b + 2 rows and diagonals, rows stored
// with an odd stride (conflict-free LDS columns).
__device__ bool band_chol(const double* __restrict__ AH_, int nc, int b, double* lds,
                          double* __restrict__ F_, double* __restrict__ G_,
                          double* __restrict__ RI_, int tid) {
  const as_cptr<1> AH = (as_cptr<1>)AH_;
  const as_ptr<1> F = (as_ptr<1>)F_, G = (as_ptr<1>)G_, RI = (as_ptr<1>)RI_;
  int w = 1;
  while (w < b + 2) w <<= 1;
  const int m = w - 1, ws = w + 1;
  const as_ptr<3> off = (as_ptr<3>)lds;  // w rows of stride ws
  const as_ptr<3> dg = off + w * ws;     // w
  // zeros outside the band, and on the padding steps
  for (int64_t q = tid; q < (int64_t)(nc + 2 * kBandPad) * 64; q += kBT) {
    F[q] = 0.0;
    G[q] = 0.0;
  }
  for (int q = tid; q < nc + 2 * kBandPad; q += kBT) RI[q] = 0.0;
  for (int q = tid; q < (b + 1) * (b + 1); q += kBT) {
    const int i = q / (b + 1), k = q - i * (b + 1);
    if (i < nc && k < i) off[(i & m) * ws + (k & m)] = AH[(int64_t)i * nc + k];
  }
  for (int i = tid; i <= b && i < nc; i += kBT) dg[i & m] = AH[(int64_t)i * nc + i];
  // this thread's pairs (di, dk), 1 <= dk <= di <= b (rows j + di, j + dk): b <= 63 gives at
  // most 2016 pairs, two per thread
  int pdi[2] = {0, 0}, pdk[2] = {0, 0};
  const int npairs = b * (b + 1) / 2;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int p = tid + u * kBT;
    if (p < npairs) {
      int di = (int)((1.0 + sqrt(1.0 + 8.0 * (double)p)) * 0.5);
      while (di * (di - 1) / 2 > p) --di;
      while (di * (di + 1) / 2 <= p) ++di;
      pdi[u] = di;
      pdk[u] = p - di * (di - 1) / 2 + 1;
    }
  }
  // entering-row entries of this thread (tid <= b): row j + b + 1, column j + 1 + tid
  auto enter_val = [&](int j) -> double {
    const int ni = j + b + 1, k = j + 1 + tid;
    return tid <= b && ni < nc ? AH[(int64_t)ni * nc + (k < ni ? k : ni)] : 0.0;
  };
  double pre0 = enter_val(0), pre1 = enter_val(1);
  __syncthreads();
  auto column = [&](int j, double v) -> bool {
    const double d = dg[j & m];
    if (!(d > 0.0)) return false;  // every thread read the same pivot
    const double ljj = sqrt(d), r = 1.0 / ljj;
    const int cj = j & m;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int di = pdi[u], dk = pdk[u];
      const int i = j + di, k = j + dk;
      if (di == 0 || i >= nc) continue;
      const double li = off[(i & m) * ws + cj] * r;
      if (dk == di) {
        dg[i & m] = dg[i & m] - li * li;
        F[band_at(j, i & 63)] = li * r;
        G[band_at(i, j & 63)] = li;
      } else {
        const double lk = off[(k & m) * ws + cj] * r;
        off[(i & m) * ws + (k & m)] = off[(i & m) * ws + (k & m)] - li * lk;
      }
    }
    if (tid == 0) RI[j + kBandPad] = r;
    // the entering row (raw A_H: no column <= j has reached it), loaded two columns before
    const int ni = j + b + 1;
    if (ni < nc && tid <= b) {
      const int k = j + 1 + tid;
      if (k < ni) off[(ni & m) * ws + (k & m)] = v;
      else dg[ni & m] = v;
    }
    __syncthreads();
    return true;
  };
  for (int j = 0; j < nc; j += 2) {  // two columns per trip: each prefetch has a column to land
    const double v0 = pre0;
    pre0 = enter_val(j + 2);
    if (!column(j, v0)) return false;
    if (j + 1 >= nc) break;
    const double v1 = pre1;
    pre1 = enter_val(j + 3);
    if (!column(j + 1, v1)) return false;
  }
  return true;
}

__global__ __launch_bounds__(1024) void k_lab(const double* AH, int nc, int b, double* F, double* G,
                                            double* RI, long long* t, int* ok) {
  extern __shared__ double lds[];
  const long long t0 = wall_clock64();
  const bool r = band_chol(AH, nc, b, lds, F, G, RI, threadIdx.x);
  if (threadIdx.x == 0) { t[0] = wall_clock64() - t0; ok[0] = r; }
}
}
using namespace mlamg;
int main() {
  const int nc = 484, b = 23;
  std::vector<double> A((size_t)nc * nc, 0.0);
  for (int i = 0; i < nc; ++i)
    for (int k = std::max(0, i - b); k <= std::min(nc - 1, i + b); ++k) A[(size_t)i * nc + k] = i == k ? 60.0 : -1.0 / (1 + std::abs(i - k));
  double *dA, *F, *G, *RI; long long* t; int* ok;
  hipMalloc(&dA, 8 * A.size()); hipMalloc(&F, 8 * 64 * (nc + 64)); hipMalloc(&G, 8 * 64 * (nc + 64));
  hipMalloc(&RI, 8 * (nc + 64)); hipMalloc(&t, 8); hipMalloc(&ok, 4);
  hipMemcpy(dA, A.data(), 8 * A.size(), hipMemcpyHostToDevice);
  for (int w = 0; w < 3; ++w) { hipLaunchKernelGGL(k_lab, 1, 1024, 64 * 1024, 0, dA, nc, b, F, G, RI, t, ok); hipDeviceSynchronize(); }
  long long h; int o; hipMemcpy(&h, t, 8, hipMemcpyDeviceToHost); hipMemcpy(&o, ok, 4, hipMemcpyDeviceToHost);
  printf("band_chol n_c %d b %d: %.1f us (%.2f us per column), ok %d\n", nc, b, h * 1e-2, h * 1e-2 / nc, o);
  return 0;
}
