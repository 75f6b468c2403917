// SpMV kernel lab: times exact-order (scipy csr_matvec summation order) SpMV variants on one
// operator dumped by tools/level_driver.py (raw .bin arrays), checks each is bitwise equal to
// the reference variant. Standalone (no torch):
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 tools/spmv_lab.hip -o spmv_lab
//   ./spmv_lab DIR/A1
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <string>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));       \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

template <class T>
static std::vector<T> load(const std::string& p) {
  FILE* f = fopen(p.c_str(), "rb");
  if (!f) {
    fprintf(stderr, "cannot open %s\n", p.c_str());
    exit(1);
  }
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  std::vector<T> v(n / sizeof(T));
  if (fread(v.data(), 1, n, f) != (size_t)n) exit(1);
  fclose(f);
  return v;
}

__device__ __forceinline__ int64_t xcd_block(int64_t b, int64_t nb) {
  const int64_t q = nb >> 3, r = nb & 7, g = b & 7, i = b >> 3;
  return (g < r ? g * (q + 1) : r * (q + 1) + (g - r) * q) + i;
}

// stream: T threads, <= T rows and <= NNZ nonzeros per block
// MODE (diagnostics, not bitwise): 1 = no x gather (x read at the nonzero's own slot),
// 2 = phase 2 reads one product per row only
template <int T, int NNZ, bool XCD, int MODE = 0>
__global__ __launch_bounds__(T) void k_stream(const int32_t* __restrict__ ip,
                                              const int32_t* __restrict__ ij,
                                              const double* __restrict__ ax,
                                              const int32_t* __restrict__ blk,
                                              const double* __restrict__ x, double* __restrict__ y) {
  __shared__ double prod[NNZ];
  __shared__ int32_t rp[T + 1];
  const int b = XCD ? (int)xcd_block(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int tid = threadIdx.x;
  const int r0 = blk[b], r1 = blk[b + 1], nr = r1 - r0;
  const int e0 = ip[r0];
  const int ne = ip[r1] - e0;
  for (int t = tid; t <= nr; t += T) rp[t] = ip[r0 + t] - e0;
  constexpr int U = NNZ / T;
  int32_t cc[U];
  double vv[U], xv[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int e = tid + u * T;
    cc[u] = e < ne ? __builtin_nontemporal_load(ij + e0 + e) : -1;
    vv[u] = e < ne ? __builtin_nontemporal_load(ax + e0 + e) : 0.0;
  }
#pragma unroll
  for (int u = 0; u < U; ++u)
    xv[u] = cc[u] >= 0 ? x[MODE == 1 ? ((tid + u * T) & 1023) : cc[u]] : 0.0;
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (tid + u * T < ne) prod[tid + u * T] = vv[u] * xv[u];
  __syncthreads();
  for (int t = tid; t < nr; t += T) {
    double s = 0.0;
    const int ka = rp[t], kb = MODE == 2 ? min(rp[t + 1], rp[t] + 1) : rp[t + 1];
    int k = ka;
    for (; k + 4 <= kb; k += 4) {
      const double p0 = prod[k], p1 = prod[k + 1], p2 = prod[k + 2], p3 = prod[k + 3];
      s += p0;
      s += p1;
      s += p2;
      s += p3;
    }
    for (; k < kb; ++k) s += prod[k];
    y[r0 + t] = s;
  }
}

// scalar: one lane per row, reads its own row straight from global memory
template <int T>
__global__ __launch_bounds__(T) void k_scalar(const int32_t* __restrict__ ip,
                                              const int32_t* __restrict__ ij,
                                              const double* __restrict__ ax, int n,
                                              const double* __restrict__ x, double* __restrict__ y) {
  const int row = (int)xcd_block(blockIdx.x, gridDim.x) * T + threadIdx.x;
  if (row >= n) return;
  const int ka = ip[row], kb = ip[row + 1];
  double s = 0.0;
  int k = ka;
  for (; k + 4 <= kb; k += 4) {
    int c[4];
    double v[4], xv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      c[u] = ij[k + u];
      v[u] = ax[k + u];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) xv[u] = x[c[u]];
#pragma unroll
    for (int u = 0; u < 4; ++u) s += v[u] * xv[u];
  }
  for (; k < kb; ++k) s += ax[k] * x[ij[k]];
  y[row] = s;
}

// wave-stream: each WAVE owns a row group (<= 64 rows, <= 64*U nonzeros), no block barrier
template <int U, int WPB>
__global__ __launch_bounds__(64 * WPB) void k_wave(const int32_t* __restrict__ ip,
                                                   const int32_t* __restrict__ ij,
                                                   const double* __restrict__ ax,
                                                   const int32_t* __restrict__ blk, int nblk,
                                                   const double* __restrict__ x,
                                                   double* __restrict__ y) {
  __shared__ double prod_all[WPB][64 * U];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int b = (int)xcd_block(blockIdx.x, gridDim.x) * WPB + w;
  if (b >= nblk) return;
  double* prod = prod_all[w];
  const int r0 = blk[b], r1 = blk[b + 1], nr = r1 - r0;
  const int e0 = ip[r0];
  const int ne = ip[r1] - e0;
  int32_t cc[U];
  double vv[U], xv[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int e = lane + u * 64;
    cc[u] = e < ne ? __builtin_nontemporal_load(ij + e0 + e) : -1;
    vv[u] = e < ne ? __builtin_nontemporal_load(ax + e0 + e) : 0.0;
  }
  const int ka = lane < nr ? ip[r0 + lane] - e0 : 0;
  const int kb = lane < nr ? ip[r0 + lane + 1] - e0 : 0;
#pragma unroll
  for (int u = 0; u < U; ++u) xv[u] = cc[u] >= 0 ? x[cc[u]] : 0.0;
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (lane + u * 64 < ne) prod[lane + u * 64] = vv[u] * xv[u];
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if (lane < nr) {
    double s = 0.0;
    int k = ka;
    for (; k + 4 <= kb; k += 4) {
      const double p0 = prod[k], p1 = prod[k + 1], p2 = prod[k + 2], p3 = prod[k + 3];
      s += p0;
      s += p1;
      s += p2;
      s += p3;
    }
    for (; k < kb; ++k) s += prod[k];
    y[r0 + lane] = s;
  }
}

// sorted-gather stream: within each block the nonzeros are stored sorted by column (so one
// wave-instruction's 64 gathers hit few cache lines), each packed as (col - base) << PB | pos,
// pos = the nonzero's CSR slot in the block; products land in LDS at their CSR slot and phase 2
// sums each row in stored order exactly as before -> bitwise the CSR-stream result.
template <int T, int NNZ, int PB>
__global__ __launch_bounds__(T) void k_sorted(const int32_t* __restrict__ ip,
                                              const uint32_t* __restrict__ pk,
                                              const double* __restrict__ av,
                                              const int32_t* __restrict__ blk,
                                              const int32_t* __restrict__ base,
                                              const double* __restrict__ x, double* __restrict__ y) {
  __shared__ double prod[NNZ];
  __shared__ int32_t rp[T + 1];
  const int b = (int)xcd_block(blockIdx.x, gridDim.x);
  const int tid = threadIdx.x;
  const int r0 = blk[b], r1 = blk[b + 1], nr = r1 - r0;
  const int e0 = ip[r0];
  const int ne = ip[r1] - e0;
  const int cb = base[b];
  for (int t = tid; t <= nr; t += T) rp[t] = ip[r0 + t] - e0;
  constexpr int U = NNZ / T;
  uint32_t w[U];
  double vv[U], xv[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int e = tid + u * T;
    w[u] = e < ne ? __builtin_nontemporal_load(pk + e0 + e) : 0xffffffffu;
    vv[u] = e < ne ? __builtin_nontemporal_load(av + e0 + e) : 0.0;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) xv[u] = w[u] != 0xffffffffu ? x[cb + (int)(w[u] >> PB)] : 0.0;
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (w[u] != 0xffffffffu) prod[w[u] & ((1u << PB) - 1)] = vv[u] * xv[u];
  __syncthreads();
  for (int t = tid; t < nr; t += T) {
    double s = 0.0;
    const int ka = rp[t], kb = rp[t + 1];
    int k = ka;
    for (; k + 4 <= kb; k += 4) {
      const double p0 = prod[k], p1 = prod[k + 1], p2 = prod[k + 2], p3 = prod[k + 3];
      s += p0;
      s += p1;
      s += p2;
      s += p3;
    }
    for (; k < kb; ++k) s += prod[k];
    y[r0 + t] = s;
  }
}

static std::vector<int32_t> partition(const std::vector<int32_t>& ip, int maxr, int maxnnz) {
  std::vector<int32_t> blk{0};
  const int n = (int)ip.size() - 1;
  int r = 0;
  while (r < n) {
    int e = r;
    while (e < n && e - r < maxr && ip[e + 1] - ip[r] <= maxnnz) ++e;
    if (e == r) {
      fprintf(stderr, "row %d longer than %d\n", r, maxnnz);
      exit(2);
    }
    blk.push_back(e);
    r = e;
  }
  return blk;
}

int main(int argc, char** argv) {
  if (argc < 2) return 1;
  std::string p = argv[1];
  auto ip = load<int32_t>(p + ".indptr.bin");
  auto ij = load<int32_t>(p + ".indices.bin");
  auto ax = load<double>(p + ".data.bin");
  auto shp = load<int64_t>(p + ".shape.bin");
  const int n = (int)shp[0], m = (int)shp[1];
  const int64_t nnz = ax.size();
  int32_t *dip, *dij;
  double *dax, *dx, *dy, *dref;
  CK(hipMalloc(&dip, ip.size() * 4));
  CK(hipMalloc(&dij, ij.size() * 4));
  CK(hipMalloc(&dax, ax.size() * 8));
  CK(hipMalloc(&dx, (size_t)m * 8));
  CK(hipMalloc(&dy, (size_t)n * 8));
  CK(hipMalloc(&dref, (size_t)n * 8));
  CK(hipMemcpy(dip, ip.data(), ip.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dij, ij.data(), ij.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dax, ax.data(), ax.size() * 8, hipMemcpyHostToDevice));
  std::vector<double> hx(m);
  uint64_t st = 12345;
  for (int i = 0; i < m; ++i) {
    st = st * 6364136223846793005ull + 1442695040888963407ull;
    hx[i] = (double)(st >> 11) / 9007199254740992.0 - 0.5;
  }
  CK(hipMemcpy(dx, hx.data(), (size_t)m * 8, hipMemcpyHostToDevice));
  const double bytes = 12.0 * nnz + 4.0 * (n + 1) + 8.0 * m + 8.0 * n;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<double> href(n), hy(n);
  bool have_ref = false;
  auto timeit = [&](const char* name, auto launch) {
    CK(hipMemset(dy, 0, (size_t)n * 8));
    launch();
    CK(hipDeviceSynchronize());
    const int reps = 20;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps;
    CK(hipMemcpy(hy.data(), dy, (size_t)n * 8, hipMemcpyDeviceToHost));
    if (!have_ref) {
      href = hy;
      have_ref = true;
    }
    const bool same = memcmp(hy.data(), href.data(), (size_t)n * 8) == 0;
    printf("%-28s %9.1f us %7.0f GB/s %s\n", name, us, bytes / us / 1e3, same ? "bitwise" : "DIFFERS");
  };
  printf("%s: n=%d m=%d nnz=%lld avg_row=%.1f algorithmic %.1f MB\n", p.c_str(), n, m,
         (long long)nnz, (double)nnz / n, bytes / 1e6);
#define STREAM(T, NNZ, XCD, ...)                                                                 \
  {                                                                                           \
    auto blk = partition(ip, T, NNZ);                                                         \
    int32_t* dblk;                                                                            \
    CK(hipMalloc(&dblk, blk.size() * 4));                                                     \
    CK(hipMemcpy(dblk, blk.data(), blk.size() * 4, hipMemcpyHostToDevice));                   \
    const int nb = (int)blk.size() - 1;                                                       \
    timeit("stream<" #T "," #NNZ "," #XCD #__VA_ARGS__ ">", [&] {                             \
      hipLaunchKernelGGL((k_stream<T, NNZ, XCD __VA_ARGS__>), dim3(nb), dim3(T), 0, 0, dip, dij, \
                         dax, dblk,                                                           \
                         dx, dy);                                                             \
    });                                                                                       \
    CK(hipFree(dblk));                                                                        \
  }
  STREAM(256, 2048, true)
  STREAM(256, 2048, false)
  STREAM(256, 1024, true)
  STREAM(128, 1024, true)
  STREAM(128, 2048, true)
  STREAM(64, 512, true)
  STREAM(64, 1024, true)
  STREAM(512, 4096, true)
  STREAM(256, 4096, true)
  STREAM(256, 2048, true, , 1)
  STREAM(256, 2048, true, , 2)
  STREAM(256, 4096, true, , 1)
  STREAM(256, 4096, true, , 2)
#define SORTED(T, NNZ, PB)                                                                   \
  {                                                                                           \
    auto blk = partition(ip, T, NNZ);                                                         \
    const int nb = (int)blk.size() - 1;                                                       \
    std::vector<uint32_t> pk(nnz);                                                            \
    std::vector<double> pv(nnz);                                                              \
    std::vector<int32_t> bs(nb);                                                              \
    bool ok = true;                                                                           \
    for (int b = 0; b < nb && ok; ++b) {                                                      \
      const int e0 = ip[blk[b]], e1 = ip[blk[b + 1]];                                         \
      std::vector<int> ord(e1 - e0);                                                          \
      for (int k = 0; k < e1 - e0; ++k) ord[k] = k;                                           \
      std::stable_sort(ord.begin(), ord.end(),                                                \
                       [&](int a, int c) { return ij[e0 + a] < ij[e0 + c]; });                \
      const int lo = e1 > e0 ? ij[e0 + ord[0]] : 0;                                           \
      const int hi = e1 > e0 ? ij[e0 + ord.back()] : 0;                                       \
      if ((int64_t)(hi - lo) >= (int64_t(1) << (32 - PB))) ok = false;                        \
      bs[b] = lo;                                                                             \
      for (int k = 0; k < e1 - e0; ++k) {                                                     \
        pk[e0 + k] = ((uint32_t)(ij[e0 + ord[k]] - lo) << PB) | (uint32_t)ord[k];             \
        pv[e0 + k] = ax[e0 + ord[k]];                                                         \
      }                                                                                       \
    }                                                                                         \
    if (!ok) {                                                                                \
      printf("sorted<" #T "," #NNZ "> column span too wide\n");                              \
    } else {                                                                                  \
      int32_t *dblk, *dbs;                                                                    \
      uint32_t* dpk;                                                                          \
      double* dpv;                                                                            \
      CK(hipMalloc(&dblk, blk.size() * 4));                                                   \
      CK(hipMalloc(&dbs, bs.size() * 4));                                                     \
      CK(hipMalloc(&dpk, pk.size() * 4));                                                     \
      CK(hipMalloc(&dpv, pv.size() * 8));                                                     \
      CK(hipMemcpy(dblk, blk.data(), blk.size() * 4, hipMemcpyHostToDevice));                 \
      CK(hipMemcpy(dbs, bs.data(), bs.size() * 4, hipMemcpyHostToDevice));                    \
      CK(hipMemcpy(dpk, pk.data(), pk.size() * 4, hipMemcpyHostToDevice));                    \
      CK(hipMemcpy(dpv, pv.data(), pv.size() * 8, hipMemcpyHostToDevice));                    \
      timeit("sorted<" #T "," #NNZ ">", [&] {                                                 \
        hipLaunchKernelGGL((k_sorted<T, NNZ, PB>), dim3(nb), dim3(T), 0, 0, dip, dpk, dpv,    \
                           dblk, dbs, dx, dy);                                                \
      });                                                                                     \
      CK(hipFree(dblk));                                                                      \
      CK(hipFree(dbs));                                                                       \
      CK(hipFree(dpk));                                                                       \
      CK(hipFree(dpv));                                                                       \
    }                                                                                         \
  }
  SORTED(256, 2048, 11)
  SORTED(256, 4096, 12)
  SORTED(512, 4096, 12)
  SORTED(128, 1024, 10)
  SORTED(64, 512, 9)
#define WAVE(U, WPB)                                                                          \
  {                                                                                           \
    auto blk = partition(ip, 64, 64 * U);                                                     \
    int32_t* dblk;                                                                            \
    CK(hipMalloc(&dblk, blk.size() * 4));                                                     \
    CK(hipMemcpy(dblk, blk.data(), blk.size() * 4, hipMemcpyHostToDevice));                   \
    const int nw = (int)blk.size() - 1;                                                       \
    timeit("wave<" #U "," #WPB ">", [&] {                                                     \
      hipLaunchKernelGGL((k_wave<U, WPB>), dim3((nw + WPB - 1) / WPB), dim3(64 * WPB), 0, 0,  \
                         dip, dij, dax, dblk, nw, dx, dy);                                    \
    });                                                                                       \
    CK(hipFree(dblk));                                                                        \
  }
  WAVE(8, 4)
  WAVE(16, 4)
  WAVE(16, 2)
  WAVE(32, 2)
  WAVE(8, 1)
  timeit("scalar<256>", [&] {
    hipLaunchKernelGGL((k_scalar<256>), dim3((n + 255) / 256), dim3(256), 0, 0, dip, dij, dax, n,
                       dx, dy);
  });
  timeit("scalar<64>", [&] {
    hipLaunchKernelGGL((k_scalar<64>), dim3((n + 63) / 64), dim3(64), 0, 0, dip, dij, dax, n, dx,
                       dy);
  });
  return 0;
}
