// Gather-pattern lab for the C4 fine-level SpMV (216^3 7-point Laplacian): how fast can the
// x gather of a 7-point stencil run on MI355X, compared with a plain stream of the same bytes?
// Diagnostics only (no bitwise claims): every variant reads x (80 MB) and writes y (80 MB).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/stencil_lab.hip -o /tmp/stencil_lab
//   /tmp/stencil_lab [n=216] [reps=50]
// Variants (MASK of neighbour offsets gathered besides the centre: bit0 +-1, bit1 +-n,
// bit2 +-n^2); ORDER 0 = XCD-chunked block order, 1 = plain blockIdx order;
// PAIR 1 = lane per row pair with 16-byte loads, 0 = lane per row with 8-byte loads.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));       \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

typedef double dbl2 __attribute__((ext_vector_type(2)));
typedef double dbl2u __attribute__((ext_vector_type(2), aligned(8)));

__device__ __forceinline__ int64_t xcd_block(int64_t b, int64_t nb) {
  const int64_t q = nb >> 3, r = nb & 7, g = b & 7, i = b >> 3;
  return (g < r ? g * (q + 1) : r * (q + 1) + (g - r) * q) + i;
}

__global__ __launch_bounds__(256) void k_copy(const double* __restrict__ x, double* __restrict__ y,
                                              int64_t N) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (2 * p + 1 < N) {
    *reinterpret_cast<dbl2*>(y + 2 * p) = *reinterpret_cast<const dbl2*>(x + 2 * p);
  }
}

// lane per row pair, every neighbour load 16 B (interior pairs; boundary pairs read clamped)
template <int MASK, int ORDER>
__global__ __launch_bounds__(256) void k_pair(const double* __restrict__ x, double* __restrict__ y,
                                              int n, int64_t N) {
  const int64_t lb = ORDER == 0 ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
  const int64_t p = lb * 256 + threadIdx.x;
  const int64_t r = 2 * p;
  if (r + 1 >= N) return;
  const int64_t n2 = (int64_t)n * n;
  const double* xr = x + r;
  dbl2 c = *reinterpret_cast<const dbl2u*>(xr);
  double s0 = 6.0 * c.x, s1 = 6.0 * c.y;
  auto nb = [&](int64_t off) {
    if (r + off >= 0 && r + off + 1 < N) {
      const dbl2 t = *reinterpret_cast<const dbl2u*>(xr + off);
      s0 -= t.x;
      s1 -= t.y;
    }
  };
  if (MASK & 1) {
    nb(-1);
    nb(1);
  }
  if (MASK & 2) {
    nb(-n);
    nb(n);
  }
  if (MASK & 4) {
    nb(-n2);
    nb(n2);
  }
  dbl2 o;
  o.x = s0;
  o.y = s1;
  *reinterpret_cast<dbl2*>(y + r) = o;
}

// as k_pair<7> but the +-1 neighbours come from the adjacent lanes' centre loads (DPP/bpermute
// shuffles); only the wave's edge lanes load them (8 B). 5 x loads of 16 B per pair instead of 7.
template <int ORDER>
__global__ __launch_bounds__(256) void k_pair_shfl(const double* __restrict__ x,
                                                   double* __restrict__ y, int n, int64_t N) {
  const int64_t lb = ORDER == 0 ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
  const int64_t p = lb * 256 + threadIdx.x;
  const int64_t r = 2 * p;
  const bool live = r + 1 < N;
  const int64_t n2 = (int64_t)n * n;
  const int lane = threadIdx.x & 63;
  dbl2 c = live ? *reinterpret_cast<const dbl2*>(x + r) : dbl2{0.0, 0.0};
  double prev = __shfl_up(c.y, 1, 64);
  double next = __shfl_down(c.x, 1, 64);
  if (lane == 0) prev = (live && r > 0) ? x[r - 1] : 0.0;
  if (lane == 63) next = (live && r + 2 < N) ? x[r + 2] : 0.0;
  if (!live) return;
  double s0 = 6.0 * c.x, s1 = 6.0 * c.y;
  s0 -= prev;
  s1 -= c.x;
  s0 -= c.y;
  s1 -= next;
  auto nb = [&](int64_t off) {
    if (r + off >= 0 && r + off + 1 < N) {
      const dbl2 t = *reinterpret_cast<const dbl2u*>(x + r + off);
      s0 -= t.x;
      s1 -= t.y;
    }
  };
  nb(-n);
  nb(n);
  nb(-n2);
  nb(n2);
  dbl2 o;
  o.x = s0;
  o.y = s1;
  *reinterpret_cast<dbl2*>(y + r) = o;
}

// lane per row, 8-byte loads
template <int MASK, int ORDER>
__global__ __launch_bounds__(256) void k_row(const double* __restrict__ x, double* __restrict__ y,
                                             int n, int64_t N) {
  const int64_t lb = ORDER == 0 ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
  const int64_t r = lb * 256 + threadIdx.x;
  if (r >= N) return;
  const int64_t n2 = (int64_t)n * n;
  double s = 6.0 * x[r];
  auto nb = [&](int64_t off) {
    if (r + off >= 0 && r + off < N) s -= x[r + off];
  };
  if (MASK & 1) {
    nb(-1);
    nb(1);
  }
  if (MASK & 2) {
    nb(-n);
    nb(n);
  }
  if (MASK & 4) {
    nb(-n2);
    nb(n2);
  }
  y[r] = s;
}

// k_pair<7,0> plus the row-pair kernel's indirections: V=1 a pattern-id byte load feeding the
// offsets (pid is all zero here), V=2 also the offsets from an LDS table indexed by the id
template <int V>
__global__ __launch_bounds__(256) void k_pair_ind(const double* __restrict__ x,
                                                  double* __restrict__ y,
                                                  const uint8_t* __restrict__ pid, int n,
                                                  int64_t N) {
  __shared__ int offt[8];
  const int64_t lb = xcd_block(blockIdx.x, gridDim.x);
  const int64_t p = lb * 256 + threadIdx.x;
  const int64_t r = 2 * p;
  const int64_t n2 = (int64_t)n * n;
  if (V == 2) {
    if (threadIdx.x < 8) {
      const int o[8] = {(int)-n2, -n, -1, 0, 1, n, (int)n2, 0};
      offt[threadIdx.x] = o[threadIdx.x];
    }
    __syncthreads();
  }
  if (r + 1 >= N) return;
  const int id = pid[p];
  const double* xr = x + r + id;
  double s0 = 0.0, s1 = 0.0;
  const int o[7] = {(int)-n2, -n, -1, 0, 1, n, (int)n2};
#pragma unroll
  for (int q = 0; q < 7; ++q) {
    const int off = V == 2 ? offt[id * 8 + q] : o[q];
    if (r + off >= 0 && r + off + 1 < N) {
      const dbl2 t = *reinterpret_cast<const dbl2u*>(xr + off);
      s0 += (q == 3 ? 6.0 : -1.0) * t.x;
      s1 += (q == 3 ? 6.0 : -1.0) * t.y;
    }
  }
  dbl2 out;
  out.x = s0;
  out.y = s1;
  *reinterpret_cast<dbl2*>(y + r) = out;
}

// LDS row window: a workgroup owns CH * 512 consecutive rows and stages x over them plus a
// halo of H >= n rows on each side with 16-byte loads (one fetch per element + 2H), so the
// in-plane neighbours (+-1, +-n) come from LDS; the +-n^2 neighbours are global 16-byte loads
// issued before the window is staged. TA instructions per 64 pairs: ~1.2 (window) + 2 (z) + 1
// (store) instead of 7 + 1.
template <int CH, int ZP>
__global__ __launch_bounds__(256) void k_pair_tile(const double* __restrict__ x,
                                                   double* __restrict__ y, int n, int64_t N) {
  extern __shared__ dbl2 win[];
  const int64_t lb = xcd_block(blockIdx.x, gridDim.x);
  const int H = (n + 1) & ~1;
  const int64_t R0 = lb * CH * 512;
  const int64_t T0 = R0 - H;
  const int wlen = (CH * 512 + 2 * H) / 2;  // dbl2 slots
  const int64_t n2 = (int64_t)n * n;
  dbl2 zm[CH], zp[CH];
  auto zload = [&]() {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int64_t r = R0 + 2 * (c * 256 + threadIdx.x);
      zm[c] = (r - n2 >= 0 && r + 1 < N) ? *reinterpret_cast<const dbl2u*>(x + r - n2) : dbl2{0.0, 0.0};
      zp[c] = (r + n2 + 1 < N) ? *reinterpret_cast<const dbl2u*>(x + r + n2) : dbl2{0.0, 0.0};
    }
  };
  if (ZP) zload();
  for (int i = threadIdx.x; i < wlen; i += 256) {
    const int64_t g = T0 + 2 * i;
    win[i] = (g >= 0 && g + 1 < N) ? *reinterpret_cast<const dbl2u*>(x + g) : dbl2{0.0, 0.0};
  }
  __syncthreads();
  if (!ZP) zload();
  const double* w = reinterpret_cast<const double*>(win);
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int64_t r = R0 + 2 * (c * 256 + threadIdx.x);
    if (r + 1 >= N) break;
    const int l = (int)(r - T0);
    const double c0 = w[l], c1 = w[l + 1];
    double s0 = 6.0 * c0, s1 = 6.0 * c1;
    s0 -= w[l - 1];
    s1 -= c0;
    s0 -= c1;
    s1 -= w[l + 2];
    s0 -= w[l - n];
    s1 -= w[l + 1 - n];
    s0 -= w[l + n];
    s1 -= w[l + 1 + n];
    s0 -= zm[c].x;
    s1 -= zm[c].y;
    s0 -= zp[c].x;
    s1 -= zp[c].y;
    dbl2 o;
    o.x = s0;
    o.y = s1;
    *reinterpret_cast<dbl2*>(y + r) = o;
  }
}

template <class F>
static float timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1000.f / reps;
}

template <int MASK, int ORDER>
static void run_pair(const double* x, double* y, int n, int64_t N, int reps) {
  const unsigned nb = (unsigned)((N / 2 + 255) / 256);
  float us = timeit([&] { hipLaunchKernelGGL((k_pair<MASK, ORDER>), dim3(nb), dim3(256), 0, 0, x, y, n, N); }, reps);
  printf("pair mask=%d order=%d: %7.1f us  %6.0f GB/s (x+y)\n", MASK, ORDER, us, 16.0 * N / us / 1e3);
}

template <int MASK, int ORDER>
static void run_row(const double* x, double* y, int n, int64_t N, int reps) {
  const unsigned nb = (unsigned)((N + 255) / 256);
  float us = timeit([&] { hipLaunchKernelGGL((k_row<MASK, ORDER>), dim3(nb), dim3(256), 0, 0, x, y, n, N); }, reps);
  printf("row  mask=%d order=%d: %7.1f us  %6.0f GB/s (x+y)\n", MASK, ORDER, us, 16.0 * N / us / 1e3);
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 216;
  const int reps = argc > 2 ? atoi(argv[2]) : 50;
  const int64_t N = (int64_t)n * n * n;
  double *x, *y;
  CK(hipMalloc(&x, sizeof(double) * N));
  CK(hipMalloc(&y, sizeof(double) * N));
  std::vector<double> h(N);
  for (int64_t i = 0; i < N; ++i) h[i] = (double)((i * 2654435761u) % 1000) / 1000.0;
  CK(hipMemcpy(x, h.data(), sizeof(double) * N, hipMemcpyHostToDevice));
  {
    const unsigned nb = (unsigned)((N / 2 + 255) / 256);
    float us = timeit([&] { hipLaunchKernelGGL(k_copy, dim3(nb), dim3(256), 0, 0, x, y, N); }, reps);
    printf("copy 16B/lane     : %7.1f us  %6.0f GB/s\n", us, 16.0 * N / us / 1e3);
  }
  run_pair<0, 0>(x, y, n, N, reps);
  run_pair<1, 0>(x, y, n, N, reps);
  run_pair<2, 0>(x, y, n, N, reps);
  run_pair<4, 0>(x, y, n, N, reps);
  run_pair<7, 0>(x, y, n, N, reps);
  run_pair<7, 1>(x, y, n, N, reps);
  {
    const unsigned nb = (unsigned)((N / 2 + 255) / 256);
    float us = timeit([&] { hipLaunchKernelGGL((k_pair_shfl<0>), dim3(nb), dim3(256), 0, 0, x, y, n, N); }, reps);
    printf("pair shfl +-1       : %7.1f us  %6.0f GB/s (x+y)\n", us, 16.0 * N / us / 1e3);
  }
  {
    uint8_t* pid;
    CK(hipMalloc(&pid, N / 2 + 1));
    CK(hipMemset(pid, 0, N / 2 + 1));
    const unsigned nb = (unsigned)((N / 2 + 255) / 256);
    float us1 = timeit([&] { hipLaunchKernelGGL((k_pair_ind<1>), dim3(nb), dim3(256), 0, 0, x, y, pid, n, N); }, reps);
    float us2 = timeit([&] { hipLaunchKernelGGL((k_pair_ind<2>), dim3(nb), dim3(256), 0, 0, x, y, pid, n, N); }, reps);
    printf("pair + pid load      : %7.1f us\npair + pid + LDS offs: %7.1f us\n", us1, us2);
  }
  for (int ch : {1, 2, 4, 11, 12}) {
    const int H = (n + 1) & ~1;
    const unsigned nb = (unsigned)((N + ch * 512 - 1) / (ch * 512));
    const size_t lds = sizeof(double) * (ch * 512 + 2 * H);
    const int c2 = ch % 10;  // 11, 12: CH 1, 2 with the z loads after the barrier
    const unsigned nb2 = (unsigned)((N + c2 * 512 - 1) / (c2 * 512));
    const size_t lds2 = sizeof(double) * (c2 * 512 + 2 * H);
    float us = timeit([&] {
      if (ch == 1) hipLaunchKernelGGL((k_pair_tile<1, 1>), dim3(nb), dim3(256), lds, 0, x, y, n, N);
      if (ch == 2) hipLaunchKernelGGL((k_pair_tile<2, 1>), dim3(nb), dim3(256), lds, 0, x, y, n, N);
      if (ch == 4) hipLaunchKernelGGL((k_pair_tile<4, 1>), dim3(nb), dim3(256), lds, 0, x, y, n, N);
      if (ch == 11) hipLaunchKernelGGL((k_pair_tile<1, 0>), dim3(nb2), dim3(256), lds2, 0, x, y, n, N);
      if (ch == 12) hipLaunchKernelGGL((k_pair_tile<2, 0>), dim3(nb2), dim3(256), lds2, 0, x, y, n, N);
    }, reps);
    printf("pair LDS window CH=%d: %7.1f us  %6.0f GB/s (x+y)\n", ch, us, 16.0 * N / us / 1e3);
  }
  run_row<0, 0>(x, y, n, N, reps);
  run_row<7, 0>(x, y, n, N, reps);
  run_row<7, 1>(x, y, n, N, reps);
  return 0;
}
