// Cold/warm lab for the C4 fine-level stencil pass (216^3 7-point, y = A x with row pairs):
// where do the ~12 us between k_pair_tile (tools/stencil_lab.hip) and k_rowpat_uni go?
// Diagnostics only (no bitwise claims). "cold" = a 512 MB read before each launch.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/stencil_lab2.hip -o /tmp/sl2
//   /tmp/sl2 [n=216] [reps=20]
// Variants of the LDS-window tile (a workgroup owns RW rows, stages x over them +- H rows,
// the +-n^2 operands are 16-byte global loads issued first):
//   NT threads per workgroup, CH row pairs per thread, PID: a pattern-id byte per pair and a
//   16-bit slot mask from an LDS table selecting each product (as k_rowpat_uni does), CL: the
//   window and far loads clamped branch-free (k_rowpat_uni's x16) instead of guarded.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef double dbl2 __attribute__((ext_vector_type(2)));
typedef double dbl2u __attribute__((ext_vector_type(2), aligned(8)));

__device__ __forceinline__ int64_t xcd_block(int64_t b, int64_t nb) {
  const int64_t q = nb >> 3, r = nb & 7, g = b & 7, i = b >> 3;
  return (g < r ? g * (q + 1) : r * (q + 1) + (g - r) * q) + i;
}

// xcd_block, then each XCD's contiguous range dealt to SUB fronts: the XCD's i-th dispatched
// workgroup takes block k = i / SUB of sub-range i % SUB, so its resident workgroups cover SUB
// narrow fronts instead of one wide one (bijective; the remainder blocks come last)
__device__ __forceinline__ int64_t xcd_block_sub(int64_t b, int64_t nb, int sub) {
  const int64_t q = nb >> 3, r = nb & 7, g = b & 7, i = b >> 3;
  const int64_t s0 = g < r ? g * (q + 1) : r * (q + 1) + (g - r) * q;
  const int64_t len = g < r ? q + 1 : q;
  const int64_t ql = len / sub;
  if (i < ql * sub) return s0 + (i % sub) * ql + i / sub;
  return s0 + i;
}

__global__ __launch_bounds__(256) void k_copy(const double* __restrict__ x, double* __restrict__ y,
                                              int64_t N) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (2 * p + 1 < N) *reinterpret_cast<dbl2*>(y + 2 * p) = *reinterpret_cast<const dbl2*>(x + 2 * p);
}

__global__ __launch_bounds__(256) void k_flush(const double* __restrict__ f, double* out, int64_t n) {
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    s += f[i];
  if (s == 1.2345) out[0] = s;
}

__device__ __forceinline__ dbl2 x16c(const double* __restrict__ x, int64_t g, int64_t n) {
  const int64_t gc = g < 0 ? 0 : (g > n - 2 ? n - 2 : g);
  const dbl2 t = *reinterpret_cast<const dbl2u*>(x + gc);
  dbl2 o;
  o.x = g == gc ? t.x : (g == n - 1 ? t.y : 0.0);
  o.y = g == gc ? t.y : (g == -1 ? t.x : 0.0);
  return o;
}
__device__ __forceinline__ dbl2 x16g(const double* __restrict__ x, int64_t g, int64_t n) {
  return (g >= 0 && g + 1 < n) ? *reinterpret_cast<const dbl2u*>(x + g) : dbl2{0.0, 0.0};
}
__device__ __forceinline__ dbl2 x16n(const double* __restrict__ x, int64_t g, int64_t n) {
  if (g >= 0 && g + 1 < n) {
    dbl2 t;
    t.x = __builtin_nontemporal_load(x + g);
    t.y = __builtin_nontemporal_load(x + g + 1);
    return t;
  }
  return dbl2{0.0, 0.0};
}

template <int NT, int CH, bool PID, bool CL, int FAR = 3, int PF = 0, int ORD = 0>
__global__ __launch_bounds__(NT) void k_tile(const double* __restrict__ x, double* __restrict__ y,
                                             const uint8_t* __restrict__ pid,
                                             const uint16_t* __restrict__ pmsk, int n, int64_t N) {
  extern __shared__ dbl2 win[];
  __shared__ uint16_t msk[256];
  const int64_t lb = (ORD == 0 || ORD > 200) ? xcd_block(blockIdx.x, gridDim.x)
                     : ORD > 100               ? xcd_block_sub(blockIdx.x, gridDim.x, ORD - 100)
                                               : blockIdx.x;
  constexpr bool FNT = ORD == 201 || ORD == 203, WNT = ORD == 202 || ORD == 203, YNT = ORD == 204;
  const int H = (n + 1) & ~1;  // halo rows (even)
  const int hw = H / 2;        // halo pairs
  const int64_t P0 = lb * CH * NT;  // first pair
  const int64_t T0 = 2 * P0 - H;    // first window row
  const int nwin = CH * NT + 2 * hw;
  const int64_t n2 = (int64_t)n * n;
  auto ld = [&](int64_t g) { return CL ? x16c(x, g, N) : x16g(x, g, N); };
  dbl2 zm[CH], zp[CH];
  int pc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int64_t p = P0 + c * NT + threadIdx.x;
    pc[c] = PID ? pid[2 * p < N ? p : 0] : 0;
    zm[c] = (FAR & 1) ? (FNT ? x16n(x, 2 * p - n2, N) : ld(2 * p - n2)) : dbl2{0.0, 0.0};
    zp[c] = (FAR & 2) ? (FNT ? x16n(x, 2 * p + n2, N) : ld(2 * p + n2)) : dbl2{0.0, 0.0};
  }
  if (PF > 0) {  // touch the x lines PF workgroups ahead of this one's +n^2 operands
    const int64_t g = 2 * (P0 + (int64_t)PF * CH * NT + threadIdx.x * CH) + n2;
    if (g < N) {
      double v = x[g];
      asm volatile("" ::"v"(v));
    }
  }
  constexpr int WQ = CH + (256 + NT - 1) / NT + 1;
  dbl2 wv[WQ];
#pragma unroll
  for (int q = 0; q < WQ; ++q) {
    const int i = threadIdx.x + q * NT;
    wv[q] = WNT ? x16n(x, T0 + 2 * (int64_t)(i < nwin ? i : 0), N)
                : ld(T0 + 2 * (int64_t)(i < nwin ? i : 0));
  }
#pragma unroll
  for (int q = 0; q < WQ; ++q) {
    const int i = threadIdx.x + q * NT;
    if (i < nwin) win[i] = wv[q];
  }
  if (PID)
    for (int i = threadIdx.x; i < 256; i += NT) msk[i] = pmsk[i];
  __syncthreads();
  const double* w = reinterpret_cast<const double*>(win);
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int64_t p = P0 + c * NT + threadIdx.x;
    const int64_t r = 2 * p;
    if (r + 1 >= N) break;
    const int l = (int)(r - T0);
    const int m = PID ? msk[pc[c]] : 0xffff;
    const double t[7][2] = {{zm[c].x, zm[c].y},           {w[l - n], w[l + 1 - n]},
                            {w[l - 1], w[l]},             {w[l], w[l + 1]},
                            {w[l + 1], w[l + 2]},         {w[l + n], w[l + 1 + n]},
                            {zp[c].x, zp[c].y}};
    const double v[7] = {-1.0, -1.0, -1.0, 6.0, -1.0, -1.0, -1.0};
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int q = 0; q < 7; ++q) {
      s0 += v[q] * (((m >> q) & 1) ? t[q][0] : 0.0);
      s1 += v[q] * (((m >> (q + 8)) & 1) ? t[q][1] : 0.0);
    }
    dbl2 o;
    o.x = s0;
    o.y = s1;
    if (YNT)
      __builtin_nontemporal_store(o, reinterpret_cast<dbl2*>(y + r));
    else
      *reinterpret_cast<dbl2*>(y + r) = o;
  }
}

struct Timer {
  const double* f;
  double* sink;
  int64_t nf;
  template <class F>
  void run(const char* name, F fn, double mb, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    fn();
    CK(hipDeviceSynchronize());
    double cold = 0.0;
    for (int i = 0; i < reps; ++i) {
      hipLaunchKernelGGL(k_flush, dim3(4096), dim3(256), 0, 0, f, sink, nf);
      CK(hipEventRecord(a));
      fn();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      cold += ms * 1e3 / reps;
    }
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) fn();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    const double warm = ms * 1e3 / reps;
    printf("%-34s cold %7.2f us (%5.0f GB/s)  warm %7.2f us (%5.0f GB/s)\n", name, cold,
           mb * 1e3 / cold, warm, mb * 1e3 / warm);
    fflush(stdout);
  }
};

template <int NT, int CH, bool PID, bool CL, int FAR = 3, int PF = 0, int ORD = 0>
static void run_tile(Timer& T, const double* x, double* y, const uint8_t* pid, const uint16_t* pm,
                     int n, int64_t N, int reps) {
  const int64_t pairs = N / 2;
  const unsigned nb = (unsigned)((pairs + CH * NT - 1) / (CH * NT));
  const int H = (n + 1) & ~1;
  const size_t lds = sizeof(dbl2) * (CH * NT + H);
  char name[96];
  snprintf(name, sizeof name, "tile NT=%d CH=%d pid=%d cl=%d far=%d pf=%d ord=%d", NT, CH, (int)PID,
           (int)CL, FAR, PF, ORD);
  T.run(name, [&] {
    hipLaunchKernelGGL((k_tile<NT, CH, PID, CL, FAR, PF, ORD>), dim3(nb), dim3(NT), lds, 0, x, y,
                       pid, pm, n, N);
  }, 16.0 * N / 1e6, reps);
}

// 2.5-D march with the far operands in registers: a workgroup owns a tile of T = 2 CH NT rows of
// a plane (tile j of every plane) and marches it through planes k0 .. k1 - 1. Each thread holds
// its own pairs of the tile (CH 16-byte slots) for planes k - 1 (far -), k (centre) and k + 1
// (far +), and the in-plane halo (+-H rows) of plane k + 1 sits in the first hw threads; the LDS
// window holds plane k only (for the +-1 / +-n neighbours). Per step: window k + 2 goes out, plane
// k is summed, window k + 1 is stored after a barrier. x is read once per plane (+ halo, + two
// planes per segment); there are no far loads.
template <int NT, int CH, int S>
__global__ __launch_bounds__(NT) void k_march2(const double* __restrict__ x, double* __restrict__ y,
                                               int n, int64_t N, int nt) {
  extern __shared__ dbl2 win[];
  const int64_t lb = xcd_block(blockIdx.x, gridDim.x);
  const int j = (int)(lb % nt);
  const int64_t k0 = (lb / nt) * S;
  const int64_t k1 = k0 + S < n ? k0 + S : n;
  const int64_t F = (int64_t)n * n;
  const int H = (n + 1) & ~1;
  const int hw = H / 2;
  constexpr int T = 2 * CH * NT;
  const int64_t t0 = (int64_t)j * T;  // first row of the tile within a plane
  const int tid = threadIdx.x;
  struct Win {
    dbl2 t[CH];
    dbl2 hl, hr;
  };
  auto wload = [&](Win& w, int64_t k) {
    const int64_t r0 = k * F + t0;  // tile row 0 of plane k
#pragma unroll
    for (int c = 0; c < CH; ++c) w.t[c] = x16c(x, r0 + 2 * (int64_t)(c * NT + tid), N);
    const bool h = tid < hw;
    w.hl = x16c(x, r0 - H + 2 * (int64_t)(h ? tid : 0), N);
    w.hr = x16c(x, r0 + T + 2 * (int64_t)(h ? tid : 0), N);
  };
  auto wstore = [&](const Win& w) {
#pragma unroll
    for (int c = 0; c < CH; ++c) win[hw + c * NT + tid] = w.t[c];
    if (tid < hw) {
      win[tid] = w.hl;
      win[hw + CH * NT + tid] = w.hr;
    }
  };
  Win wm, wc, wn, wnn;
  wload(wm, k0 - 1);
  wload(wc, k0);
  wload(wn, k0 + 1);
  wstore(wc);
  __syncthreads();
  const double* w = reinterpret_cast<const double*>(win);
  for (int64_t k = k0; k < k1; ++k) {
    if (k + 2 <= k1) wload(wnn, k + 2);
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int lp = 2 * (c * NT + tid);  // row within the tile
      const int64_t r = k * F + t0 + lp;
      if (t0 + lp >= F || r + 1 >= N) continue;
      const int l = H + lp;
      const double t[7][2] = {{wm.t[c].x, wm.t[c].y},     {w[l - n], w[l + 1 - n]},
                              {w[l - 1], wc.t[c].x},       {wc.t[c].x, wc.t[c].y},
                              {wc.t[c].y, w[l + 2]},       {w[l + n], w[l + 1 + n]},
                              {wn.t[c].x, wn.t[c].y}};
      const double v[7] = {-1.0, -1.0, -1.0, 6.0, -1.0, -1.0, -1.0};
      double s0 = 0.0, s1 = 0.0;
#pragma unroll
      for (int q = 0; q < 7; ++q) {
        s0 += v[q] * t[q][0];
        s1 += v[q] * t[q][1];
      }
      dbl2 o;
      o.x = s0;
      o.y = s1;
      *reinterpret_cast<dbl2*>(y + r) = o;
    }
    __syncthreads();
    wstore(wn);
    __syncthreads();
    wm = wc;
    wc = wn;
    wn = wnn;
  }
}

template <int NT, int CH, int S>
static void run_march2(Timer& T, const double* x, double* y, int n, int64_t N, int reps) {
  const int64_t F = (int64_t)n * n;
  const int Tr = 2 * CH * NT;
  const int nt = (int)((F + Tr - 1) / Tr);
  const unsigned nb = (unsigned)(nt * ((n + S - 1) / S));
  const int H = (n + 1) & ~1;
  const size_t lds = sizeof(dbl2) * (CH * NT + H);
  char name[96];
  snprintf(name, sizeof name, "march2 NT=%d CH=%d S=%d (%u wg)", NT, CH, S, nb);
  T.run(name, [&] {
    hipLaunchKernelGGL((k_march2<NT, CH, S>), dim3(nb), dim3(NT), lds, 0, x, y, n, N, nt);
  }, 16.0 * N / 1e6, reps);
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 216;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const int64_t N = (int64_t)n * n * n;
  double *x, *y, *f, *sink;
  uint8_t* pid;
  uint16_t* pm;
  const int64_t nf = 64ll << 20;  // 512 MB
  CK(hipMalloc(&x, sizeof(double) * N));
  CK(hipMalloc(&y, sizeof(double) * N));
  CK(hipMalloc(&f, sizeof(double) * nf));
  CK(hipMalloc(&sink, 8));
  CK(hipMalloc(&pid, N / 2 + 1));
  CK(hipMalloc(&pm, 512));
  CK(hipMemset(f, 0, sizeof(double) * nf));
  CK(hipMemset(pid, 0, N / 2 + 1));
  std::vector<uint16_t> hm(256, 0xffff);
  CK(hipMemcpy(pm, hm.data(), 512, hipMemcpyHostToDevice));
  std::vector<double> h(N);
  for (int64_t i = 0; i < N; ++i) h[i] = (double)((i * 2654435761u) % 1000) / 1000.0;
  CK(hipMemcpy(x, h.data(), sizeof(double) * N, hipMemcpyHostToDevice));
  Timer T{f, sink, nf};
  T.run("copy 16B/lane", [&] {
    hipLaunchKernelGGL(k_copy, dim3((unsigned)((N / 2 + 255) / 256)), dim3(256), 0, 0, x, y, N);
  }, 16.0 * N / 1e6, reps);
  run_tile<256, 2, false, false>(T, x, y, pid, pm, n, N, reps);
  run_tile<256, 2, false, false, 3, 0, 201>(T, x, y, pid, pm, n, N, reps);
  run_tile<256, 2, false, false, 3, 0, 202>(T, x, y, pid, pm, n, N, reps);
  run_tile<256, 2, false, false, 3, 0, 203>(T, x, y, pid, pm, n, N, reps);
  run_tile<256, 2, false, false, 3, 0, 204>(T, x, y, pid, pm, n, N, reps);
  run_tile<256, 2, false, false>(T, x, y, pid, pm, n, N, reps);
  return 0;
}
