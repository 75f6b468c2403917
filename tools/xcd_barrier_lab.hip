// Micro-benchmark (diagnostic, not part of the library; VERDICT r05 Next #2b): what an in-kernel
// barrier among the few workgroups of a coarse-level V-cycle tail costs on MI355X, against the
// dependent kernel boundary it would replace.
//   boundary  : S dependent launches of an empty 32-workgroup kernel, per launch (stream, graph)
//   barrier   : S barriers inside one launch of N workgroups (lane 0: agent-scope relaxed atomic
//               add on one counter, then an sc1-load poll until all N arrived; the rest of the
//               workgroup waits at __syncthreads), per barrier; N = 8, 32, 256
//   same-XCD  : N = 8 / 32 participants taken as the blocks b with b % 8 == 0 of an 8N-block
//               grid (the dispatcher deals blocks round-robin over the 8 XCDs), the others exit
//               at once; the XCC id of every participant is read (s_getreg HW_REG_XCC_ID) and
//               the run reports whether they shared one XCD
// Build: hipcc --offload-arch=gfx950 -O3 tools/xcd_barrier_lab.hip -o tools/xcd_barrier_lab.bin
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                        \
    }                                                                                  \
  } while (0)

__global__ void k_empty(int* sink) {
  if (sink && threadIdx.x == 0 && blockIdx.x == 1u << 30) *sink = 1;
}

__device__ __forceinline__ int xcc_id() {
  int v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xf;
}

// stride > 1: only blocks b with b % stride == 0 take part (N = gridDim / stride)
__global__ __launch_bounds__(256) void k_barriers(unsigned* ctr, int steps, int stride,
                                                  int* xcc_out, unsigned long long* spin_out) {
  if (blockIdx.x % stride) return;
  const unsigned n = gridDim.x / stride;
  const int me = blockIdx.x / stride;
  __shared__ unsigned long long spins;
  if (threadIdx.x == 0) {
    spins = 0;
    xcc_out[me] = xcc_id();
  }
  for (int s = 1; s <= steps; ++s) {
    __syncthreads();
    if (threadIdx.x == 0) {
      __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = (unsigned)s * n;
      unsigned long long guard = 0;
      while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++guard > (1ull << 26)) break;  // a lab bound: never spin forever
      }
      spins += guard;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) spin_out[me] = spins;
}

// streaming read of n doubles by the participating blocks (b % stride == 0), 16-B loads, one
// partial sum per block (so nothing is optimised away)
__global__ __launch_bounds__(256) void k_read(const double2* __restrict__ p, int64_t n2,
                                              int stride, double* out) {
  if (blockIdx.x % stride) return;
  const int64_t nb = gridDim.x / stride, me = blockIdx.x / stride;
  double s = 0.0;
  for (int64_t i = me * 256 + threadIdx.x; i < n2; i += nb * 256) {
    const double2 v = p[i];
    s += v.x + v.y;
  }
  if (s == 1.2345) out[me] = s;
}

template <class F>
static float time_ms(F f, int reps, hipStream_t st) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  f();
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a, st);  // on the stream the work goes to (a non-blocking one)
  for (int r = 0; r < reps; ++r) f();
  (void)hipEventRecord(b, st);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return ms / reps;
}

int main() {
  const int S = 200;
  unsigned* ctr;
  int* xcc;
  unsigned long long* spin;
  CK(hipMalloc(&ctr, sizeof(unsigned)));
  CK(hipMalloc(&xcc, sizeof(int) * 2048));
  CK(hipMalloc(&spin, sizeof(unsigned long long) * 2048));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  // 1. dependent kernel boundaries
  const float t_stream = time_ms([&] {
    for (int s = 0; s < S; ++s) hipLaunchKernelGGL(k_empty, dim3(32), dim3(256), 0, st, nullptr);
  }, 5, st);
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  for (int s = 0; s < S; ++s) hipLaunchKernelGGL(k_empty, dim3(32), dim3(256), 0, st, nullptr);
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  const float t_graph = time_ms([&] { (void)hipGraphLaunch(ge, st); }, 5, st);
  std::printf("{\"boundary_us_stream\": %.3f, \"boundary_us_graph\": %.3f", 1e3f * t_stream / S,
              1e3f * t_graph / S);
  // 2. in-kernel barriers
  struct Cfg {
    const char* name;
    int n, stride;
  } cfgs[] = {{"spread_8", 8, 1},   {"spread_32", 32, 1},  {"spread_256", 256, 1},
              {"samexcd_8", 8, 8},  {"samexcd_32", 32, 8}};
  for (const Cfg& c : cfgs) {
    auto run = [&](int steps) {
      (void)hipMemsetAsync(ctr, 0, sizeof(unsigned), st);
      hipLaunchKernelGGL(k_barriers, dim3(c.n * c.stride), dim3(256), 0, st, ctr, steps,
                         c.stride, xcc, spin);
    };
    const float t0 = time_ms([&] { run(0); }, 10, st);
    const float t1 = time_ms([&] { run(S); }, 10, st);
    CK(hipGetLastError());
    CK(hipStreamSynchronize(st));
    std::vector<int> h(c.n);
    std::vector<unsigned long long> sp(c.n);
    CK(hipMemcpy(h.data(), xcc, sizeof(int) * c.n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(sp.data(), spin, sizeof(unsigned long long) * c.n, hipMemcpyDeviceToHost));
    int same = 1, timeouts = 0;
    for (int i = 0; i < c.n; ++i) {
      same &= h[i] == h[0];
      timeouts += sp[i] > (1ull << 26) * (unsigned long long)S / 2;
    }
    std::printf(", \"barrier_us_%s\": %.3f, \"one_xcd_%s\": %s", c.name, 1e3f * (t1 - t0) / S,
                c.name, same ? "true" : "false");
    if (timeouts) std::printf(", \"timeouts_%s\": %d", c.name, timeouts);
  }
  // 3. what one XCD can stream: a coarse tail's working set (the C2 levels >= 2 + dense
  // coarse inverse, ~18 MB, resident in the Infinity Cache across cycles) read by 32 blocks on
  // one XCD vs 256 blocks on all eight, warm (back to back)
  for (int mb : {4, 18, 64}) {
    const int64_t n2 = (int64_t)mb * (1 << 20) / 16;
    double2* buf;
    CK(hipMalloc(&buf, n2 * 16));
    CK(hipMemset(buf, 0, n2 * 16));
    double* out;
    CK(hipMalloc(&out, sizeof(double) * 256));
    const float t_one = time_ms([&] {
      hipLaunchKernelGGL(k_read, dim3(256), dim3(256), 0, st, buf, n2, 8, out);
    }, 20, st);
    const float t_all = time_ms([&] {
      hipLaunchKernelGGL(k_read, dim3(256), dim3(256), 0, st, buf, n2, 1, out);
    }, 20, st);
    CK(hipGetLastError());
    std::printf(", \"read_%dMB_one_xcd_GBps\": %.0f, \"read_%dMB_all_GBps\": %.0f", mb,
                n2 * 16 / (t_one * 1e6), mb, n2 * 16 / (t_all * 1e6));
    CK(hipFree(buf));
    CK(hipFree(out));
  }
  std::printf("}\n");
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipStreamDestroy(st));
  return 0;
}
