// Micro-benchmark (diagnostic, not part of the library): cost of one workgroup step of the
// batched small-problem solver (csrc/batch.hip) — a barrier plus an LDS gather — for
// __syncthreads() vs a bare s_barrier, at 256 / 1024 threads, and a dependent global load chain.
// Build: hipcc --offload-arch=gfx950 -O3 tools/barrier_lab.hip -o tools/barrier_lab.bin
#include <hip/hip_runtime.h>
#include <cstdio>

template <int NT, bool FULL>
__global__ __launch_bounds__(NT) void k_steps(double* out, int steps) {
  __shared__ double x[4096];
  for (int i = threadIdx.x; i < 4096; i += NT) x[i] = i;
  __syncthreads();
  double acc = 0.0;
  for (int s = 0; s < steps; ++s) {
    const int idx = (threadIdx.x * 7 + s * 13) & 4095;
    acc += x[idx];
    if (threadIdx.x < 64) x[(threadIdx.x + s) & 4095] = acc;
    if (FULL) __syncthreads();
    else __builtin_amdgcn_s_barrier();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = acc;
}

__global__ void k_chain(const int* __restrict__ next, int steps, int* out) {
  int p = threadIdx.x;
  for (int s = 0; s < steps; ++s) p = next[p];
  if (threadIdx.x == 0) out[blockIdx.x] = p;
}

template <class F>
float time_ms(F f) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  f();
  hipDeviceSynchronize();
  hipEventRecord(a);
  f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main() {
  double* out;
  hipMalloc(&out, 1024 * sizeof(double));
  const int steps = 20000;
  for (int blocks : {1, 48}) {
    float t1 = time_ms([&] { k_steps<1024, true><<<blocks, 1024>>>(out, steps); });
    float t2 = time_ms([&] { k_steps<1024, false><<<blocks, 1024>>>(out, steps); });
    float t3 = time_ms([&] { k_steps<256, true><<<blocks, 256>>>(out, steps); });
    float t4 = time_ms([&] { k_steps<256, false><<<blocks, 256>>>(out, steps); });
    printf("blocks %d: per step  1024 thr __syncthreads %.1f ns, s_barrier %.1f ns;  256 thr "
           "__syncthreads %.1f ns, s_barrier %.1f ns\n",
           blocks, t1 * 1e6 / steps, t2 * 1e6 / steps, t3 * 1e6 / steps, t4 * 1e6 / steps);
  }
  // dependent global load chain: L2-resident (64 KB) and HBM-sized (512 MB)
  for (size_t n : {size_t(16384), size_t(128) << 20}) {
    int* next;
    hipMalloc(&next, n * sizeof(int));
    int* h = (int*)malloc(n * sizeof(int));
    for (size_t i = 0; i < n; ++i) h[i] = (int)((i * 2654435761ull + 12345) % n);
    hipMemcpy(next, h, n * sizeof(int), hipMemcpyHostToDevice);
    int* o;
    hipMalloc(&o, 64 * sizeof(int));
    const int cs = 4000;
    float t = time_ms([&] { k_chain<<<1, 64>>>(next, cs, o); });
    printf("dependent load chain over %zu KB: %.1f ns per load\n", n * 4 / 1024, t * 1e6 / cs);
    hipFree(next);
    hipFree(o);
    free(h);
  }
  return 0;
}
