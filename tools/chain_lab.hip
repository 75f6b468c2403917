// Micro-benchmark (diagnostic, not part of the library): cost per element of a left-to-right
// fp64 sum (scipy's csr_matvec order) by one lane — the phase-2 chain of the LDS-staged SpMV
// kernels — from registers, from LDS with U reads issued before the adds, and with many lanes
// summing their own rows at once.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/chain_lab.hip -o tools/chain_lab.bin
#include <hip/hip_runtime.h>
#include <cstdio>

// register-only dependent chain: s = s + v, n times
__global__ void k_reg(double* out, int n, double v) {
  double s = 0.0, w = v;
  for (int i = 0; i < n; ++i) {
    s += w;
    w = w * 1.0000001;  // independent of s: keeps the add's operand non-constant
  }
  out[threadIdx.x] = s;
}

// LDS chain with U entries read ahead of their adds (one batch per iteration); lanes < active
// sum their own row (row r at offset r * len + skew) of length len
template <int U>
__global__ __launch_bounds__(256) void k_lds(double* out, int len, int active, int reps,
                                             long long* cyc) {
  __shared__ double p[4096];
  for (int i = threadIdx.x; i < 4096; i += 256) p[i] = 1.0 + i * 1e-9;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  double s = 0.0;
  long long t0 = clock64();
  if (lane < active) {
    const int base = ((lane + wave * active) * len + lane * 3) & 2047;
    for (int r = 0; r < reps; ++r) {
      int k = base;
      const int kb = base + len;
      for (; k + U <= kb; k += U) {
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = p[k + u];
#pragma unroll
        for (int u = 0; u < U; ++u) s += v[u];
      }
      for (; k < kb; ++k) s += p[k];
    }
  }
  long long t1 = clock64();
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  double* out;
  long long* cyc;
  hipMalloc(&out, 4096 * sizeof(double));
  hipMalloc(&cyc, 4096 * sizeof(long long));
  long long h[1];
  // registers
  {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int n = 1 << 20;
    k_reg<<<1, 64>>>(out, n, 1.0);
    hipDeviceSynchronize();
    hipEventRecord(a);
    k_reg<<<1, 64>>>(out, n, 1.0);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("register chain: %.2f ns per dependent v_add_f64 (+ one independent mul)\n",
           ms * 1e6 / n);
  }
  const int len = 1000, reps = 20;
  for (int active : {1, 16, 64}) {
    for (int blocks : {1, 256, 1024}) {
#define RUN(U)                                                                          \
  {                                                                                     \
    k_lds<U><<<blocks, 256>>>(out, len, active, reps, cyc);                             \
    hipDeviceSynchronize();                                                             \
    k_lds<U><<<blocks, 256>>>(out, len, active, reps, cyc);                             \
    hipMemcpy(h, cyc, sizeof(long long), hipMemcpyDeviceToHost);                        \
    printf("LDS chain U=%2d active lanes/wave %2d blocks %4d: %.1f cycles per element\n", U, \
           active, blocks, (double)h[0] / (len * reps));                                \
  }
      RUN(1) RUN(4) RUN(8) RUN(16) RUN(32)
    }
  }
  return 0;
}
