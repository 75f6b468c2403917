// Latency of one dependent step of a wave-level substitution chain, by broadcast primitive:
//   valu:     s = s - c * s                      (fp64 multiply + subtract, no broadcast)
//   readlane: s = s - c * readlane(s, j & 63)   (two v_readlane_b32 to SGPRs)
//   shfl:     s = s - c * __shfl(s, j & 63)     (ds_bpermute through the LDS crossbar)
//   lds:      owner writes s to LDS, wave reads it back
// hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/bcast_lab.hip -o tools/bcast_lab
#include <hip/hip_runtime.h>
#include <cstdio>
__device__ __forceinline__ double readlane_d(double v, int l) {
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)x, l);
  const int hi = __builtin_amdgcn_readlane((int)(x >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
template <int MODE>
__global__ void k(double* out, long long* t, int steps, double c) {
  __shared__ double sh[64];
  const int lane = threadIdx.x;
  double s = 1.0 + lane * 1e-3;
  const long long t0 = wall_clock64();
  for (int j = 0; j < steps; ++j) {
    double v;
    if (MODE == 0) v = s;
    else if (MODE == 1) v = readlane_d(s, j & 63);
    else if (MODE == 2) v = __shfl(s, j & 63, 64);
    else {
      if (lane == (j & 63)) sh[0] = s;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      v = sh[0];
    }
    s = s - c * v;
  }
  const long long t1 = wall_clock64();
  out[lane] = s;
  if (lane == 0) t[0] = t1 - t0;
}
int main() {
  double* o; long long* t; hipMalloc(&o, 512); hipMalloc(&t, 8);
  const int steps = 100000;
  const char* names[4] = {"valu", "readlane", "shfl", "lds"};
  for (int m = 0; m < 4; ++m) {
    for (int w = 0; w < 2; ++w) {
      if (m == 0) hipLaunchKernelGGL(k<0>, 1, 64, 0, 0, o, t, steps, 1e-9);
      if (m == 1) hipLaunchKernelGGL(k<1>, 1, 64, 0, 0, o, t, steps, 1e-9);
      if (m == 2) hipLaunchKernelGGL(k<2>, 1, 64, 0, 0, o, t, steps, 1e-9);
      if (m == 3) hipLaunchKernelGGL(k<3>, 1, 64, 0, 0, o, t, steps, 1e-9);
      hipDeviceSynchronize();
    }
    long long h; hipMemcpy(&h, t, 8, hipMemcpyDeviceToHost);
    printf("%-9s %.1f ns per step\n", names[m], h * 10.0 / steps);
  }
  return 0;
}
