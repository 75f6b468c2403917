// Seed selection of the reference's aggregation: `np.random.RandomState(seed).permutation(n)[:k]`
// (ns/lib/graph.py:230-231, utils/evaluate_dataset.py:80-85), bit for bit.
//
// numpy's legacy RandomState.permutation(n) is a Fisher-Yates shuffle of arange(n): for
// i = n-1 .. 1, j_i = random_interval(i) (32-bit MT19937 draws masked to the smallest all-ones
// mask >= i, redrawn while > i), swap(a[i], a[j_i]). On the host that is n swaps at random
// addresses of an 80 MB array (~1 s at n = 10 M). Here only the draws stay on the host (one
// sequential MT19937 stream, ~n draws), and the first k entries of the result are evaluated on
// the device from them: position p ends up holding the index reached by following p through the
// transpositions in order — at step i a tracked position q moves to j_i if q == i, to i if
// q == j_i (i > q then), else stays — so each thread walks only the steps that touch its position:
// q's own step and the steps whose j_i == q (a sorted list per q, the transpose of the (i, j_i)
// map), a few per position.
#include "common.hpp"

#include <vector>

namespace mlamg {

// MT19937 with numpy's legacy seeding (mt19937_seed = init_genrand)
struct Mt19937 {
  uint32_t mt[624];
  int idx = 624;
  explicit Mt19937(uint32_t seed) {
    mt[0] = seed;
    for (int i = 1; i < 624; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
  }
  void twist() {
    for (int k = 0; k < 624; ++k) {
      const uint32_t y = (mt[k] & 0x80000000u) | (mt[(k + 1) % 624] & 0x7fffffffu);
      mt[k] = mt[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    idx = 0;
  }
  uint32_t next() {
    if (idx >= 624) twist();
    uint32_t y = mt[idx++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }
  // numpy random_interval(max) for max < 2^32
  uint32_t interval(uint32_t max) {
    if (max == 0) return 0;
    uint32_t mask = max;
    mask |= mask >> 1;
    mask |= mask >> 2;
    mask |= mask >> 4;
    mask |= mask >> 8;
    mask |= mask >> 16;
    uint32_t v;
    while ((v = next() & mask) > max) {
    }
    return v;
  }
};

// out[p] for p < k: follow position p through the steps i = 1 .. n-1
__global__ void k_perm_chase(const int32_t* __restrict__ js, const int32_t* __restrict__ tp,
                             const int32_t* __restrict__ tj, int64_t n, int64_t k,
                             int32_t* __restrict__ out) {
  const int64_t p = blockIdx.x * 256ll + threadIdx.x;
  if (p >= k) return;
  int32_t q = (int32_t)p;
  int64_t t = 1;
  for (;;) {
    // next step >= t touching q: its own step (q >= t) or the first i >= t with j_i == q
    int64_t e = (q >= t && q >= 1) ? q : INT64_MAX;
    int32_t lo = tp[q], hi = tp[q + 1];
    while (lo < hi) {  // lower bound of t in the ascending list of steps with j_i == q
      const int32_t mid = (lo + hi) >> 1;
      if (tj[mid] < t) lo = mid + 1;
      else hi = mid;
    }
    if (lo < tp[q + 1]) e = min<int64_t>(e, tj[lo]);
    if (e == INT64_MAX) break;
    q = (e == q) ? js[e] : (int32_t)e;
    t = e + 1;
  }
  out[p] = q;
}

__global__ void k_perm_pairs(const int32_t* __restrict__ js, int64_t n, int32_t* __restrict__ ip,
                             int32_t* __restrict__ ij, double* __restrict__ ax) {
  const int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i > n) return;
  // row i (1 .. n-1) holds the single column j_i; row 0 is empty
  ip[i] = (int32_t)(i == 0 ? 0 : i - 1);
  if (i >= 1 && i < n) {
    ij[i - 1] = js[i];
    ax[i - 1] = 1.0;
  }
}

}  // namespace mlamg

using namespace mlamg;

extern "C" {

int mlamg_legacy_permutation(uint32_t seed, int64_t n, int64_t k, int32_t* out, void* stream) {
  MLAMG_REQUIRE(n >= 0 && k >= 0 && k <= n, "need 0 <= k <= n");
  MLAMG_REQUIRE(n < (int64_t(1) << 31), "n must fit int32");
  MLAMG_REQUIRE(k == 0 || out, "NULL argument");
  if (k == 0) return MLAMG_OK;
  hipStream_t s = S(stream);
  // the draws: j_i for i = n-1 .. 1, in numpy's order (js[0] unused)
  std::vector<int32_t> js((size_t)std::max<int64_t>(n, 1), 0);
  Mt19937 rng(seed);
  for (int64_t i = n - 1; i >= 1; --i) js[i] = (int32_t)rng.interval((uint32_t)i);
  int32_t* d_js = nullptr;
  MLAMG_HIP(hipMalloc(&d_js, sizeof(int32_t) * js.size()));
  mlamg_csr* J = nullptr;
  mlamg_csr* T = nullptr;
  int rc = csr_alloc(n, n, std::max<int64_t>(n - 1, 0), &J);
  if (rc == MLAMG_OK) {
    (void)hipMemcpyAsync(d_js, js.data(), sizeof(int32_t) * js.size(), hipMemcpyHostToDevice, s);
    hipLaunchKernelGGL(k_perm_pairs, dim3((unsigned)((n + 256) / 256)), dim3(256), 0, s, d_js, n,
                       J->indptr, J->indices, J->data);
    rc = transpose_impl(J, &T, s);  // row q: the steps i with j_i == q, ascending
  }
  if (rc == MLAMG_OK) {
    hipLaunchKernelGGL(k_perm_chase, dim3((unsigned)((k + 255) / 256)), dim3(256), 0, s, d_js,
                       T->indptr, T->indices, n, k, out);
    if (hipStreamSynchronize(s) != hipSuccess) {
      set_error("legacy_permutation: kernel failed");
      rc = MLAMG_EHIP;
    }
  }
  (void)hipStreamSynchronize(s);
  (void)hipFree(d_js);
  if (J) csr_free(J);
  if (T) csr_free(T);
  return rc;
}

}  // extern "C"
