// Aggregation kernels: seeded Bellman-Ford (ns/lib/graph.py:7-53), aggregate operator
// (graph.py:56-86, 234-238) and pyamg 4.x lloyd_cluster (called at graph.py:232).
//
// Distances. The reference relaxes edges sequentially in place; every relaxation is the
// monotone map d_j <- min(d_j, fl(d_i + w_ij)). Any fair order of monotone relaxations from the
// same start reaches the same (greatest) common fixed point, so the parallel in-place sweeps
// here (atomicMin on the order-preserving bit pattern of non-negative floats) end on exactly
// the reference distances, bit for bit, in fp32 (torch) or fp64 (pyamg) arithmetic.
// Labels. Which seed wins a node whose shortest path is not unique depends on the sequential
// sweep order, which a parallel sweep cannot reproduce. The rule here is order-independent:
// label(j) = min over tight in-edges (fl(d_i + w_ij) == d_j) of label(i), seeds labelled by
// themselves. With unique shortest paths (tie-free weights) it equals the reference's label.
#include "common.hpp"

#include <cfloat>

namespace mlamg {

// ---------------------------------------------------------------- fp32 Bellman-Ford (torch ref)
__global__ void k_bf_init(float* __restrict__ d, int32_t* __restrict__ lab, int64_t n) {
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  d[i] = __int_as_float(0x7f800000);  // +inf
  lab[i] = INT32_MAX;
}

__global__ void k_bf_seeds(const int32_t* __restrict__ seeds, int32_t k, float* __restrict__ d,
                           int32_t* __restrict__ lab, int32_t* __restrict__ is_seed) {
  int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= k) return;
  const int32_t c = seeds[t];
  d[c] = 0.0f;
  lab[c] = c;
  is_seed[c] = 1;
}

// push relaxation over the out-edges of row i (edge i -> j, weight g_ij in fp32)
__global__ void k_bf_sweep(const int32_t* __restrict__ ip, const int32_t* __restrict__ ij,
                           const float* __restrict__ w, int64_t n, float* d,
                           int32_t* __restrict__ changed) {
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  const float di = __hip_atomic_load(d + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (!(di < __int_as_float(0x7f800000))) return;
  int any = 0;
  for (int k = ip[i]; k < ip[i + 1]; ++k) {
    const int32_t j = ij[k];
    const float cand = di + w[k];
    const float dj = __hip_atomic_load(d + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cand < dj) {
      // non-negative floats order like their int bit patterns
      const int old = atomicMin(reinterpret_cast<int*>(d + j), __float_as_int(cand));
      if (cand < __int_as_float(old)) any = 1;
    }
  }
  if (any) *changed = 1;
}

// min-label propagation along tight edges
__global__ void k_bf_label(const int32_t* __restrict__ ip, const int32_t* __restrict__ ij,
                           const float* __restrict__ w, int64_t n, const float* __restrict__ d,
                           const int32_t* __restrict__ is_seed, int32_t* lab,
                           int32_t* __restrict__ changed) {
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  const float di = d[i];
  if (!(di < __int_as_float(0x7f800000))) return;
  const int32_t li = __hip_atomic_load(lab + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (li == INT32_MAX) return;
  int any = 0;
  for (int k = ip[i]; k < ip[i + 1]; ++k) {
    const int32_t j = ij[k];
    if (is_seed[j]) continue;
    if (di + w[k] == d[j]) {
      const int32_t lj = __hip_atomic_load(lab + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (li < lj) {
        const int32_t old = atomicMin(lab + j, li);
        if (li < old) any = 1;
      }
    }
  }
  if (any) *changed = 1;
}

__global__ void k_lab_finish(int32_t* __restrict__ lab, int64_t n) {
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i < n && lab[i] == INT32_MAX) lab[i] = -1;
}

__global__ void k_to_f32(const double* __restrict__ x, int64_t n, float* __restrict__ y) {
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i < n) y[i] = (float)x[i];
}

// ---------------------------------------------------------------- aggregate operator
__global__ void k_pos_init(int32_t* __restrict__ pos, int64_t n) {
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i < n) pos[i] = -1;
}
__global__ void k_pos_scatter(const int32_t* __restrict__ seeds, int32_t k, int32_t* pos) {
  int t = blockIdx.x * 256 + threadIdx.x;
  if (t < k) pos[seeds[t]] = t;  // duplicate seeds: python dict keeps the last, so does this
}
__global__ void k_pos_gather(const int32_t* __restrict__ lab, const int32_t* __restrict__ pos,
                             int64_t n, int32_t* __restrict__ col) {
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  const int32_t l = lab[i];
  col[i] = l >= 0 ? pos[l] : -1;
}

__global__ void k_agg_count(const int32_t* __restrict__ col, int64_t n, int32_t* __restrict__ cnt) {
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i < n) cnt[i] = col[i] >= 0 ? 1 : 0;
}
__global__ void k_agg_fill(const int32_t* __restrict__ col, const int32_t* __restrict__ ip,
                           int64_t n, int32_t* __restrict__ aj, double* __restrict__ ax) {
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  if (col[i] >= 0) {
    aj[ip[i]] = col[i];
    ax[ip[i]] = 1.0;
  }
}

// ---------------------------------------------------------------- pyamg lloyd_cluster (fp64)
// pyamg amg_core bellman_ford is a PULL relaxation: x_i <- min(x_i, A_ij + x_j) over row i.
__global__ void k_ll_init(double* __restrict__ d, int32_t* __restrict__ c, int64_t n) {
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  d[i] = DBL_MAX;
  c[i] = -1;
}
__global__ void k_ll_seeds(const int32_t* __restrict__ s, int32_t k, double* __restrict__ d,
                           int32_t* __restrict__ c) {
  int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= k) return;
  d[s[t]] = 0.0;
  c[s[t]] = t;
}

__global__ void k_ll_pull(const int32_t* __restrict__ ip, const int32_t* __restrict__ ij,
                          const double* __restrict__ w, int64_t n, double* d,
                          int32_t* __restrict__ changed) {
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  double xi = __hip_atomic_load(d + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const double x0 = xi;
  for (int k = ip[i]; k < ip[i + 1]; ++k) {
    const double dj = __hip_atomic_load(d + ij[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const double cand = w[k] + dj;
    if (cand < xi) xi = cand;
  }
  if (xi < x0) {
    __hip_atomic_store(d + i, xi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *changed = 1;
  }
}

// cluster = min cluster index over tight pull-neighbours (fl(A_ij + x_j) == x_i)
__global__ void k_ll_label(const int32_t* __restrict__ ip, const int32_t* __restrict__ ij,
                           const double* __restrict__ w, int64_t n, const double* __restrict__ d,
                           int32_t* c, const int32_t* __restrict__ is_seed,
                           int32_t* __restrict__ changed) {
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n || is_seed[i]) return;
  const double xi = d[i];
  if (!(xi < DBL_MAX)) return;
  int32_t best = __hip_atomic_load(c + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int32_t b0 = best;
  for (int k = ip[i]; k < ip[i + 1]; ++k) {
    const int32_t j = ij[k];
    if (w[k] + d[j] == xi) {
      const int32_t cj = __hip_atomic_load(c + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cj >= 0 && (best < 0 || cj < best)) best = cj;
    }
  }
  if (best != b0) {
    __hip_atomic_store(c + i, best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *changed = 1;
  }
}

__global__ void k_ll_boundary(const int32_t* __restrict__ ip, const int32_t* __restrict__ ij,
                              int64_t n, const int32_t* __restrict__ c, double* __restrict__ d) {
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  double v = DBL_MAX;
  for (int k = ip[i]; k < ip[i + 1]; ++k)
    if (c[i] != c[ij[k]]) {
      v = 0.0;
      break;
    }
  d[i] = v;
}

__global__ void k_ll_clusters_init(unsigned long long* __restrict__ mx, int32_t* __restrict__ mi,
                                   int32_t k) {
  int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= k) return;
  mx[t] = 0ull;
  mi[t] = INT32_MAX;
}
__global__ void k_ll_cluster_max(const int32_t* __restrict__ c, const double* __restrict__ d,
                                 int64_t n, unsigned long long* __restrict__ mx) {
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n || c[i] < 0) return;
  atomicMax(mx + c[i], (unsigned long long)__double_as_longlong(d[i]));  // d >= 0
}
__global__ void k_ll_cluster_argmax(const int32_t* __restrict__ c, const double* __restrict__ d,
                                    int64_t n, const unsigned long long* __restrict__ mx,
                                    int32_t* __restrict__ mi) {
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n || c[i] < 0) return;
  if ((unsigned long long)__double_as_longlong(d[i]) == mx[c[i]]) atomicMin(mi + c[i], (int32_t)i);
}
// sequential pyamg rule `if d[s[seed]] < d[i]: s[seed] = i` over ascending i ends on the old
// seed if it already holds the cluster maximum, else on the first index attaining it
__global__ void k_ll_recentre(int32_t* __restrict__ s, int32_t k, const double* __restrict__ d,
                              const unsigned long long* __restrict__ mx,
                              const int32_t* __restrict__ mi, int32_t* __restrict__ moved) {
  int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= k) return;
  const int32_t old = s[t];
  if ((unsigned long long)__double_as_longlong(d[old]) == mx[t]) return;
  if (mi[t] != INT32_MAX && mi[t] != old) {
    s[t] = mi[t];
    *moved = 1;
  }
}

__global__ void k_mark_seeds(const int32_t* __restrict__ s, int32_t k, int32_t* __restrict__ f) {
  int t = blockIdx.x * 256 + threadIdx.x;
  if (t < k) f[s[t]] = 1;
}

// ---------------------------------------------------------------- pyamg 4.x bellman_ford (exact)
// pyamg.graph.bellman_ford (the aggregation step of FullAggNet.forward, ns/model/agg_interp.py
// :475): amg_core sweeps rows 0..n-1 in place, x_i <- min(x_i, fl(G_ij + x_j)) in the graph's
// dtype with a strict <, nearest seed taken from the first strictly better neighbour, until a
// sweep changes no distance. Labels then depend on the sweep order, so this is the sequential
// sweep itself, run level-scheduled in one workgroup: level(i) = 1 + max level(j) over j < i
// coupled to i in either direction (the Gauss-Seidel schedule of gs.hip). A level's rows see the
// final values of every earlier-coupled row and the old values of every later-coupled one, and
// rows of a level touch no common entry: every (x, z) is bit for bit the sequential sweep's.
constexpr int kBfBlock = 1024;

template <typename T>
__global__ void k_bfp_init(T* __restrict__ x, int32_t* __restrict__ z, int64_t n, T big) {
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  x[i] = big;
  z[i] = -1;
}
template <typename T>
__global__ void k_bfp_seeds(const int32_t* __restrict__ s, int32_t k, T* __restrict__ x,
                            int32_t* __restrict__ z) {
  int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= k) return;
  x[s[t]] = T(0);
  z[s[t]] = s[t];
}

template <typename T>
__global__ __launch_bounds__(kBfBlock) void k_bf_pyamg(const int32_t* __restrict__ ip,
                                                       const int32_t* __restrict__ ij,
                                                       const double* __restrict__ ax,
                                                       const int32_t* __restrict__ rows,
                                                       const int32_t* __restrict__ lptr,
                                                       int32_t n_levels, int32_t max_sweeps, T* x,
                                                       int32_t* z, int32_t* __restrict__ out) {
  __shared__ int32_t changed;
  int32_t sweeps = 0, c = 0;
  do {
    if (threadIdx.x == 0) changed = 0;
    __syncthreads();
    for (int32_t l = 0; l < n_levels; ++l) {
      const int32_t a = lptr[l], e = lptr[l + 1];
      for (int32_t t = a + (int32_t)threadIdx.x; t < e; t += kBfBlock) {
        const int32_t i = rows[t];
        const T x0 = x[i];
        T xi = x0;
        int32_t zi = z[i];
        for (int32_t k = ip[i]; k < ip[i + 1]; ++k) {
          const int32_t j = ij[k];
          const T d = (T)ax[k] + x[j];  // the row's own entry reads the old x_i, as amg_core
          if (d < xi) {
            xi = d;
            zi = z[j];
          }
        }
        if (xi != x0) changed = 1;  // pyamg: (old_distances == distances).all()
        x[i] = xi;
        z[i] = zi;
      }
      __syncthreads();
    }
    ++sweeps;
    c = changed;
    __syncthreads();  // every thread has read the flag before it is reset
  } while (c && sweeps < max_sweeps);
  if (threadIdx.x == 0) {
    out[0] = sweeps;
    out[1] = c;
  }
}

static inline dim3 g1(int64_t n) { return dim3((unsigned)std::max<int64_t>(1, (n + 255) / 256)); }

static int read_flag(int32_t* dflag, hipStream_t s, int32_t* out) {
  MLAMG_HIP(hipMemcpyAsync(out, dflag, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  MLAMG_HIP(hipStreamSynchronize(s));
  return MLAMG_OK;
}

}  // namespace mlamg

using namespace mlamg;

extern "C" {

int mlamg_bellman_ford(const mlamg_csr* G, const int32_t* seeds, int32_t k, float* dist,
                       int32_t* cluster, int32_t* iters_host, void* stream) {
  MLAMG_REQUIRE(G && dist && cluster && (k == 0 || seeds), "NULL argument");
  MLAMG_REQUIRE(G->n_rows == G->n_cols, "graph must be square");
  hipStream_t s = S(stream);
  const int64_t n = G->n_rows;
  int64_t bad = 0;
  MLAMG_TRY(count_out_of_range(seeds, k, 0, n, s, &bad));
  MLAMG_REQUIRE(bad == 0, "seed index out of range [0, n)");
  float* w = nullptr;
  int32_t* flags = nullptr;
  MLAMG_HIP(hipMalloc(&w, sizeof(float) * std::max<int64_t>(G->nnz, 1)));
  MLAMG_HIP(hipMalloc(&flags, sizeof(int32_t) * (n + 1)));
  struct Free {
    void* a;
    void* b;
    ~Free() {
      (void)hipFree(a);
      (void)hipFree(b);
    }
  } guard{w, flags};
  int32_t* changed = flags + n;
  int32_t* is_seed = flags;
  if (G->nnz) hipLaunchKernelGGL(k_to_f32, g1(G->nnz), dim3(256), 0, s, G->data, G->nnz, w);
  MLAMG_HIP(hipMemsetAsync(flags, 0, sizeof(int32_t) * (n + 1), s));
  if (n) hipLaunchKernelGGL(k_bf_init, g1(n), dim3(256), 0, s, dist, cluster, n);
  if (k) hipLaunchKernelGGL(k_bf_seeds, g1(k), dim3(256), 0, s, seeds, k, dist, cluster, is_seed);
  MLAMG_HIP(hipGetLastError());
  int32_t sweeps = 0, h = 1;
  while (n && h) {
    MLAMG_HIP(hipMemsetAsync(changed, 0, sizeof(int32_t), s));
    hipLaunchKernelGGL(k_bf_sweep, g1(n), dim3(256), 0, s, G->indptr, G->indices, w, n, dist,
                       changed);
    MLAMG_TRY(read_flag(changed, s, &h));
    ++sweeps;
  }
  h = 1;
  while (n && h) {
    MLAMG_HIP(hipMemsetAsync(changed, 0, sizeof(int32_t), s));
    hipLaunchKernelGGL(k_bf_label, g1(n), dim3(256), 0, s, G->indptr, G->indices, w, n, dist,
                       is_seed, cluster, changed);
    MLAMG_TRY(read_flag(changed, s, &h));
  }
  if (n) hipLaunchKernelGGL(k_lab_finish, g1(n), dim3(256), 0, s, cluster, n);
  MLAMG_HIP(hipStreamSynchronize(s));
  if (iters_host) *iters_host = sweeps;
  return MLAMG_OK;
}

int mlamg_bellman_ford_pyamg(const mlamg_csr* G, const int32_t* seeds, int32_t k, int fp64,
                             void* dist, int32_t* nearest, int32_t* sweeps_host, void* stream) {
  MLAMG_REQUIRE(G && dist && nearest && (k == 0 || seeds), "NULL argument");
  MLAMG_REQUIRE(G->n_rows == G->n_cols, "graph must be square");
  MLAMG_REQUIRE(fp64 == 0 || fp64 == 1, "fp64 must be 0 (float32 graph) or 1 (float64 graph)");
  MLAMG_REQUIRE(k >= 0, "negative seed count");
  hipStream_t s = S(stream);
  const int64_t n = G->n_rows;
  MLAMG_REQUIRE(n < INT32_MAX, "graph too large for int32 rows");
  int64_t bad = 0;
  MLAMG_TRY(count_out_of_range(seeds, k, 0, n, s, &bad));
  MLAMG_REQUIRE(bad == 0, "seed index out of range [0, n)");
  // level schedule of the sequential sweep (host, O(nnz))
  std::vector<int32_t> ip(n + 1), ij(G->nnz);
  MLAMG_HIP(hipMemcpyAsync(ip.data(), G->indptr, sizeof(int32_t) * (n + 1), hipMemcpyDeviceToHost, s));
  if (G->nnz)
    MLAMG_HIP(hipMemcpyAsync(ij.data(), G->indices, sizeof(int32_t) * G->nnz, hipMemcpyDeviceToHost, s));
  MLAMG_HIP(hipStreamSynchronize(s));
  std::vector<int32_t> level(n, 0), req(n, 0);
  int32_t nlev = n ? 1 : 0;
  for (int64_t i = 0; i < n; ++i) {
    int32_t L = req[i];
    for (int32_t q = ip[i]; q < ip[i + 1]; ++q)
      if (ij[q] < i) L = std::max(L, level[ij[q]] + 1);
    level[i] = L;
    for (int32_t q = ip[i]; q < ip[i + 1]; ++q)
      if (ij[q] > i) req[ij[q]] = std::max(req[ij[q]], L + 1);
    nlev = std::max(nlev, L + 1);
  }
  std::vector<int32_t> plan((size_t)nlev + 1 + n + 2, 0);  // lptr | rows | out
  int32_t* lp = plan.data();
  for (int64_t i = 0; i < n; ++i) lp[level[i] + 1]++;
  for (int32_t l = 0; l < nlev; ++l) lp[l + 1] += lp[l];
  std::vector<int32_t> fill(lp, lp + nlev);
  int32_t* rows = lp + nlev + 1;
  for (int64_t i = 0; i < n; ++i) rows[fill[level[i]]++] = (int32_t)i;
  int32_t* dplan = nullptr;
  MLAMG_HIP(hipMalloc(&dplan, sizeof(int32_t) * plan.size()));
  struct Free {
    void* a;
    ~Free() { (void)hipFree(a); }
  } guard{dplan};
  MLAMG_HIP(hipMemcpyAsync(dplan, plan.data(), sizeof(int32_t) * plan.size(), hipMemcpyHostToDevice, s));
  int32_t* dout = dplan + nlev + 1 + n;
  // nonnegative weights converge within n + 1 sweeps; more means a negative cycle, on which
  // pyamg would never return
  const int32_t max_sweeps = (int32_t)std::min<int64_t>(n + 2, INT32_MAX);
  if (fp64) {
    double* x = static_cast<double*>(dist);
    if (n) hipLaunchKernelGGL(k_bfp_init<double>, g1(n), dim3(256), 0, s, x, nearest, n, DBL_MAX);
    if (k) hipLaunchKernelGGL(k_bfp_seeds<double>, g1(k), dim3(256), 0, s, seeds, k, x, nearest);
    if (n)
      hipLaunchKernelGGL(k_bf_pyamg<double>, dim3(1), dim3(kBfBlock), 0, s, G->indptr, G->indices,
                         G->data, dplan + nlev + 1, dplan, nlev, max_sweeps, x, nearest, dout);
  } else {
    float* x = static_cast<float*>(dist);
    if (n) hipLaunchKernelGGL(k_bfp_init<float>, g1(n), dim3(256), 0, s, x, nearest, n, FLT_MAX);
    if (k) hipLaunchKernelGGL(k_bfp_seeds<float>, g1(k), dim3(256), 0, s, seeds, k, x, nearest);
    if (n)
      hipLaunchKernelGGL(k_bf_pyamg<float>, dim3(1), dim3(kBfBlock), 0, s, G->indptr, G->indices,
                         G->data, dplan + nlev + 1, dplan, nlev, max_sweeps, x, nearest, dout);
  }
  MLAMG_HIP(hipGetLastError());
  int32_t res[2] = {n ? 0 : 1, 0};
  if (n) MLAMG_HIP(hipMemcpyAsync(res, dout, sizeof(res), hipMemcpyDeviceToHost, s));
  MLAMG_HIP(hipStreamSynchronize(s));
  MLAMG_REQUIRE(res[1] == 0, "bellman_ford: no fixed point after n + 2 sweeps (negative cycle)");
  if (sweeps_host) *sweeps_host = res[0];
  return MLAMG_OK;
}

int mlamg_labels_to_columns(const int32_t* label, int64_t n, const int32_t* seeds, int32_t k,
                            int32_t* col, void* stream) {
  MLAMG_REQUIRE(label && col && (k == 0 || seeds), "NULL argument");
  hipStream_t s = S(stream);
  int64_t bad = 0;
  MLAMG_TRY(count_out_of_range(seeds, k, 0, n, s, &bad));
  MLAMG_REQUIRE(bad == 0, "seed index out of range [0, n)");
  MLAMG_TRY(count_out_of_range(label, n, -1, n, s, &bad));
  MLAMG_REQUIRE(bad == 0, "label out of range [-1, n)");
  int32_t* pos = nullptr;
  MLAMG_HIP(hipMalloc(&pos, sizeof(int32_t) * std::max<int64_t>(n, 1)));
  if (n) hipLaunchKernelGGL(k_pos_init, g1(n), dim3(256), 0, s, pos, n);
  if (k) hipLaunchKernelGGL(k_pos_scatter, g1(k), dim3(256), 0, s, seeds, k, pos);
  if (n) hipLaunchKernelGGL(k_pos_gather, g1(n), dim3(256), 0, s, label, pos, n, col);
  hipError_t e = hipStreamSynchronize(s);
  (void)hipFree(pos);
  MLAMG_HIP(e);
  return MLAMG_OK;
}

int mlamg_aggregate_op(const int32_t* col, int64_t n, int64_t k, mlamg_csr** out, void* stream) {
  MLAMG_REQUIRE(out && (n == 0 || col), "NULL argument");
  hipStream_t s = S(stream);
  int64_t bad = 0;
  MLAMG_TRY(count_out_of_range(col, n, -1, k, s, &bad));
  MLAMG_REQUIRE(bad == 0, "aggregate column out of range [-1, k)");
  int32_t* cnt = nullptr;
  MLAMG_HIP(hipMalloc(&cnt, sizeof(int32_t) * (n + 1)));
  int32_t* ip = nullptr;
  hipError_t e = hipMalloc(&ip, sizeof(int32_t) * (n + 1));
  if (e != hipSuccess) {
    (void)hipFree(cnt);
    MLAMG_HIP(e);
  }
  int rc = MLAMG_OK;
  if (n) hipLaunchKernelGGL(k_agg_count, g1(n), dim3(256), 0, s, col, n, cnt);
  rc = exclusive_scan_i32(cnt, ip, n, s);
  int32_t nnz = 0;
  if (rc == MLAMG_OK) {
    (void)hipMemcpyAsync(&nnz, ip + n, sizeof(int32_t), hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
  }
  mlamg_csr* A = nullptr;
  if (rc == MLAMG_OK) rc = csr_alloc(n, k, nnz, &A);
  if (rc == MLAMG_OK) {
    (void)hipMemcpyAsync(A->indptr, ip, sizeof(int32_t) * (n + 1), hipMemcpyDeviceToDevice, s);
    if (n) hipLaunchKernelGGL(k_agg_fill, g1(n), dim3(256), 0, s, col, ip, n, A->indices, A->data);
    rc = csr_finalize(A, s);
  }
  (void)hipStreamSynchronize(s);
  (void)hipFree(cnt);
  (void)hipFree(ip);
  if (rc != MLAMG_OK) {
    csr_free(A);
    return rc;
  }
  *out = A;
  return MLAMG_OK;
}

int mlamg_lloyd_cluster(const mlamg_csr* G, int32_t* seeds, int32_t k, int maxiter, double* d,
                        int32_t* c, int32_t* iters_host, void* stream) {
  MLAMG_REQUIRE(G && seeds && d && c, "NULL argument");
  MLAMG_REQUIRE(k >= 1, "at least one seed is required");
  MLAMG_REQUIRE(maxiter >= 1, "maxiter must be positive");
  MLAMG_REQUIRE(G->n_rows == G->n_cols, "graph must be square");
  hipStream_t s = S(stream);
  const int64_t n = G->n_rows;
  int64_t bad = 0;
  MLAMG_TRY(count_out_of_range(seeds, k, 0, n, s, &bad));
  MLAMG_REQUIRE(bad == 0, "seed index out of range [0, n)");
  int32_t* iw = nullptr;
  unsigned long long* mx = nullptr;
  MLAMG_HIP(hipMalloc(&iw, sizeof(int32_t) * (n + k + 2)));
  hipError_t e0 = hipMalloc(&mx, sizeof(unsigned long long) * k);
  if (e0 != hipSuccess) {
    (void)hipFree(iw);
    MLAMG_HIP(e0);
  }
  struct Free {
    void* a;
    void* b;
    ~Free() {
      (void)hipFree(a);
      (void)hipFree(b);
    }
  } guard{iw, mx};
  int32_t* is_seed = iw;
  int32_t* mi = iw + n;
  int32_t* flag = iw + n + k;
  int it = 0;
  for (; it < maxiter; ++it) {
    MLAMG_HIP(hipMemsetAsync(is_seed, 0, sizeof(int32_t) * n, s));
    hipLaunchKernelGGL(k_mark_seeds, g1(k), dim3(256), 0, s, seeds, k, is_seed);
    hipLaunchKernelGGL(k_ll_init, g1(n), dim3(256), 0, s, d, c, n);
    hipLaunchKernelGGL(k_ll_seeds, g1(k), dim3(256), 0, s, seeds, k, d, c);
    int32_t h = 1;
    while (h) {  // outward distances
      MLAMG_HIP(hipMemsetAsync(flag, 0, sizeof(int32_t), s));
      hipLaunchKernelGGL(k_ll_pull, g1(n), dim3(256), 0, s, G->indptr, G->indices, G->data, n, d,
                         flag);
      MLAMG_TRY(read_flag(flag, s, &h));
    }
    h = 1;
    while (h) {  // cluster labels
      MLAMG_HIP(hipMemsetAsync(flag, 0, sizeof(int32_t), s));
      hipLaunchKernelGGL(k_ll_label, g1(n), dim3(256), 0, s, G->indptr, G->indices, G->data, n,
                         d, c, is_seed, flag);
      MLAMG_TRY(read_flag(flag, s, &h));
    }
    hipLaunchKernelGGL(k_ll_boundary, g1(n), dim3(256), 0, s, G->indptr, G->indices, n, c, d);
    h = 1;
    while (h) {  // inward distances (clusters cannot change: see header)
      MLAMG_HIP(hipMemsetAsync(flag, 0, sizeof(int32_t), s));
      hipLaunchKernelGGL(k_ll_pull, g1(n), dim3(256), 0, s, G->indptr, G->indices, G->data, n, d,
                         flag);
      MLAMG_TRY(read_flag(flag, s, &h));
    }
    hipLaunchKernelGGL(k_ll_clusters_init, g1(k), dim3(256), 0, s, mx, mi, k);
    hipLaunchKernelGGL(k_ll_cluster_max, g1(n), dim3(256), 0, s, c, d, n, mx);
    hipLaunchKernelGGL(k_ll_cluster_argmax, g1(n), dim3(256), 0, s, c, d, n, mx, mi);
    MLAMG_HIP(hipMemsetAsync(flag, 0, sizeof(int32_t), s));
    hipLaunchKernelGGL(k_ll_recentre, g1(k), dim3(256), 0, s, seeds, k, d, mx, mi, flag);
    MLAMG_TRY(read_flag(flag, s, &h));
    if (!h) {
      ++it;
      break;  // pyamg: `if (seeds == last_seeds).all(): break`
    }
  }
  MLAMG_HIP(hipGetLastError());
  if (iters_host) *iters_host = it;
  return MLAMG_OK;
}

}  // extern "C"
