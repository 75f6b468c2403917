// Aggregation kernels: seeded Bellman-Ford (ns/lib/graph.py:7-53), aggregate operator
// (graph.py:56-86, 234-238), pyamg 4.x lloyd_cluster (called at graph.py:232) and pyamg 4.x
// graph.bellman_ford (ns/model/agg_interp.py:475).
//
// Two label rules.
// * Reference order (the drop-in entry points mlamg_bellman_ford, mlamg_lloyd_cluster,
//   mlamg_bellman_ford_pyamg). The reference sweeps are sequential and in place, so which seed
//   wins a node whose shortest path is not unique depends on the sweep order. These entry points
//   run that order itself, level-scheduled (below), so distances AND labels are bitwise the
//   reference's on every input, ties included.
// * Order-independent (mlamg_bellman_ford_canon, mlamg_lloyd_cluster_canon; the multilevel and
//   distributed hierarchy, which have no reference counterpart). Every relaxation is the monotone
//   map d_j <- min(d_j, fl(d_i + w_ij)); any fair order of monotone relaxations from the same
//   start reaches the same (greatest) common fixed point, so parallel in-place sweeps (atomicMin
//   on the order-preserving bit pattern of non-negative floats) end on exactly the reference
//   distances. label(j) = min over tight in-edges (fl(d_i + w_ij) == d_j) of label(i), seeds
//   labelled by themselves; with unique shortest paths it equals the reference's label.
#include "common.hpp"

#include <cfloat>
#include <limits>

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
  atomicMax(c + s[t], t);  // c starts at -1; a repeated seed keeps its last index, as amg_core
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

// ---------------------------------------------------------------- sequential sweeps (exact)
// pyamg's pull sweep (amg_core bellman_ford: graph.bellman_ford at ns/model/agg_interp.py:475,
// and the outward pass of lloyd_cluster behind ns/lib/graph.py:232): rows 0..n-1 in place,
// x_i <- min(x_i, fl(G_ij + x_j)) over the row's stored entries with a strict <, the label taken
// from the first strictly better neighbour, until a sweep changes no distance. Run
// level-scheduled: level(i) = 1 + max level(j) over j < i coupled to i in either direction (the
// Gauss-Seidel schedule of gs.hip). A level's rows see the final values of every earlier-coupled
// row and the old values of every later-coupled one, and rows of a level touch no common entry:
// every (x, z) is bit for bit the sequential sweep's.
//
// The reference's push sweep (ns/lib/graph.py:40-51, modified_bellman_ford): for every edge
// (i, j) of the coalesced COO in row-major order, in place, fp32, strict <,
// `if d[i] + w_ij < d[j]: d[j] = d[i] + w_ij; nearest[j] = nearest[i]`. Row i's pushes use d[i]
// as it stands when row i is reached: its value at the end of the previous sweep folded with the
// pushes of the rows k < i into it, in ascending k. Call that mid_i. Node j ends the sweep at
// mid_j folded further with the pushes of the rows k > j, which also carry their mid_k, again in
// ascending k. So a sweep is two passes over the in-edge lists (transpose, sources ascending):
// mid, level-scheduled on in-edges from lower rows (level(j) = 1 + max level(k), k < j, k -> j),
// then end, fully parallel. A self-loop never pushes when w_jj >= 0; a negative one makes the
// reference loop forever and is refused.
constexpr int kBfBlock = 1024;
constexpr int64_t kSeqOneBlockMax = 1 << 18;  // wider graphs: one launch per level

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

// one row of the pull sweep; returns whether x_i changed
template <typename T>
__device__ inline int pull_row(int32_t i, const int32_t* __restrict__ ip,
                               const int32_t* __restrict__ ij, const double* __restrict__ ax,
                               T* x, int32_t* z) {
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
  x[i] = xi;
  z[i] = zi;
  return xi != x0;  // pyamg: (old_distances == distances).all()
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
    int any = 0;
    for (int32_t l = 0; l < n_levels; ++l) {
      const int32_t a = lptr[l], e = lptr[l + 1];
      for (int32_t t = a + (int32_t)threadIdx.x; t < e; t += kBfBlock)
        any |= pull_row<T>(rows[t], ip, ij, ax, x, z);
      __syncthreads();
    }
    if (any) changed = 1;
    __syncthreads();
    ++sweeps;
    c = changed;
    __syncthreads();  // every thread has read the flag before it is reset
  } while (c && sweeps < max_sweeps);
  if (threadIdx.x == 0) {
    out[0] = sweeps;
    out[1] = c;
  }
}

// one level of the pull sweep over the whole GPU (graphs above kSeqOneBlockMax rows)
template <typename T>
__global__ void k_bfp_level(const int32_t* __restrict__ ip, const int32_t* __restrict__ ij,
                            const double* __restrict__ ax, const int32_t* __restrict__ rows,
                            int32_t cnt, T* x, int32_t* z, int32_t* __restrict__ changed) {
  const int32_t t = blockIdx.x * 256 + threadIdx.x;
  if (t >= cnt) return;
  if (pull_row<T>(rows[t], ip, ij, ax, x, z)) *changed = 1;
}

// push sweep: mid_j (in-edges from rows k < j) and end_j (then rows k > j), see above
__device__ inline void push_mid(int32_t j, const int32_t* __restrict__ tip,
                                const int32_t* __restrict__ tsrc, const float* __restrict__ tw,
                                const float* d, const int32_t* z, float* dm, int32_t* zm) {
  float cur = d[j];
  int32_t lab = z[j];
  for (int32_t e = tip[j]; e < tip[j + 1]; ++e) {
    const int32_t k = tsrc[e];
    if (k >= j) break;
    const float cand = dm[k] + tw[e];
    if (cand < cur) {
      cur = cand;
      lab = zm[k];
    }
  }
  dm[j] = cur;
  zm[j] = lab;
}
__device__ inline int push_end(int32_t j, const int32_t* __restrict__ tip,
                               const int32_t* __restrict__ tsrc, const float* __restrict__ tw,
                               float* d, int32_t* z, const float* dm, const int32_t* zm) {
  float cur = dm[j];
  int32_t lab = zm[j];
  int32_t e0 = tip[j];
  while (e0 < tip[j + 1] && tsrc[e0] <= j) ++e0;
  for (int32_t e = e0; e < tip[j + 1]; ++e) {
    const int32_t k = tsrc[e];
    const float cand = dm[k] + tw[e];
    if (cand < cur) {
      cur = cand;
      lab = zm[k];
    }
  }
  const int ch = cur < d[j];  // distances only decrease: any update leaves end < start
  d[j] = cur;
  z[j] = lab;
  return ch;
}

__global__ __launch_bounds__(kBfBlock) void k_bf_push(
    const int32_t* __restrict__ tip, const int32_t* __restrict__ tsrc,
    const float* __restrict__ tw, const int32_t* __restrict__ rows,
    const int32_t* __restrict__ lptr, int32_t n_levels, int32_t n, int32_t max_sweeps, float* d,
    int32_t* z, float* dm, int32_t* zm, int32_t* __restrict__ out) {
  __shared__ int32_t changed;
  int32_t sweeps = 0, c = 0;
  do {
    if (threadIdx.x == 0) changed = 0;
    __syncthreads();
    for (int32_t l = 0; l < n_levels; ++l) {
      const int32_t a = lptr[l], e = lptr[l + 1];
      for (int32_t t = a + (int32_t)threadIdx.x; t < e; t += kBfBlock)
        push_mid(rows[t], tip, tsrc, tw, d, z, dm, zm);
      __syncthreads();
    }
    int any = 0;
    for (int32_t j = (int32_t)threadIdx.x; j < n; j += kBfBlock)
      any |= push_end(j, tip, tsrc, tw, d, z, dm, zm);
    if (any) changed = 1;
    __syncthreads();
    ++sweeps;
    c = changed;
    __syncthreads();
  } while (c && sweeps < max_sweeps);
  if (threadIdx.x == 0) {
    out[0] = sweeps;
    out[1] = c;
  }
}
__global__ void k_push_level(const int32_t* __restrict__ tip, const int32_t* __restrict__ tsrc,
                             const float* __restrict__ tw, const int32_t* __restrict__ rows,
                             int32_t cnt, const float* d, const int32_t* z, float* dm,
                             int32_t* zm) {
  const int32_t t = blockIdx.x * 256 + threadIdx.x;
  if (t < cnt) push_mid(rows[t], tip, tsrc, tw, d, z, dm, zm);
}
__global__ void k_push_end(const int32_t* __restrict__ tip, const int32_t* __restrict__ tsrc,
                           const float* __restrict__ tw, int32_t n, float* d, int32_t* z,
                           const float* dm, const int32_t* zm, int32_t* __restrict__ changed) {
  const int32_t j = blockIdx.x * 256 + threadIdx.x;
  if (j < n && push_end(j, tip, tsrc, tw, d, z, dm, zm)) *changed = 1;
}

static inline dim3 g1(int64_t n) { return dim3((unsigned)std::max<int64_t>(1, (n + 255) / 256)); }

static int read_flag(int32_t* dflag, hipStream_t s, int32_t* out) {
  MLAMG_HIP(hipMemcpyAsync(out, dflag, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  MLAMG_HIP(hipStreamSynchronize(s));
  return MLAMG_OK;
}

// ---------------------------------------------------------------- sequential-sweep plans (host)
// lptr[nlev + 1] | rows[n] (level order) | out[2] (sweeps, unconverged) [| tip[n+1] | tsrc[nnz]]
struct SeqPlan {
  int32_t* d = nullptr;  // device copy of the int32 plan
  float* tw = nullptr;   // push plan: in-edge weights (fp32), source order
  int32_t nlev = 0;
  int64_t n = 0, nnz = 0;
  ~SeqPlan() {
    if (d) (void)hipFree(d);
    if (tw) (void)hipFree(tw);
  }
  const int32_t* lptr() const { return d; }
  const int32_t* rows() const { return d + nlev + 1; }
  int32_t* out() const { return d + nlev + 1 + n; }
  const int32_t* tip() const { return d + nlev + 1 + n + 2; }
  const int32_t* tsrc() const { return d + nlev + 1 + n + 2 + n + 1; }
  std::vector<int32_t> h_lptr;  // host copy of lptr (per-level launches)
};

static int fetch_pattern(const mlamg_csr* G, hipStream_t s, std::vector<int32_t>& ip,
                         std::vector<int32_t>& ij, std::vector<double>* ax) {
  const int64_t n = G->n_rows;
  ip.assign(n + 1, 0);
  ij.assign(G->nnz, 0);
  MLAMG_HIP(hipMemcpyAsync(ip.data(), G->indptr, sizeof(int32_t) * (n + 1), hipMemcpyDeviceToHost, s));
  if (G->nnz)
    MLAMG_HIP(hipMemcpyAsync(ij.data(), G->indices, sizeof(int32_t) * G->nnz, hipMemcpyDeviceToHost, s));
  if (ax) {
    ax->assign(G->nnz, 0.0);
    if (G->nnz)
      MLAMG_HIP(hipMemcpyAsync(ax->data(), G->data, sizeof(double) * G->nnz, hipMemcpyDeviceToHost, s));
  }
  MLAMG_HIP(hipStreamSynchronize(s));
  return MLAMG_OK;
}

// rows bucketed by level; extra = trailing int32 words reserved after rows | out
static void plan_levels(const std::vector<int32_t>& level, int32_t nlev, size_t extra,
                        std::vector<int32_t>& plan) {
  const int64_t n = (int64_t)level.size();
  plan.assign((size_t)nlev + 1 + n + 2 + extra, 0);
  int32_t* lp = plan.data();
  for (int64_t i = 0; i < n; ++i) lp[level[i] + 1]++;
  for (int32_t l = 0; l < nlev; ++l) lp[l + 1] += lp[l];
  std::vector<int32_t> fill(lp, lp + nlev);
  int32_t* rows = lp + nlev + 1;
  for (int64_t i = 0; i < n; ++i) rows[fill[level[i]]++] = (int32_t)i;
}

// pull sweep (pyamg): level(i) = 1 + max level(j) over j < i coupled either way
static int build_pull_plan(const mlamg_csr* G, hipStream_t s, SeqPlan& P) {
  const int64_t n = G->n_rows;
  std::vector<int32_t> ip, ij;
  MLAMG_TRY(fetch_pattern(G, s, ip, ij, nullptr));
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
  std::vector<int32_t> plan;
  plan_levels(level, nlev, 0, plan);
  P.n = n;
  P.nnz = G->nnz;
  P.nlev = nlev;
  P.h_lptr.assign(plan.begin(), plan.begin() + nlev + 1);
  MLAMG_HIP(hipMalloc(&P.d, sizeof(int32_t) * plan.size()));
  MLAMG_HIP(hipMemcpyAsync(P.d, plan.data(), sizeof(int32_t) * plan.size(), hipMemcpyHostToDevice, s));
  MLAMG_HIP(hipStreamSynchronize(s));  // `plan` is pageable and goes out of scope
  return MLAMG_OK;
}

// pull sweeps to the fixed point on (x, z); *sweeps = pyamg's count (the last changes nothing)
template <typename T>
static int run_pull(const mlamg_csr* G, const SeqPlan& P, T* x, int32_t* z, hipStream_t s,
                    int32_t* sweeps) {
  const int64_t n = P.n;
  if (n == 0) {
    *sweeps = 1;
    return MLAMG_OK;
  }
  // nonnegative weights converge within n + 1 sweeps; more means a negative cycle, on which
  // pyamg would never return
  const int32_t max_sweeps = (int32_t)std::min<int64_t>(n + 2, INT32_MAX);
  int32_t res[2] = {0, 0};
  if (n <= kSeqOneBlockMax) {
    hipLaunchKernelGGL(k_bf_pyamg<T>, dim3(1), dim3(kBfBlock), 0, s, G->indptr, G->indices,
                       G->data, P.rows(), P.lptr(), P.nlev, max_sweeps, x, z, P.out());
    MLAMG_HIP(hipGetLastError());
    MLAMG_HIP(hipMemcpyAsync(res, P.out(), sizeof(res), hipMemcpyDeviceToHost, s));
    MLAMG_HIP(hipStreamSynchronize(s));
  } else {
    int32_t h = 1;
    while (h && res[0] < max_sweeps) {
      MLAMG_HIP(hipMemsetAsync(P.out() + 1, 0, sizeof(int32_t), s));
      for (int32_t l = 0; l < P.nlev; ++l) {
        const int32_t a = P.h_lptr[l], cnt = P.h_lptr[l + 1] - a;
        hipLaunchKernelGGL(k_bfp_level<T>, g1(cnt), dim3(256), 0, s, G->indptr, G->indices,
                           G->data, P.rows() + a, cnt, x, z, P.out() + 1);
      }
      MLAMG_HIP(hipGetLastError());
      MLAMG_TRY(read_flag(P.out() + 1, s, &h));
      ++res[0];
    }
    res[1] = h;
  }
  MLAMG_REQUIRE(res[1] == 0, "bellman_ford: no fixed point after n + 2 sweeps (negative cycle)");
  *sweeps = res[0];
  return MLAMG_OK;
}

// self-loops whose fp32 weight is negative (the reference's sweep would never terminate)
__global__ void k_neg_self_loops(const int32_t* __restrict__ ip, const int32_t* __restrict__ ij,
                                 const double* __restrict__ ax, int64_t n,
                                 int32_t* __restrict__ bad) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= n) return;
  for (int32_t q = ip[k]; q < ip[k + 1]; ++q)
    if (ij[q] == k && (float)ax[q] < 0.0f) *bad = 1;
}

// push sweep (ns/lib/graph.py:40-51): in-edge lists with sources ascending, fp32 weights, and
// the mid-pass schedule level(j) = 1 + max level(k) over edges k -> j with k < j. The in-edge
// lists are G's transpose (a stable sort by destination keeps the sources ascending: the
// reference's row-major push order), built on the device; only the level recurrence, a
// sequential pass, runs on the host over the pattern (round 5: C4 0.75 s before, values and
// the edge lists no longer cross PCIe).
static int build_push_plan(const mlamg_csr* G, hipStream_t s, SeqPlan& P) {
  const int64_t n = G->n_rows, nnz = G->nnz;
  int32_t* bad = nullptr;
  MLAMG_HIP(hipMalloc(&bad, sizeof(int32_t)));
  int32_t hbad = 0;
  hipError_t e = hipMemsetAsync(bad, 0, sizeof(int32_t), s);
  if (e == hipSuccess && n) {
    hipLaunchKernelGGL(k_neg_self_loops, g1(n), dim3(256), 0, s, G->indptr, G->indices, G->data,
                       n, bad);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(&hbad, bad, sizeof(int32_t), hipMemcpyDeviceToHost, s);
  // the in-edge lists: G's transpose on the device (it syncs s, so hbad is in too)
  mlamg_csr* T = nullptr;
  int rc = e == hipSuccess ? MLAMG_OK : MLAMG_EHIP;
  if (rc == MLAMG_OK) rc = transpose_impl(G, &T, s);
  (void)hipFree(bad);
  if (rc != MLAMG_OK) {
    if (e != hipSuccess) set_error(std::string("bellman_ford plan: ") + hipGetErrorString(e));
    return rc;
  }
  struct FreeT {
    mlamg_csr* t;
    ~FreeT() { csr_free(t); }
  } tguard{T};
  MLAMG_REQUIRE(hbad == 0, "negative self-loop weight: the reference sweep never terminates");
  std::vector<int32_t> ip, ij;
  MLAMG_TRY(fetch_pattern(G, s, ip, ij, nullptr));
  std::vector<int32_t> level(n, 0);
  int32_t nlev = n ? 1 : 0;
  for (int64_t k = 0; k < n; ++k) {
    nlev = std::max(nlev, level[k] + 1);
    const int32_t lk = level[k] + 1;
    for (int32_t q = ip[k]; q < ip[k + 1]; ++q) {
      const int32_t j = ij[q];
      if (j > k && level[j] < lk) level[j] = lk;
    }
  }
  std::vector<int32_t> plan;
  plan_levels(level, nlev, 0, plan);  // lptr | rows | out (the edge lists go in on the device)
  const size_t head = plan.size();
  P.n = n;
  P.nnz = nnz;
  P.nlev = nlev;
  P.h_lptr.assign(plan.begin(), plan.begin() + nlev + 1);
  MLAMG_HIP(hipMalloc(&P.d, sizeof(int32_t) * (head + n + 1 + std::max<int64_t>(nnz, 1))));
  MLAMG_HIP(hipMalloc(&P.tw, sizeof(float) * std::max<int64_t>(nnz, 1)));
  MLAMG_HIP(hipMemcpyAsync(P.d, plan.data(), sizeof(int32_t) * head, hipMemcpyHostToDevice, s));
  MLAMG_HIP(hipMemcpyAsync(P.d + head, T->indptr, sizeof(int32_t) * (n + 1),
                           hipMemcpyDeviceToDevice, s));
  if (nnz) {
    MLAMG_HIP(hipMemcpyAsync(P.d + head + n + 1, T->indices, sizeof(int32_t) * nnz,
                             hipMemcpyDeviceToDevice, s));
    // torch COO values are fp32 (ns/lib/sparse.py:28)
    hipLaunchKernelGGL(k_to_f32, g1(nnz), dim3(256), 0, s, T->data, nnz, P.tw);
    MLAMG_HIP(hipGetLastError());
  }
  MLAMG_HIP(hipStreamSynchronize(s));  // `plan` is pageable and goes out of scope
  return MLAMG_OK;
}

static int run_push(const SeqPlan& P, float* d, int32_t* z, float* dm, int32_t* zm, hipStream_t s,
                    int32_t* sweeps) {
  const int64_t n = P.n;
  if (n == 0) {
    *sweeps = 1;
    return MLAMG_OK;
  }
  const int32_t max_sweeps = (int32_t)std::min<int64_t>(n + 2, INT32_MAX);
  int32_t res[2] = {0, 0};
  if (n <= kSeqOneBlockMax) {
    hipLaunchKernelGGL(k_bf_push, dim3(1), dim3(kBfBlock), 0, s, P.tip(), P.tsrc(), P.tw,
                       P.rows(), P.lptr(), P.nlev, (int32_t)n, max_sweeps, d, z, dm, zm, P.out());
    MLAMG_HIP(hipGetLastError());
    MLAMG_HIP(hipMemcpyAsync(res, P.out(), sizeof(res), hipMemcpyDeviceToHost, s));
    MLAMG_HIP(hipStreamSynchronize(s));
  } else {
    int32_t h = 1;
    while (h && res[0] < max_sweeps) {
      MLAMG_HIP(hipMemsetAsync(P.out() + 1, 0, sizeof(int32_t), s));
      for (int32_t l = 0; l < P.nlev; ++l) {
        const int32_t a = P.h_lptr[l], cnt = P.h_lptr[l + 1] - a;
        hipLaunchKernelGGL(k_push_level, g1(cnt), dim3(256), 0, s, P.tip(), P.tsrc(), P.tw,
                           P.rows() + a, cnt, d, z, dm, zm);
      }
      hipLaunchKernelGGL(k_push_end, g1(n), dim3(256), 0, s, P.tip(), P.tsrc(), P.tw, (int32_t)n,
                         d, z, dm, zm, P.out() + 1);
      MLAMG_HIP(hipGetLastError());
      MLAMG_TRY(read_flag(P.out() + 1, s, &h));
      ++res[0];
    }
    res[1] = h;
  }
  MLAMG_REQUIRE(res[1] == 0, "modified_bellman_ford: no fixed point after n + 2 sweeps "
                             "(negative cycle: the reference would not return)");
  *sweeps = res[0];
  return MLAMG_OK;
}

}  // namespace mlamg

using namespace mlamg;

extern "C" {

int mlamg_bellman_ford_canon(const mlamg_csr* G, const int32_t* seeds, int32_t k, float* dist,
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

int mlamg_bf_canon_begin(const mlamg_csr* G, const int32_t* seeds, int32_t k, float* w,
                         float* dist, int32_t* cluster, int32_t* is_seed, void* stream) {
  MLAMG_REQUIRE(G && w && dist && cluster && is_seed && (k == 0 || seeds), "NULL argument");
  MLAMG_REQUIRE(G->n_rows == G->n_cols, "graph must be square");
  MLAMG_REQUIRE(k >= 0 && k <= G->n_rows, "seed count out of range");
  hipStream_t s = S(stream);
  const int64_t n = G->n_rows;
  int64_t bad = 0;
  MLAMG_TRY(count_out_of_range(seeds, k, 0, n, s, &bad));
  MLAMG_REQUIRE(bad == 0, "seed index out of range [0, n)");
  if (G->nnz) hipLaunchKernelGGL(k_to_f32, g1(G->nnz), dim3(256), 0, s, G->data, G->nnz, w);
  if (n) {
    MLAMG_HIP(hipMemsetAsync(is_seed, 0, sizeof(int32_t) * n, s));
    hipLaunchKernelGGL(k_bf_init, g1(n), dim3(256), 0, s, dist, cluster, n);
  }
  if (k) hipLaunchKernelGGL(k_bf_seeds, g1(k), dim3(256), 0, s, seeds, k, dist, cluster, is_seed);
  MLAMG_HIP(hipGetLastError());
  return MLAMG_OK;
}

int mlamg_bf_canon_sweep(const mlamg_csr* G, const float* w, float* dist, int32_t* changed,
                         void* stream) {
  MLAMG_REQUIRE(G && w && dist && changed, "NULL argument");
  MLAMG_REQUIRE(G->n_rows == G->n_cols, "graph must be square");
  if (G->n_rows)
    hipLaunchKernelGGL(k_bf_sweep, g1(G->n_rows), dim3(256), 0, S(stream), G->indptr, G->indices,
                       w, G->n_rows, dist, changed);
  MLAMG_HIP(hipGetLastError());
  return MLAMG_OK;
}

int mlamg_bf_canon_label(const mlamg_csr* G, const float* w, const float* dist,
                         const int32_t* is_seed, int32_t* cluster, int32_t* changed,
                         void* stream) {
  MLAMG_REQUIRE(G && w && dist && is_seed && cluster && changed, "NULL argument");
  MLAMG_REQUIRE(G->n_rows == G->n_cols, "graph must be square");
  if (G->n_rows)
    hipLaunchKernelGGL(k_bf_label, g1(G->n_rows), dim3(256), 0, S(stream), G->indptr, G->indices,
                       w, G->n_rows, dist, is_seed, cluster, changed);
  MLAMG_HIP(hipGetLastError());
  return MLAMG_OK;
}

int mlamg_bf_canon_end(int32_t* cluster, int64_t n, void* stream) {
  MLAMG_REQUIRE(n == 0 || cluster, "NULL argument");
  if (n) hipLaunchKernelGGL(k_lab_finish, g1(n), dim3(256), 0, S(stream), cluster, n);
  MLAMG_HIP(hipGetLastError());
  return MLAMG_OK;
}

int mlamg_bellman_ford(const mlamg_csr* G, const int32_t* seeds, int32_t k, float* dist,
                       int32_t* nearest, int32_t* sweeps_host, void* stream) {
  MLAMG_REQUIRE(G && dist && nearest && (k == 0 || seeds), "NULL argument");
  MLAMG_REQUIRE(G->n_rows == G->n_cols, "graph must be square");
  MLAMG_REQUIRE(k >= 0, "negative seed count");
  hipStream_t s = S(stream);
  const int64_t n = G->n_rows;
  MLAMG_REQUIRE(n < INT32_MAX, "graph too large for int32 rows");
  int64_t bad = 0;
  MLAMG_TRY(count_out_of_range(seeds, k, 0, n, s, &bad));
  MLAMG_REQUIRE(bad == 0, "seed index out of range [0, n)");
  SeqPlan P;
  MLAMG_TRY(build_push_plan(G, s, P));
  float* dm = nullptr;
  MLAMG_HIP(hipMalloc(&dm, sizeof(float) * 2 * std::max<int64_t>(n, 1)));
  struct Free {
    void* a;
    ~Free() { (void)hipFree(a); }
  } guard{dm};
  int32_t* zm = reinterpret_cast<int32_t*>(dm + std::max<int64_t>(n, 1));
  // graph.py:30-35: distance inf, nearest 0 (here -1: an unreached node never pushes, so the
  // initial label is only ever read back), centers 0 / themselves
  if (n) hipLaunchKernelGGL(k_bfp_init<float>, g1(n), dim3(256), 0, s, dist, nearest, n,
                            std::numeric_limits<float>::infinity());
  if (k) hipLaunchKernelGGL(k_bfp_seeds<float>, g1(k), dim3(256), 0, s, seeds, k, dist, nearest);
  MLAMG_HIP(hipGetLastError());
  int32_t sweeps = 0;
  MLAMG_TRY(run_push(P, dist, nearest, dm, zm, s, &sweeps));
  if (sweeps_host) *sweeps_host = sweeps;
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
  SeqPlan P;
  MLAMG_TRY(build_pull_plan(G, s, P));
  int32_t sweeps = 0;
  if (fp64) {
    double* x = static_cast<double*>(dist);
    if (n) hipLaunchKernelGGL(k_bfp_init<double>, g1(n), dim3(256), 0, s, x, nearest, n, DBL_MAX);
    if (k) hipLaunchKernelGGL(k_bfp_seeds<double>, g1(k), dim3(256), 0, s, seeds, k, x, nearest);
    MLAMG_HIP(hipGetLastError());
    MLAMG_TRY(run_pull<double>(G, P, x, nearest, s, &sweeps));
  } else {
    float* x = static_cast<float*>(dist);
    if (n) hipLaunchKernelGGL(k_bfp_init<float>, g1(n), dim3(256), 0, s, x, nearest, n, FLT_MAX);
    if (k) hipLaunchKernelGGL(k_bfp_seeds<float>, g1(k), dim3(256), 0, s, seeds, k, x, nearest);
    MLAMG_HIP(hipGetLastError());
    MLAMG_TRY(run_pull<float>(G, P, x, nearest, s, &sweeps));
  }
  if (sweeps_host) *sweeps_host = sweeps;
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

static int lloyd_impl(const mlamg_csr* G, int32_t* seeds, int32_t k, int maxiter, double* d,
                      int32_t* c, int32_t* iters_host, void* stream, bool exact) {
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
  SeqPlan P;
  if (exact) MLAMG_TRY(build_pull_plan(G, s, P));
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
    if (exact) {  // outward distances and clusters in amg_core's sweep order
      int32_t sw = 0;
      MLAMG_TRY(run_pull<double>(G, P, d, c, s, &sw));
    } else {
      while (h) {  // outward distances
        MLAMG_HIP(hipMemsetAsync(flag, 0, sizeof(int32_t), s));
        hipLaunchKernelGGL(k_ll_pull, g1(n), dim3(256), 0, s, G->indptr, G->indices, G->data, n,
                           d, flag);
        MLAMG_TRY(read_flag(flag, s, &h));
      }
      h = 1;
      while (h) {  // cluster labels
        MLAMG_HIP(hipMemsetAsync(flag, 0, sizeof(int32_t), s));
        hipLaunchKernelGGL(k_ll_label, g1(n), dim3(256), 0, s, G->indptr, G->indices, G->data, n,
                           d, c, is_seed, flag);
        MLAMG_TRY(read_flag(flag, s, &h));
      }
    }
    hipLaunchKernelGGL(k_ll_boundary, g1(n), dim3(256), 0, s, G->indptr, G->indices, n, c, d);
    // inward distances: the boundary nodes (d = 0) never improve with weights >= 0, and every
    // other node's neighbours all share its cluster, so amg_core's in-place label updates can
    // only copy a node's own cluster: clusters are unchanged and the distances are the
    // order-independent fixed point
    h = 1;
    while (h) {
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

int mlamg_lloyd_cluster(const mlamg_csr* G, int32_t* seeds, int32_t k, int maxiter, double* d,
                        int32_t* c, int32_t* iters_host, void* stream) {
  return lloyd_impl(G, seeds, k, maxiter, d, c, iters_host, stream, true);
}

int mlamg_lloyd_cluster_canon(const mlamg_csr* G, int32_t* seeds, int32_t k, int maxiter,
                              double* d, int32_t* c, int32_t* iters_host, void* stream) {
  return lloyd_impl(G, seeds, k, maxiter, d, c, iters_host, stream, false);
}

}  // extern "C"
