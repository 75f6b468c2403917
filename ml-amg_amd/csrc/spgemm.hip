// Setup-phase sparse kernels: transpose, SpGEMM (expand-sort-compress), Galerkin (R@A)@P,
// smoothed-aggregation smoother S = I - (w*Dinv)@A, row scaling, strength-of-connection maps.
//
// Bitwise contract with scipy sparsetools (scipy 1.15.3, the version in this image):
//  * csr_matmat sums C_ij = 0 + A_ik1*B_k1j + A_ik2*B_k2j + ... with k in the stored order of A's
//    row i, and drops entries whose sum is exactly zero. Expand writes the products of row i in
//    exactly that order; the segmented sort key (col << idx_bits | product index) is unique, so
//    equal columns stay in product order and the compress pass reproduces the sum bit for bit.
//  * P.T@A@P (multigrid.py:165, MLAMG.py:121) runs through scipy's CSC kernels, whose per-entry
//    accumulation order is ascending k; R = P^T built here has ascending columns, so (R@A)@P
//    with this SpGEMM (sorted-order mode for the intermediate) gives the same values; the
//    Galerkin output is sorted (scipy's is an unsorted CSC; values do not depend on that).
//  * csr_matmat emits each row's columns in reverse order of first appearance; mlamg_spgemm
//    reproduces that layout (order mode 1), because it is the summation order of a later C@x.
//  * (w*Dinv)@A (multigrid.py:44,106) goes dia -> csr -> csr_matmat, which emits a row's columns
//    in reverse stored order; I - that (multigrid.py:106) goes through csr_binop_csr_general,
//    which emits A's stored order without the diagonal, then the diagonal. Both orders matter
//    downstream (they are the summation orders of the next product) and are reproduced here.
#include "common.hpp"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>

#include <rocprim/rocprim.hpp>

namespace mlamg {

static int bits_for(int64_t v) {  // bits to represent values in [0, v)
  int b = 1;
  while ((int64_t(1) << b) < v) ++b;
  return b;
}

// ---------------------------------------------------------------- transpose
__global__ void k_entry_rows(const int32_t* __restrict__ indptr, int64_t n, int32_t* __restrict__ rows) {
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  for (int k = indptr[i]; k < indptr[i + 1]; ++k) rows[k] = (int32_t)i;
}

__global__ void k_transpose_keys(const int32_t* __restrict__ rows, const int32_t* __restrict__ cols,
                                 int64_t nnz, int rbits, uint64_t* __restrict__ keys,
                                 int32_t* __restrict__ perm, int32_t* __restrict__ colcnt) {
  int64_t e = blockIdx.x * 256ll + threadIdx.x;
  if (e >= nnz) return;
  const uint64_t c = (uint32_t)cols[e];
  keys[e] = (c << rbits) | (uint32_t)rows[e];
  perm[e] = (int32_t)e;
  atomicAdd(&colcnt[c], 1);
}

__global__ void k_transpose_fill(const uint64_t* __restrict__ skeys, const int32_t* __restrict__ sperm,
                                 const double* __restrict__ vals, int64_t nnz, uint64_t rmask,
                                 int32_t* __restrict__ out_idx, double* __restrict__ out_val) {
  int64_t e = blockIdx.x * 256ll + threadIdx.x;
  if (e >= nnz) return;
  out_idx[e] = (int32_t)(skeys[e] & rmask);
  out_val[e] = vals[sperm[e]];
}

int transpose_impl(const mlamg_csr* A, mlamg_csr** out, hipStream_t s) {
  mlamg_csr* T = nullptr;
  MLAMG_TRY(csr_alloc(A->n_cols, A->n_rows, A->nnz, &T));
  const int64_t nnz = A->nnz;
  int32_t* colcnt = nullptr;
  int32_t* rows = nullptr;
  uint64_t *k0 = nullptr, *k1 = nullptr;
  int32_t *p0 = nullptr, *p1 = nullptr;
  void* tmp = nullptr;
  int rc = MLAMG_OK;
  auto fail = [&](hipError_t e, const char* what) {
    set_error(std::string("transpose: ") + what + ": " + hipGetErrorString(e));
    rc = MLAMG_EHIP;
  };
  hipError_t e = hipMalloc(&colcnt, sizeof(int32_t) * (A->n_cols + 1));
  if (e == hipSuccess) e = hipMemsetAsync(colcnt, 0, sizeof(int32_t) * (A->n_cols + 1), s);
  if (e == hipSuccess && nnz) {
    e = hipMalloc(&rows, sizeof(int32_t) * nnz);
    if (e == hipSuccess) e = hipMalloc(&k0, sizeof(uint64_t) * nnz);
    if (e == hipSuccess) e = hipMalloc(&k1, sizeof(uint64_t) * nnz);
    if (e == hipSuccess) e = hipMalloc(&p0, sizeof(int32_t) * nnz);
    if (e == hipSuccess) e = hipMalloc(&p1, sizeof(int32_t) * nnz);
  }
  if (e != hipSuccess) fail(e, "alloc");
  if (rc == MLAMG_OK && nnz) {
    const int rbits = bits_for(std::max<int64_t>(A->n_rows, 2));
    const int cbits = bits_for(std::max<int64_t>(A->n_cols, 2));
    hipLaunchKernelGGL(k_entry_rows, dim3((A->n_rows + 255) / 256), dim3(256), 0, s, A->indptr,
                       A->n_rows, rows);
    hipLaunchKernelGGL(k_transpose_keys, dim3((nnz + 255) / 256), dim3(256), 0, s, rows,
                       A->indices, nnz, rbits, k0, p0, colcnt);
    size_t tb = 0;
    e = rocprim::radix_sort_pairs(nullptr, tb, k0, k1, p0, p1, (size_t)nnz, 0, rbits + cbits, s);
    if (e == hipSuccess) e = hipMalloc(&tmp, tb + 16);
    if (e == hipSuccess)
      e = rocprim::radix_sort_pairs(tmp, tb, k0, k1, p0, p1, (size_t)nnz, 0, rbits + cbits, s);
    if (e != hipSuccess) fail(e, "sort");
    if (rc == MLAMG_OK) {
      hipLaunchKernelGGL(k_transpose_fill, dim3((nnz + 255) / 256), dim3(256), 0, s, k1, p1,
                         A->data, nnz, (uint64_t(1) << rbits) - 1, T->indices, T->data);
    }
  }
  if (rc == MLAMG_OK) rc = exclusive_scan_i32(colcnt, T->indptr, A->n_cols, s);
  if (rc == MLAMG_OK) rc = csr_finalize(T, s);  // syncs
  else (void)hipStreamSynchronize(s);
  for (void* p : {(void*)colcnt, (void*)rows, (void*)k0, (void*)k1, (void*)p0, (void*)p1, tmp})
    if (p) (void)hipFree(p);
  if (rc != MLAMG_OK) {
    csr_free(T);
    return rc;
  }
  *out = T;
  return MLAMG_OK;
}

// ---------------------------------------------------------------- SpGEMM (ESC)
__global__ void k_count_products(const int32_t* __restrict__ ap, const int32_t* __restrict__ aj,
                                 const int32_t* __restrict__ bp, int64_t n,
                                 int64_t* __restrict__ cnt) {
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  int64_t c = 0;
  for (int k = ap[i]; k < ap[i + 1]; ++k) {
    const int j = aj[k];
    c += bp[j + 1] - bp[j];
  }
  cnt[i] = c;
}

__global__ void k_row_max(const int64_t* __restrict__ cnt, int64_t n, unsigned long long* mx) {
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  atomicMax(mx, (unsigned long long)cnt[i]);
}

// products of row i in csr_matmat order: A's stored order, then B row's stored order
__global__ void k_expand(const int32_t* __restrict__ ap, const int32_t* __restrict__ aj,
                         const double* __restrict__ ax, const int32_t* __restrict__ bp,
                         const int32_t* __restrict__ bj, const double* __restrict__ bx, int64_t n,
                         const int64_t* __restrict__ off, int ibits, uint64_t* __restrict__ keys,
                         double* __restrict__ prods) {
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  int64_t o = off[i];
  uint32_t t = 0;
  for (int k = ap[i]; k < ap[i + 1]; ++k) {
    const int j = aj[k];
    const double v = ax[k];
    for (int kk = bp[j]; kk < bp[j + 1]; ++kk) {
      keys[o + t] = ((uint64_t)(uint32_t)bj[kk] << ibits) | t;
      prods[o + t] = v * bx[kk];
      ++t;
    }
  }
}

// walk the sorted keys of row i; sum runs of equal columns in product order; keep nonzeros.
// order 0: output columns ascending. order 1: scipy csr_matmat order — columns in reverse order
// of their first appearance in the product stream (its linked list pushes each new column at
// the head). prods[] entries are read exactly once, so a finished run's sum can be parked in
// the slot of its first product.
__global__ void k_compress(const uint64_t* __restrict__ keys, double* __restrict__ prods,
                           const int64_t* __restrict__ off, int64_t n, int ibits, int order,
                           int32_t* __restrict__ mark, int32_t* __restrict__ tcol,
                           double* __restrict__ tval, int32_t* __restrict__ rowcnt) {
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  const int64_t a = off[i], b = off[i + 1];
  const uint64_t imask = (uint64_t(1) << ibits) - 1;
  int32_t m = 0;
  int64_t p = a;
  while (p < b) {
    const uint64_t col = keys[p] >> ibits;
    const int64_t tf = (int64_t)(keys[p] & imask);
    double sum = 0.0;
    while (p < b && (keys[p] >> ibits) == col) {
      sum += prods[a + (int64_t)(keys[p] & imask)];
      ++p;
    }
    if (sum != 0.0) {
      if (order == 0) {
        tcol[a + m] = (int32_t)col;
        tval[a + m] = sum;
        ++m;
      } else {
        prods[a + tf] = sum;
        mark[a + tf] = (int32_t)col;
      }
    }
  }
  if (order != 0) {
    for (int64_t t = b - 1; t >= a; --t) {
      const int32_t c = mark[t];
      if (c >= 0) {
        tcol[a + m] = c;
        tval[a + m] = prods[t];
        ++m;
      }
    }
  }
  rowcnt[i] = m;
}

__global__ void k_scatter_rows(const int64_t* __restrict__ off, const int32_t* __restrict__ cip,
                               const int32_t* __restrict__ tcol, const double* __restrict__ tval,
                               int64_t n, int32_t* __restrict__ cj, double* __restrict__ cx) {
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  const int64_t a = off[i];
  const int32_t o = cip[i];
  const int32_t m = cip[i + 1] - o;
  for (int32_t t = 0; t < m; ++t) {
    cj[o + t] = tcol[a + t];
    cx[o + t] = tval[a + t];
  }
}

// Setup temporaries (SpGEMM products, sort buffers, ...) come from a process-wide pool of
// device blocks instead of a hipMalloc/hipFree pair per buffer per call: a hierarchy build runs
// ~10 SpGEMMs whose temporaries reach several GB each, and every hipFree of such a block is an
// implicit device synchronisation plus an unmap. Blocks are reused best-fit (up to 2x the
// request) and returned to the pool when the DevBuf releases them (after a device sync, as
// hipFree would); mlamg_scratch_trim() frees the cached blocks (Hierarchy.build does at its end).
struct ScratchPool {
  std::mutex mu;
  std::multimap<size_t, void*> free_blocks;
  size_t cached = 0;
};
static ScratchPool& scratch_pool() {
  static ScratchPool p;
  return p;
}

static hipError_t pool_get(void** p, size_t bytes, size_t* got) {
  bytes = (std::max<size_t>(bytes, 1) + (size_t(2) << 20) - 1) & ~((size_t(2) << 20) - 1);
  ScratchPool& P = scratch_pool();
  {
    std::lock_guard<std::mutex> lk(P.mu);
    auto it = P.free_blocks.lower_bound(bytes);
    if (it != P.free_blocks.end() && it->first <= 2 * bytes) {
      *p = it->second;
      *got = it->first;
      P.cached -= it->first;
      P.free_blocks.erase(it);
      return hipSuccess;
    }
  }
  *got = bytes;
  hipError_t e = hipMalloc(p, bytes);
  if (e == hipErrorOutOfMemory) {  // drop the cache and retry once
    (void)hipGetLastError();
    size_t freed = 0;
    (void)mlamg_scratch_trim(&freed);
    e = hipMalloc(p, bytes);
  }
  return e;
}

static void pool_put(void* p, size_t bytes) {
  ScratchPool& P = scratch_pool();
  std::lock_guard<std::mutex> lk(P.mu);
  P.free_blocks.emplace(bytes, p);
  P.cached += bytes;
}

struct DevBuf {
  std::vector<std::pair<void*, size_t>> blocks;
  void release() {
    if (blocks.empty()) return;
    // kernels of this call may still read the blocks (error paths): wait, as hipFree would
    (void)hipDeviceSynchronize();
    for (auto& b : blocks) pool_put(b.first, b.second);
    blocks.clear();
  }
  ~DevBuf() { release(); }
  template <class T>
  hipError_t get(T** p, size_t count) {
    *p = nullptr;
    size_t got = 0;
    hipError_t e = pool_get((void**)p, sizeof(T) * std::max<size_t>(count, 1), &got);
    if (e == hipSuccess) blocks.emplace_back((void*)*p, got);
    return e;
  }
};

// Per-phase wall times of the sorted SpGEMM (Galerkin products), accumulated over calls and
// read by mlamg_setup_phase_times: the stream is synchronised at each phase boundary (setup
// only), so the times are the phases' own. Order: count, alloc, expand, sort, runsum, emit,
// finalize, free.
constexpr int kPhases = 8;
static const char* const kPhaseNames[kPhases] = {"count", "alloc", "expand", "sort",
                                                 "runsum", "emit", "finalize", "free"};
static std::mutex g_phase_mu;
static double g_phase_ms[kPhases] = {};

#define DB_CHECK(expr)                                                          \
  do {                                                                          \
    hipError_t _e = (expr);                                                     \
    if (_e != hipSuccess) {                                                     \
      set_error(std::string("spgemm: ") + #expr + ": " + hipGetErrorString(_e)); \
      return MLAMG_EHIP;                                                        \
    }                                                                           \
  } while (0)

// ---------------------------------------------------------------- SpGEMM, sorted output
// Global formulation of the same expand-sort-compress for order 0 (ascending columns): one
// thread per nonzero of A expands its products (row i, A's stored order, then B's row order
// = csr_matmat's accumulation order); a STABLE radix sort by (row, col) keeps equal keys in that
// order; each run head sums its run left to right and the nonzero sums are compacted in key
// order, which is already CSR order. Every phase is a flat data-parallel pass (no thread walks
// a whole long row), so it scales with the product count instead of the longest row.
__global__ void k_prod_len(const int32_t* __restrict__ aj, const int32_t* __restrict__ bp,
                           int64_t nnz, int64_t* __restrict__ len) {
  int64_t k = blockIdx.x * 256ll + threadIdx.x;
  if (k >= nnz) return;
  const int j = aj[k];
  len[k] = bp[j + 1] - bp[j];
}

// Block-cooperative expansion: a workgroup owns 256 consecutive nonzeros of A, whose products
// form one contiguous output range [poff[k0], poff[k0+256]); every thread walks that range with
// stride 256 (coalesced key/value stores), finding its nonzero by binary search in LDS.
__global__ __launch_bounds__(256) void k_expand_entries(const int32_t* __restrict__ rows,
                                                        const int32_t* __restrict__ aj,
                                                        const double* __restrict__ ax,
                                                        const int32_t* __restrict__ bp,
                                                        const int32_t* __restrict__ bj,
                                                        const double* __restrict__ bx, int64_t nnz,
                                                        const int64_t* __restrict__ poff, int cbits,
                                                        uint64_t* __restrict__ keys,
                                                        double* __restrict__ vals) {
  __shared__ int64_t off[257];
  __shared__ int32_t bstart[256];
  __shared__ uint64_t hi[256];
  __shared__ double av[256];
  const int64_t k0 = (int64_t)blockIdx.x * 256;
  const int cnt = (int)std::min<int64_t>(256, nnz - k0);
  const int t = threadIdx.x;
  if (t < cnt) {
    const int64_t k = k0 + t;
    off[t] = poff[k];
    const int j = aj[k];
    bstart[t] = bp[j];
    hi[t] = (uint64_t)(uint32_t)rows[k] << cbits;
    av[t] = ax[k];
  }
  if (t == 0) off[cnt] = poff[k0 + cnt];
  __syncthreads();
  const int64_t o0 = off[0], o1 = off[cnt];
  for (int64_t o = o0 + t; o < o1; o += 256) {
    int lo = 0, up = cnt;  // largest i with off[i] <= o
    while (up - lo > 1) {
      const int mid = (lo + up) >> 1;
      if (off[mid] <= o) lo = mid;
      else up = mid;
    }
    const int kk = bstart[lo] + (int)(o - off[lo]);
    keys[o] = hi[lo] | (uint32_t)bj[kk];
    vals[o] = av[lo] * bx[kk];
  }
}

// Run sums over LDS chunks of 2048 sorted products: run heads sum their run left to right
// (continuing in global memory when a run crosses the chunk end); keep = sum != 0.
__global__ __launch_bounds__(256) void k_run_sums(const uint64_t* __restrict__ keys,
                                                  const double* __restrict__ vals, int64_t total,
                                                  double* __restrict__ sums,
                                                  int32_t* __restrict__ keep) {
  constexpr int C = 2048;
  __shared__ uint64_t kk[C];
  __shared__ double vv[C];
  const int64_t c0 = (int64_t)blockIdx.x * C;
  const int m = (int)std::min<int64_t>(C, total - c0);
  for (int i = threadIdx.x; i < m; i += 256) {
    kk[i] = keys[c0 + i];
    vv[i] = vals[c0 + i];
  }
  const uint64_t before = c0 > 0 ? keys[c0 - 1] : ~0ull;
  __syncthreads();
  for (int i = threadIdx.x; i < m; i += 256) {
    const uint64_t key = kk[i];
    const bool head = i > 0 ? kk[i - 1] != key : (c0 == 0 || before != key);
    if (!head) {
      keep[c0 + i] = 0;
      continue;
    }
    double acc = 0.0;
    int f = i;
    for (; f < m && kk[f] == key; ++f) acc += vv[f];
    if (f == m)  // the run may continue into the next chunk
      for (int64_t g = c0 + m; g < total && keys[g] == key; ++g) acc += vals[g];
    sums[c0 + i] = acc;
    keep[c0 + i] = acc != 0.0 ? 1 : 0;
  }
}

__global__ void k_emit(const uint64_t* __restrict__ keys, const double* __restrict__ sums,
                       const int32_t* __restrict__ keep, const int32_t* __restrict__ pos,
                       int64_t total, int cbits, int32_t* __restrict__ cj,
                       double* __restrict__ cx, int32_t* __restrict__ crow) {
  int64_t e = blockIdx.x * 256ll + threadIdx.x;
  if (e >= total || !keep[e]) return;
  const uint64_t key = keys[e];
  const int32_t p = pos[e];
  cj[p] = (int32_t)(key & ((uint64_t(1) << cbits) - 1));
  cx[p] = sums[e];
  crow[p] = (int32_t)(key >> cbits);
}

// indptr from the (row-sorted) output rows: entry p opens rows crow[p-1]+1 .. crow[p]
__global__ void k_rowptr(const int32_t* __restrict__ crow, int64_t nnz, int64_t n,
                         int32_t* __restrict__ indptr) {
  const int64_t p = blockIdx.x * 256ll + threadIdx.x;
  if (p > nnz) return;
  const int64_t r0 = p > 0 ? crow[p - 1] + 1 : 0;
  const int64_t r1 = p < nnz ? crow[p] : n;
  for (int64_t r = r0; r <= r1; ++r) indptr[r] = (int32_t)p;
}

static int spgemm_sorted_impl(const mlamg_csr* A, const mlamg_csr* B, mlamg_csr** out,
                              int rbits, int cbits, hipStream_t s) {
  const int64_t n = A->n_rows, nz = A->nnz;
  // per-phase wall times (stream synchronised at each boundary), accumulated for
  // mlamg_setup_phase_times; MLAMG_TIMING=1 also prints them on stderr
  static const bool timing = std::getenv("MLAMG_TIMING") != nullptr;
  auto t_prev = std::chrono::steady_clock::now();
  auto tick = [&](const char* what) {
    (void)hipStreamSynchronize(s);
    const auto t = std::chrono::steady_clock::now();
    const double ms = std::chrono::duration<double, std::milli>(t - t_prev).count();
    t_prev = t;
    {
      std::lock_guard<std::mutex> lk(g_phase_mu);
      for (int i = 0; i < kPhases; ++i)
        if (std::strcmp(kPhaseNames[i], what) == 0) g_phase_ms[i] += ms;
    }
    if (timing)
      std::fprintf(stderr, "[spgemm %lldx%lld nnzA=%lld] %-8s %8.2f ms\n", (long long)n,
                   (long long)B->n_cols, (long long)nz, what, ms);
  };
  DevBuf db;
  int32_t* rows = nullptr;
  int64_t *len = nullptr, *poff = nullptr;
  DB_CHECK(db.get(&rows, nz));
  DB_CHECK(db.get(&len, nz + 1));
  DB_CHECK(db.get(&poff, nz + 1));
  if (n) hipLaunchKernelGGL(k_entry_rows, dim3((n + 255) / 256), dim3(256), 0, s, A->indptr, n, rows);
  if (nz)
    hipLaunchKernelGGL(k_prod_len, dim3((nz + 255) / 256), dim3(256), 0, s, A->indices, B->indptr,
                       nz, len);
  MLAMG_TRY(exclusive_scan_i64(len, poff, nz, s));
  int64_t total = 0;
  DB_CHECK(hipMemcpyAsync(&total, poff + nz, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  DB_CHECK(hipStreamSynchronize(s));
  MLAMG_REQUIRE(total < (int64_t(1) << 31) - 1, "too many intermediate products (>2G)");
  tick("count");
  if (timing) std::fprintf(stderr, "[spgemm] products %lld\n", (long long)total);
  uint64_t *k0 = nullptr, *k1 = nullptr;
  double *v0 = nullptr, *v1 = nullptr, *sums = nullptr;
  int32_t *keep = nullptr, *pos = nullptr, *crow = nullptr;
  DB_CHECK(db.get(&k0, total));
  DB_CHECK(db.get(&k1, total));
  DB_CHECK(db.get(&v0, total));
  DB_CHECK(db.get(&v1, total));
  DB_CHECK(db.get(&sums, total));
  DB_CHECK(db.get(&keep, total + 1));
  DB_CHECK(db.get(&pos, total + 1));
  tick("alloc");
  if (nz)
    hipLaunchKernelGGL(k_expand_entries, dim3((unsigned)((nz + 255) / 256)), dim3(256), 0, s, rows,
                       A->indices, A->data, B->indptr, B->indices, B->data, nz, poff, cbits, k0, v0);
  tick("expand");
  if (total > 0) {
    size_t tb = 0;
    DB_CHECK(rocprim::radix_sort_pairs(nullptr, tb, k0, k1, v0, v1, (size_t)total, 0,
                                       rbits + cbits, s));
    void* tmp = nullptr;
    DB_CHECK(db.get((char**)&tmp, tb + 16));
    DB_CHECK(rocprim::radix_sort_pairs(tmp, tb, k0, k1, v0, v1, (size_t)total, 0, rbits + cbits,
                                       s));
    tick("sort");
    hipLaunchKernelGGL(k_run_sums, dim3((unsigned)((total + 2047) / 2048)), dim3(256), 0, s, k1,
                       v1, total, sums, keep);
    tick("runsum");
  }
  MLAMG_TRY(exclusive_scan_i32(keep, pos, total, s));
  int32_t nnzc = 0;
  DB_CHECK(hipMemcpyAsync(&nnzc, pos + total, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  DB_CHECK(hipStreamSynchronize(s));
  mlamg_csr* C = nullptr;
  DB_CHECK(db.get(&crow, (size_t)nnzc + 1));
  MLAMG_TRY(csr_alloc(n, B->n_cols, nnzc, &C));
  if (total > 0)
    hipLaunchKernelGGL(k_emit, dim3((total + 255) / 256), dim3(256), 0, s, k1, sums, keep, pos,
                       total, cbits, C->indices, C->data, crow);
  hipLaunchKernelGGL(k_rowptr, dim3((unsigned)((nnzc + 1 + 255) / 256)), dim3(256), 0, s, crow,
                     (int64_t)nnzc, n, C->indptr);
  int rc = MLAMG_OK;
  if (hipGetLastError() != hipSuccess) {
    set_error("spgemm: kernel launch failed");
    rc = MLAMG_EHIP;
  }
  tick("emit");
  if (rc == MLAMG_OK) rc = csr_finalize(C, s);  // syncs before DevBuf frees
  else (void)hipStreamSynchronize(s);
  tick("finalize");
  if (rc != MLAMG_OK) {
    csr_free(C);
    return rc;
  }
  *out = C;
  db.release();
  tick("free");
  return MLAMG_OK;
}

// ---------------------------------------------------------------- SpGEMM, dense row accumulator
// For a narrow product (B->n_cols doubles fit in LDS) with long rows — the coarsest Galerkin
// products, where expand-sort would materialise ~0.7 G products: one workgroup per row of C
// keeps the whole row in LDS. It walks A's row in stored order; at each step the entries of B's
// row are distinct columns, so its threads add in parallel without conflicts, and a barrier
// orders consecutive steps: every C_ij is 0 + A_ik1 B_k1j + A_ik2 B_k2j + ... in csr_matmat's
// order, bit for bit. Zeros (never touched or cancelled) are dropped like scipy drops them.
constexpr int kDenseMaxCols = 15360;  // 120 KiB of LDS

__global__ __launch_bounds__(512) void k_dense_rows(const int32_t* __restrict__ ap,
                                                    const int32_t* __restrict__ aj,
                                                    const double* __restrict__ ax,
                                                    const int32_t* __restrict__ bp,
                                                    const int32_t* __restrict__ bj,
                                                    const double* __restrict__ bx, int ncols,
                                                    double* __restrict__ dense,
                                                    int32_t* __restrict__ rowcnt) {
  extern __shared__ double acc[];
  __shared__ int32_t cnt[512 / 64];
  const int64_t i = blockIdx.x;
  const int t = threadIdx.x;
  for (int j = t; j < ncols; j += 512) acc[j] = 0.0;
  __syncthreads();
  for (int k = ap[i]; k < ap[i + 1]; ++k) {
    const int r = aj[k];
    const double a = ax[k];
    for (int e = bp[r] + t; e < bp[r + 1]; e += 512) acc[bj[e]] += a * bx[e];
    __syncthreads();
  }
  int c = 0;
  double* row = dense + i * (int64_t)ncols;
  for (int j = t; j < ncols; j += 512) {
    const double v = acc[j];
    row[j] = v;
    c += v != 0.0;
  }
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
  if ((t & 63) == 0) cnt[t >> 6] = c;
  __syncthreads();
  if (t == 0) {
    int tot = 0;
    for (int w = 0; w < 512 / 64; ++w) tot += cnt[w];
    rowcnt[i] = tot;
  }
}

// compact the dense rows (ascending columns) into CSR; one workgroup per row
__global__ __launch_bounds__(256) void k_dense_compact(const double* __restrict__ dense, int ncols,
                                                       const int32_t* __restrict__ ip,
                                                       int32_t* __restrict__ cj,
                                                       double* __restrict__ cx) {
  __shared__ int32_t wsum[4];
  __shared__ int32_t base;
  const int64_t i = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const double* row = dense + i * (int64_t)ncols;
  if (t == 0) base = ip[i];
  __syncthreads();
  for (int j0 = 0; j0 < ncols; j0 += 256) {
    const int j = j0 + t;
    const double v = j < ncols ? row[j] : 0.0;
    const bool nz = v != 0.0;
    const unsigned long long m = __ballot(nz);
    const int before = __popcll(m & ((1ull << lane) - 1));
    if (lane == 0) wsum[w] = __popcll(m);
    __syncthreads();
    int off = base;
    for (int q = 0; q < w; ++q) off += wsum[q];
    if (nz) {
      cj[off + before] = j;
      cx[off + before] = v;
    }
    __syncthreads();
    if (t == 0) base += wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
  }
}

static int spgemm_dense_impl(const mlamg_csr* A, const mlamg_csr* B, mlamg_csr** out,
                             hipStream_t s) {
  const int64_t n = A->n_rows, nc = B->n_cols;
  DevBuf db;
  double* dense = nullptr;
  int32_t* rowcnt = nullptr;
  DB_CHECK(db.get(&dense, (size_t)(n * nc)));
  DB_CHECK(db.get(&rowcnt, n + 1));
  if (n)
    hipLaunchKernelGGL(k_dense_rows, dim3((unsigned)n), dim3(512), sizeof(double) * nc, s,
                       A->indptr, A->indices, A->data, B->indptr, B->indices, B->data, (int)nc,
                       dense, rowcnt);
  int32_t* cip = nullptr;
  DB_CHECK(db.get(&cip, n + 1));
  MLAMG_TRY(exclusive_scan_i32(rowcnt, cip, n, s));
  int32_t nnzc = 0;
  DB_CHECK(hipMemcpyAsync(&nnzc, cip + n, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  DB_CHECK(hipStreamSynchronize(s));
  mlamg_csr* C = nullptr;
  MLAMG_TRY(csr_alloc(n, nc, nnzc, &C));
  int rc = MLAMG_OK;
  if (hipMemcpyAsync(C->indptr, cip, sizeof(int32_t) * (n + 1), hipMemcpyDeviceToDevice, s) !=
      hipSuccess) {
    set_error("spgemm(dense): indptr copy failed");
    rc = MLAMG_EHIP;
  }
  if (rc == MLAMG_OK && n)
    hipLaunchKernelGGL(k_dense_compact, dim3((unsigned)n), dim3(256), 0, s, dense, (int)nc, cip,
                       C->indices, C->data);
  if (rc == MLAMG_OK && hipGetLastError() != hipSuccess) {
    set_error("spgemm(dense): kernel launch failed");
    rc = MLAMG_EHIP;
  }
  if (rc == MLAMG_OK) rc = csr_finalize(C, s);  // syncs before DevBuf frees
  else (void)hipStreamSynchronize(s);
  if (rc != MLAMG_OK) {
    csr_free(C);
    return rc;
  }
  *out = C;
  return MLAMG_OK;
}

int spgemm_impl(const mlamg_csr* A, const mlamg_csr* B, mlamg_csr** out, int order,
                hipStream_t s) {
  MLAMG_REQUIRE(A->n_cols == B->n_rows, "inner dimensions differ");
  if (order == 0) {
    // narrow output with many products per entry: dense LDS rows (no sort, no product buffers).
    // MLAMG_SPGEMM=dense|esc forces a path where it applies (tests cover both).
    const char* force = std::getenv("MLAMG_SPGEMM");
    const bool fits = B->n_cols <= kDenseMaxCols && A->n_rows * B->n_cols <= (int64_t(1) << 28);
    const bool heavy = (double)A->nnz * ((double)B->nnz / std::max<int64_t>(B->n_rows, 1)) >
                       8.0 * (double)A->n_rows * (double)std::min<int64_t>(B->n_cols, 2048);
    const bool want_dense = force ? std::strcmp(force, "dense") == 0 : heavy;
    if (fits && want_dense) return spgemm_dense_impl(A, B, out, s);
    const int rbits = bits_for(std::max<int64_t>(A->n_rows, 2));
    const int cb = bits_for(std::max<int64_t>(B->n_cols, 2));
    if (rbits + cb <= 64) return spgemm_sorted_impl(A, B, out, rbits, cb, s);
  }
  const int64_t n = A->n_rows;
  DevBuf db;
  int64_t* cnt = nullptr;
  int64_t* off = nullptr;
  unsigned long long* dmax = nullptr;
  DB_CHECK(db.get(&cnt, n + 1));
  DB_CHECK(db.get(&off, n + 1));
  DB_CHECK(db.get(&dmax, 1));
  DB_CHECK(hipMemsetAsync(dmax, 0, sizeof(unsigned long long), s));
  if (n) {
    hipLaunchKernelGGL(k_count_products, dim3((n + 255) / 256), dim3(256), 0, s, A->indptr,
                       A->indices, B->indptr, n, cnt);
    hipLaunchKernelGGL(k_row_max, dim3((n + 255) / 256), dim3(256), 0, s, cnt, n, dmax);
  }
  MLAMG_TRY(exclusive_scan_i64(cnt, off, n, s));
  int64_t total = 0;
  unsigned long long rmax = 0;
  DB_CHECK(hipMemcpyAsync(&total, off + n, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  DB_CHECK(hipMemcpyAsync(&rmax, dmax, sizeof(rmax), hipMemcpyDeviceToHost, s));
  DB_CHECK(hipStreamSynchronize(s));
  MLAMG_REQUIRE(total < (int64_t(1) << 32) - 1, "too many intermediate products (>4G)");
  const int ibits = bits_for(std::max<int64_t>((int64_t)rmax, 2));
  const int cbits = bits_for(std::max<int64_t>(B->n_cols, 2));
  MLAMG_REQUIRE(ibits + cbits <= 64, "key does not fit 64 bits");

  uint64_t *k0 = nullptr, *k1 = nullptr;
  double* prods = nullptr;
  int32_t* tcol = nullptr;
  double* tval = nullptr;
  int32_t* rowcnt = nullptr;
  DB_CHECK(db.get(&k0, total));
  DB_CHECK(db.get(&k1, total));
  DB_CHECK(db.get(&prods, total));
  DB_CHECK(db.get(&tcol, total));
  DB_CHECK(db.get(&tval, total));
  DB_CHECK(db.get(&rowcnt, n + 1));
  int32_t* mark = nullptr;
  if (order != 0) {
    DB_CHECK(db.get(&mark, total));
    DB_CHECK(hipMemsetAsync(mark, 0xFF, sizeof(int32_t) * std::max<int64_t>(total, 1), s));
  }
  if (n) {
    hipLaunchKernelGGL(k_expand, dim3((n + 255) / 256), dim3(256), 0, s, A->indptr, A->indices,
                       A->data, B->indptr, B->indices, B->data, n, off, ibits, k0, prods);
  }
  if (total > 0) {
    size_t tb = 0;
    DB_CHECK(rocprim::segmented_radix_sort_keys(nullptr, tb, k0, k1, (unsigned)total, (unsigned)n,
                                                off, off + 1, 0, ibits + cbits, s));
    void* tmp = nullptr;
    DB_CHECK(db.get((char**)&tmp, tb + 16));
    DB_CHECK(rocprim::segmented_radix_sort_keys(tmp, tb, k0, k1, (unsigned)total, (unsigned)n,
                                                off, off + 1, 0, ibits + cbits, s));
  }
  if (n) {
    hipLaunchKernelGGL(k_compress, dim3((n + 255) / 256), dim3(256), 0, s, k1, prods, off, n,
                       ibits, order, mark, tcol, tval, rowcnt);
  }
  int32_t* cip = nullptr;
  DB_CHECK(db.get(&cip, n + 1));
  MLAMG_TRY(exclusive_scan_i32(rowcnt, cip, n, s));
  int32_t nnzc = 0;
  DB_CHECK(hipMemcpyAsync(&nnzc, cip + n, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  DB_CHECK(hipStreamSynchronize(s));
  mlamg_csr* C = nullptr;
  MLAMG_TRY(csr_alloc(n, B->n_cols, nnzc, &C));
  if (hipMemcpyAsync(C->indptr, cip, sizeof(int32_t) * (n + 1), hipMemcpyDeviceToDevice, s) !=
      hipSuccess) {
    csr_free(C);
    set_error("spgemm: indptr copy failed");
    return MLAMG_EHIP;
  }
  if (n)
    hipLaunchKernelGGL(k_scatter_rows, dim3((n + 255) / 256), dim3(256), 0, s, off, cip, tcol,
                       tval, n, C->indices, C->data);
  int rc = csr_finalize(C, s);  // syncs before DevBuf frees
  if (rc != MLAMG_OK) {
    csr_free(C);
    return rc;
  }
  *out = C;
  return MLAMG_OK;
}

// ---------------------------------------------------------------- row scaling / SA smoother
// mode 0: M = diag(d)@A, reversed stored order, zeros dropped (csr_matmat of dia@csr)
// mode 1: S = I - diag(d)@A in csr_binop_csr_general order (A's stored order sans diagonal,
//         then the diagonal), zeros dropped
// mode 2: M = diag(d)@A in place of A's values (csr_scale_rows: same pattern, same order,
//         nothing dropped — pyamg's scale_rows(A, d, copy=True))
__global__ void k_scale_count(const int32_t* __restrict__ ap, const int32_t* __restrict__ aj,
                              const double* __restrict__ ax, const double* __restrict__ d,
                              int64_t n, int mode, int32_t* __restrict__ cnt) {
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  const double di = d[i];
  int32_t c = 0;
  if (mode == 2) {
    c = ap[i + 1] - ap[i];
  } else if (mode == 0) {
    for (int k = ap[i]; k < ap[i + 1]; ++k) c += (di * ax[k] != 0.0);
  } else {
    double mdiag = 0.0;
    for (int k = ap[i]; k < ap[i + 1]; ++k) {
      const double m = di * ax[k];
      if (aj[k] == (int32_t)i) {
        mdiag = m;
      } else {
        c += (0.0 - m != 0.0);
      }
    }
    c += (1.0 - mdiag != 0.0);
  }
  cnt[i] = c;
}

__global__ void k_scale_fill(const int32_t* __restrict__ ap, const int32_t* __restrict__ aj,
                             const double* __restrict__ ax, const double* __restrict__ d,
                             int64_t n, int mode, const int32_t* __restrict__ cp,
                             int32_t* __restrict__ cj, double* __restrict__ cx) {
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  const double di = d[i];
  int32_t o = cp[i];
  if (mode == 2) {
    for (int k = ap[i]; k < ap[i + 1]; ++k, ++o) {
      cj[o] = aj[k];
      cx[o] = ax[k] * di;  // csr_scale_rows: Ax[jj] *= Xx[i]
    }
  } else if (mode == 0) {
    for (int k = ap[i + 1] - 1; k >= ap[i]; --k) {
      const double m = di * ax[k];
      if (m != 0.0) {
        cj[o] = aj[k];
        cx[o] = m;
        ++o;
      }
    }
  } else {
    double mdiag = 0.0;
    for (int k = ap[i]; k < ap[i + 1]; ++k) {
      const double m = di * ax[k];
      if (aj[k] == (int32_t)i) {
        mdiag = m;
        continue;
      }
      const double v = 0.0 - m;
      if (v != 0.0) {
        cj[o] = aj[k];
        cx[o] = v;
        ++o;
      }
    }
    const double v = 1.0 - mdiag;
    if (v != 0.0) {
      cj[o] = (int32_t)i;
      cx[o] = v;
    }
  }
}

int scale_rows_impl(const mlamg_csr* A, const double* d, int mode, mlamg_csr** out,
                    hipStream_t s) {
  const int64_t n = A->n_rows;
  DevBuf db;
  int32_t* cnt = nullptr;
  int32_t* cp = nullptr;
  DB_CHECK(db.get(&cnt, n + 1));
  DB_CHECK(db.get(&cp, n + 1));
  if (n)
    hipLaunchKernelGGL(k_scale_count, dim3((n + 255) / 256), dim3(256), 0, s, A->indptr,
                       A->indices, A->data, d, n, mode, cnt);
  MLAMG_TRY(exclusive_scan_i32(cnt, cp, n, s));
  int32_t nnz = 0;
  DB_CHECK(hipMemcpyAsync(&nnz, cp + n, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  DB_CHECK(hipStreamSynchronize(s));
  mlamg_csr* C = nullptr;
  MLAMG_TRY(csr_alloc(n, A->n_cols, nnz, &C));
  if (hipMemcpyAsync(C->indptr, cp, sizeof(int32_t) * (n + 1), hipMemcpyDeviceToDevice, s) !=
      hipSuccess) {
    csr_free(C);
    set_error("scale_rows: copy failed");
    return MLAMG_EHIP;
  }
  if (n)
    hipLaunchKernelGGL(k_scale_fill, dim3((n + 255) / 256), dim3(256), 0, s, A->indptr,
                       A->indices, A->data, d, n, mode, cp, C->indices, C->data);
  int rc = csr_finalize(C, s);
  if (rc != MLAMG_OK) {
    csr_free(C);
    return rc;
  }
  *out = C;
  return MLAMG_OK;
}

int diag_inv_impl(const mlamg_csr* A, double omega, double* dinv, hipStream_t s);

// ---------------------------------------------------------------- strength / distance maps
// mode 0 abs |a| (common.py:26; graph.py:204), 1 inverse 1/|a| (common.py:28; graph.py:206),
// 2 unit 1 (common.py:29; graph.py:202), 3 same a (graph.py:208)
__global__ void k_strength(const double* __restrict__ x, int64_t nnz, int mode,
                           double* __restrict__ y) {
  int64_t e = blockIdx.x * 256ll + threadIdx.x;
  if (e >= nnz) return;
  const double v = x[e];
  double r;
  switch (mode) {
    case 0: r = fabs(v); break;
    case 1: r = 1.0 / fabs(v); break;
    case 2: r = 1.0; break;
    default: r = v; break;
  }
  y[e] = r;
}

}  // namespace mlamg

using namespace mlamg;

extern "C" {

int mlamg_scratch_trim(size_t* freed_bytes) {
  ScratchPool& P = scratch_pool();
  std::lock_guard<std::mutex> lk(P.mu);
  size_t f = 0;
  for (auto& b : P.free_blocks) {
    (void)hipFree(b.second);
    f += b.first;
  }
  P.free_blocks.clear();
  P.cached = 0;
  if (freed_bytes) *freed_bytes = f;
  return MLAMG_OK;
}

int mlamg_setup_phase_times(double* ms_out, int n, int reset) {
  MLAMG_REQUIRE(ms_out && n >= 0, "NULL argument");
  std::lock_guard<std::mutex> lk(g_phase_mu);
  for (int i = 0; i < std::min(n, kPhases); ++i) ms_out[i] = g_phase_ms[i];
  if (reset)
    for (int i = 0; i < kPhases; ++i) g_phase_ms[i] = 0.0;
  return MLAMG_OK;
}

int mlamg_transpose(const mlamg_csr* A, mlamg_csr** out, void* stream) {
  MLAMG_REQUIRE(A && out, "NULL argument");
  return transpose_impl(A, out, S(stream));
}

int mlamg_spgemm(const mlamg_csr* A, const mlamg_csr* B, mlamg_csr** out, void* stream) {
  MLAMG_REQUIRE(A && B && out, "NULL argument");
  return spgemm_impl(A, B, out, 1, S(stream));
}

int mlamg_galerkin(const mlamg_csr* R, const mlamg_csr* A, const mlamg_csr* P, mlamg_csr** out,
                   void* stream) {
  MLAMG_REQUIRE(R && A && P && out, "NULL argument");
  MLAMG_REQUIRE(R->n_cols == A->n_rows && A->n_cols == P->n_rows, "shape mismatch");
  mlamg_csr* M = nullptr;
  MLAMG_TRY(spgemm_impl(R, A, &M, 0, S(stream)));
  int rc = spgemm_impl(M, P, out, 0, S(stream));
  csr_free(M);
  return rc;
}

int mlamg_csr_scale_rows(const mlamg_csr* A, const double* d, int reverse, mlamg_csr** out,
                         void* stream) {
  MLAMG_REQUIRE(A && d && out, "NULL argument");
  MLAMG_REQUIRE(reverse == 0 || reverse == 1, "reverse must be 0 or 1");
  return scale_rows_impl(A, d, reverse ? 0 : 2, out, S(stream));
}

int mlamg_sa_smoother(const mlamg_csr* A, double omega, mlamg_csr** out, void* stream) {
  MLAMG_REQUIRE(A && out, "NULL argument");
  MLAMG_REQUIRE(A->n_rows == A->n_cols, "square matrix required");
  double* d = nullptr;
  MLAMG_HIP(hipMalloc(&d, sizeof(double) * std::max<int64_t>(A->n_rows, 1)));
  int rc = mlamg_diag_inv(A, omega, d, stream);
  if (rc == MLAMG_OK) rc = scale_rows_impl(A, d, 1, out, S(stream));
  (void)hipStreamSynchronize(S(stream));
  (void)hipFree(d);
  return rc;
}

int mlamg_strength(const mlamg_csr* A, int mode, mlamg_csr** out, void* stream) {
  MLAMG_REQUIRE(A && out, "NULL argument");
  MLAMG_REQUIRE(mode >= 0 && mode <= 3, "mode must be 0 abs, 1 inv, 2 unit, 3 same");
  hipStream_t s = S(stream);
  mlamg_csr* C = nullptr;
  MLAMG_TRY(csr_alloc(A->n_rows, A->n_cols, A->nnz, &C));
  hipError_t e =
      hipMemcpyAsync(C->indptr, A->indptr, sizeof(int32_t) * (A->n_rows + 1), hipMemcpyDeviceToDevice, s);
  if (e == hipSuccess && A->nnz)
    e = hipMemcpyAsync(C->indices, A->indices, sizeof(int32_t) * A->nnz, hipMemcpyDeviceToDevice, s);
  if (e != hipSuccess) {
    csr_free(C);
    set_error("strength: copy failed");
    return MLAMG_EHIP;
  }
  if (A->nnz)
    hipLaunchKernelGGL(k_strength, dim3((A->nnz + 255) / 256), dim3(256), 0, s, A->data, A->nnz,
                       mode, C->data);
  int rc = csr_finalize(C, s);
  if (rc != MLAMG_OK) {
    csr_free(C);
    return rc;
  }
  *out = C;
  return MLAMG_OK;
}

}  // extern "C"
