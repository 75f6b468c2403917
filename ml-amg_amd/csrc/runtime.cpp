// Runtime pieces of libmlamg_hip: error state, device CSR handle lifecycle, CSR-stream
// partitioning, scratch buffers. Host C++ compiled by hipcc; no torch dependency.
#include "common.hpp"

#include <atomic>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <unordered_map>

namespace mlamg {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
const char* get_error() { return g_last_error.c_str(); }

// ---------------------------------------------------------------- device allocation cache
// Size classes: powers of two up to 1 MiB, then 8 steps per power of two (<= 12.5 % slack).
namespace {
size_t size_class(size_t b) {
  b = std::max<size_t>(b, 256);
  size_t p2 = 256;
  while (p2 < b) p2 <<= 1;
  if (p2 <= (size_t(1) << 20)) return p2;
  const size_t step = p2 >> 4;  // p2 / 2 < b <= p2: steps of p2 / 16
  return (b + step - 1) / step * step;
}
struct DevCache {
  std::mutex mu;
  std::unordered_map<void*, std::pair<int, size_t>> live;         // ptr -> (device, class)
  std::map<std::pair<int, size_t>, std::vector<void*>> free_list;  // (device, class) -> blocks
  size_t cached = 0, limit = 0, max_block = 0;
  int64_t hits = 0, misses = 0;
  DevCache() {
    const char* e = std::getenv("MLAMG_DEVICE_CACHE_MB");
    // bounded well below what a torch process may need: torch's allocator cannot reclaim these
    // blocks (mlamg_device_cache_trim gives them back; an OOM in this library flushes them)
    limit = (e ? (size_t)std::strtoull(e, nullptr, 10) : size_t(2048)) << 20;
    // blocks above this size bypass the cache (allocated at their exact size, really freed):
    // the hierarchy's large operators and vectors then sit where a plain hipMalloc puts them
    // (the C4 bench cycle measured 1-3 % slower on recycled, class-rounded blocks), while the
    // many small buffers of a two-level call, whose hipFree cost dominates, are cached
    const char* m = std::getenv("MLAMG_DEVICE_CACHE_MAX_BLOCK_MB");
    max_block = (m ? (size_t)std::strtoull(m, nullptr, 10) : size_t(16)) << 20;
  }
  // really free every cached block (caller holds mu)
  size_t flush() {
    size_t n = 0;
    for (auto& kv : free_list) {
      int cur = 0;
      (void)hipGetDevice(&cur);
      (void)hipSetDevice(kv.first.first);
      for (void* q : kv.second) {
        (void)(hipFree)(q);
        n += kv.first.second;
      }
      (void)hipSetDevice(cur);
    }
    free_list.clear();
    cached = 0;
    return n;
  }
};
DevCache& dev_cache() {
  static DevCache* c = new DevCache();  // never destroyed: thread-exit frees may come late
  return *c;
}
}  // namespace

hipError_t cached_malloc(void** p, size_t bytes) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  DevCache& c = dev_cache();
  if (bytes > c.max_block) {  // not tracked: cached_free frees it
    e = (hipMalloc)(p, bytes);
    if (e == hipSuccess) return e;
    // out of memory: the cached small blocks (up to the cap) may be what is missing
    (void)hipGetLastError();
    std::lock_guard<std::mutex> lk(c.mu);
    if (c.flush() == 0) return e;
    return (hipMalloc)(p, bytes);
  }
  const size_t cls = size_class(bytes);
  std::lock_guard<std::mutex> lk(c.mu);
  auto it = c.free_list.find({dev, cls});
  if (it != c.free_list.end() && !it->second.empty()) {
    *p = it->second.back();
    it->second.pop_back();
    c.cached -= cls;
    c.live[*p] = {dev, cls};
    ++c.hits;
    return hipSuccess;
  }
  e = (hipMalloc)(p, cls);
  if (e != hipSuccess) {  // out of memory: give the cached blocks back and retry once
    (void)hipGetLastError();
    if (c.flush() == 0) return e;
    e = (hipMalloc)(p, cls);
    if (e != hipSuccess) return e;
  }
  c.live[*p] = {dev, cls};
  ++c.misses;
  return hipSuccess;
}

hipError_t cached_free(void* p) {
  if (!p) return hipSuccess;
  DevCache& c = dev_cache();
  std::pair<int, size_t> key;
  {
    std::lock_guard<std::mutex> lk(c.mu);
    auto it = c.live.find(p);
    if (it == c.live.end()) return (hipFree)(p);  // not ours
    key = it->second;
    c.live.erase(it);
  }
  // hipFree's ordering: no kernel still in flight may see the block handed out again. The
  // lock is not held here, so other host threads (one per rank in the loopback executor) keep
  // allocating and launching while this one waits.
  int cur = 0;
  (void)hipGetDevice(&cur);
  if (cur != key.first) (void)hipSetDevice(key.first);
  hipError_t e = hipDeviceSynchronize();
  if (cur != key.first) (void)hipSetDevice(cur);
  std::lock_guard<std::mutex> lk(c.mu);
  if (e != hipSuccess || c.cached + key.second > c.limit) return (hipFree)(p);
  c.free_list[key].push_back(p);
  c.cached += key.second;
  return hipSuccess;
}

size_t device_cache_trim() {
  DevCache& c = dev_cache();
  std::lock_guard<std::mutex> lk(c.mu);
  (void)hipDeviceSynchronize();
  return c.flush();
}

void device_cache_stats(size_t* cached, int64_t* hits, int64_t* misses) {
  DevCache& c = dev_cache();
  std::lock_guard<std::mutex> lk(c.mu);
  if (cached) *cached = c.cached;
  if (hits) *hits = c.hits;
  if (misses) *misses = c.misses;
}

// ---------------------------------------------------------------- scratch
// Per host thread: work submitted from different threads (one stream each, e.g. concurrent
// independent solves) never shares a scratch buffer; calls from one thread are stream-ordered.
namespace {
struct Scratch {
  void* p = nullptr;
  size_t bytes = 0;
};
struct ScratchCache {
  std::vector<std::vector<Scratch>> v;  // [device][slot]
  ~ScratchCache() {
    for (auto& d : v)
      for (auto& s : d)
        if (s.p) (void)hipFree(s.p);
  }
};
thread_local ScratchCache g_scratch_tl;
}  // namespace

void* scratch(size_t bytes, int slot) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  auto& g_scratch = g_scratch_tl.v;
  if ((int)g_scratch.size() <= dev) g_scratch.resize(dev + 1);
  auto& v = g_scratch[dev];
  if ((int)v.size() <= slot) v.resize(slot + 1);
  Scratch& s = v[slot];
  if (s.bytes < bytes) {
    if (s.p) {
      (void)hipDeviceSynchronize();
      (void)hipFree(s.p);
    }
    s.p = nullptr;
    s.bytes = 0;
    size_t want = std::max<size_t>(bytes, 256);
    if (hipMalloc(&s.p, want) != hipSuccess) return nullptr;
    s.bytes = want;
  }
  return s.p;
}

// ---------------------------------------------------------------- CSR handle
int csr_alloc(int64_t n_rows, int64_t n_cols, int64_t nnz, mlamg_csr** out) {
  MLAMG_REQUIRE(out != nullptr, "out is NULL");
  MLAMG_REQUIRE(n_rows >= 0 && n_cols >= 0 && nnz >= 0, "negative size");
  MLAMG_REQUIRE(n_rows < (int64_t(1) << 31) - 1 && n_cols < (int64_t(1) << 31) - 1,
                "dimension exceeds int32 index range");
  MLAMG_REQUIRE(nnz < (int64_t(1) << 31) - 1, "nnz exceeds int32 indptr range");
  auto* A = new mlamg_csr();
  A->n_rows = n_rows;
  A->n_cols = n_cols;
  A->nnz = nnz;
  A->owns = true;
  (void)hipGetDevice(&A->device);
  if (hipMalloc(&A->indptr, sizeof(int32_t) * (n_rows + 1)) != hipSuccess ||
      hipMalloc(&A->indices, sizeof(int32_t) * std::max<int64_t>(nnz, 1)) != hipSuccess ||
      hipMalloc(&A->data, sizeof(double) * std::max<int64_t>(nnz, 1)) != hipSuccess) {
    csr_free(A);
    set_error("csr_alloc: hipMalloc failed (out of device memory?)");
    return MLAMG_ENOMEM;
  }
  *out = A;
  return MLAMG_OK;
}

void csr_free(mlamg_csr* A) {
  if (!A) return;
  if (A->owns) {
    if (A->indptr) (void)hipFree(A->indptr);
    if (A->indices) (void)hipFree(A->indices);
    if (A->data) (void)hipFree(A->data);
  }
  if (A->blk) (void)hipFree(A->blk);
  if (A->sell_ptr) (void)hipFree(A->sell_ptr);
  if (A->sell_col) (void)hipFree(A->sell_col);
  if (A->sell_val) (void)hipFree(A->sell_val);
  if (A->sell_perm) (void)hipFree(A->sell_perm);
  if (A->dict_code) (void)hipFree(A->dict_code);
  if (A->dict_ptr) (void)hipFree(A->dict_ptr);
  if (A->dict_off) (void)hipFree(A->dict_off);
  if (A->dict_val) (void)hipFree(A->dict_val);
  if (A->srt_blk) (void)hipFree(A->srt_blk);
  if (A->srt_base) (void)hipFree(A->srt_base);
  if (A->srt_pk) (void)hipFree(A->srt_pk);
  if (A->srt_val) (void)hipFree(A->srt_val);
  if (A->srt_vi) (void)hipFree(A->srt_vi);
  if (A->srt_vtab) (void)hipFree(A->srt_vtab);
  if (A->srt_vc) (void)hipFree(A->srt_vc);
  if (A->srt_vblk) (void)hipFree(A->srt_vblk);
  if (A->vec_idx16) (void)hipFree(A->vec_idx16);
  if (A->rp_pid) (void)hipFree(A->rp_pid);
  if (A->rp_ptr) (void)hipFree(A->rp_ptr);
  if (A->rp_off) (void)hipFree(A->rp_off);
  if (A->rp_val) (void)hipFree(A->rp_val);
  if (A->rp_dinv) (void)hipFree(A->rp_dinv);
  if (A->rp_slot) (void)hipFree(A->rp_slot);
  if (A->rp_msk) (void)hipFree(A->rp_msk);
  if (A->lg_tile) (void)hipFree(A->lg_tile);
  delete A;
}

// Greedy row-block partition for the CSR-stream kernels: consecutive rows while the block has
// <= kBlockRows rows and <= kBlockNnz nonzeros; an over-long row gets a block of its own.
int csr_finalize(mlamg_csr* A, hipStream_t stream) {
  const int64_t n = A->n_rows;
  std::vector<int32_t> ip(n + 1);
  MLAMG_HIP(hipMemcpyAsync(ip.data(), A->indptr, sizeof(int32_t) * (n + 1), hipMemcpyDeviceToHost,
                           stream));
  MLAMG_HIP(hipStreamSynchronize(stream));
  MLAMG_REQUIRE(ip[0] == 0, "indptr[0] != 0");
  MLAMG_REQUIRE(ip[n] == A->nnz, "indptr[n] != nnz");
  int64_t bad = 0;
  MLAMG_TRY(count_out_of_range(A->indices, A->nnz, 0, A->n_cols, stream, &bad));
  MLAMG_REQUIRE(bad == 0, "column index out of range [0, n_cols)");
  std::vector<int32_t>& blk = A->blk_host;
  blk.clear();
  blk.reserve(n / 64 + 2);
  blk.push_back(0);
  int32_t maxlen = 0;
  int64_t r = 0;
  while (r < n) {
    int32_t len = ip[r + 1] - ip[r];
    MLAMG_REQUIRE(len >= 0, "indptr not monotone");
    if (len > kBlockNnz) {
      maxlen = std::max(maxlen, len);
      ++r;
      blk.push_back((int32_t)r);
      continue;
    }
    int64_t start = r;
    int64_t nz = 0;
    while (r < n && r - start < kBlockRows) {
      len = ip[r + 1] - ip[r];
      MLAMG_REQUIRE(len >= 0, "indptr not monotone");
      if (nz + len > kBlockNnz) break;
      maxlen = std::max(maxlen, len);
      nz += len;
      ++r;
    }
    blk.push_back((int32_t)r);
  }
  A->n_blocks = (int32_t)(blk.size() - 1);
  A->n_part = A->n_blocks;
  A->max_row_len = maxlen;
  A->avg_row_len = n ? double(A->nnz) / double(n) : 0.0;
  if (A->blk) (void)hipFree(A->blk);
  A->blk = nullptr;
  MLAMG_HIP(hipMalloc(&A->blk, sizeof(int32_t) * blk.size()));
  MLAMG_HIP(hipMemcpyAsync(A->blk, blk.data(), sizeof(int32_t) * blk.size(),
                           hipMemcpyHostToDevice, stream));
  MLAMG_HIP(hipStreamSynchronize(stream));
  return MLAMG_OK;
}

}  // namespace mlamg

using namespace mlamg;

extern "C" {

int mlamg_version(void) { return 10000; /* 0.1.0 */ }
const char* mlamg_last_error(void) { return get_error(); }

int mlamg_set_device(int dev) {
  MLAMG_HIP(hipSetDevice(dev));
  return MLAMG_OK;
}
int mlamg_get_device(int* dev) {
  MLAMG_REQUIRE(dev, "dev is NULL");
  MLAMG_HIP(hipGetDevice(dev));
  return MLAMG_OK;
}
int mlamg_stream_sync(void* stream) {
  MLAMG_HIP(hipStreamSynchronize(S(stream)));
  return MLAMG_OK;
}

int mlamg_csr_create(int64_t n_rows, int64_t n_cols, int64_t nnz, const int32_t* indptr,
                     const int32_t* indices, const double* data, int where, mlamg_csr** out) {
  MLAMG_REQUIRE(out != nullptr, "out is NULL");
  MLAMG_REQUIRE(indptr != nullptr, "indptr is NULL");
  MLAMG_REQUIRE(nnz == 0 || (indices && data), "indices/data NULL with nnz > 0");
  MLAMG_REQUIRE(where >= 0 && where <= 2, "where must be 0 (host), 1 (device copy), 2 (wrap)");
  // int32 indptr/indices (scipy's choice below 2^31 nonzeros): larger operators would wrap
  MLAMG_REQUIRE(nnz <= INT32_MAX && n_rows < INT32_MAX && n_cols <= INT32_MAX,
                "nnz / n_rows / n_cols exceed the int32 index range of the CSR handle");
  hipStream_t s = nullptr;
  mlamg_csr* A = nullptr;
  if (where == MLAMG_WRAP_DEVICE) {
    MLAMG_REQUIRE(n_rows >= 0 && n_cols >= 0 && nnz >= 0, "negative size");
    A = new mlamg_csr();
    A->n_rows = n_rows;
    A->n_cols = n_cols;
    A->nnz = nnz;
    A->owns = false;
    (void)hipGetDevice(&A->device);
    A->indptr = const_cast<int32_t*>(indptr);
    A->indices = const_cast<int32_t*>(indices);
    A->data = const_cast<double*>(data);
  } else {
    MLAMG_TRY(csr_alloc(n_rows, n_cols, nnz, &A));
    hipMemcpyKind k = where == MLAMG_COPY_HOST ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice;
    hipError_t e = hipMemcpyAsync(A->indptr, indptr, sizeof(int32_t) * (n_rows + 1), k, s);
    if (e == hipSuccess && nnz)
      e = hipMemcpyAsync(A->indices, indices, sizeof(int32_t) * nnz, k, s);
    if (e == hipSuccess && nnz) e = hipMemcpyAsync(A->data, data, sizeof(double) * nnz, k, s);
    if (e != hipSuccess) {
      csr_free(A);
      set_error(std::string("mlamg_csr_create: copy failed: ") + hipGetErrorString(e));
      return MLAMG_EHIP;
    }
  }
  int rc = csr_finalize(A, s);
  if (rc != MLAMG_OK) {
    csr_free(A);
    return rc;
  }
  *out = A;
  return MLAMG_OK;
}

int mlamg_csr_destroy(mlamg_csr* A) {
  csr_free(A);
  return MLAMG_OK;
}

int mlamg_csr_shape(const mlamg_csr* A, int64_t* n_rows, int64_t* n_cols, int64_t* nnz) {
  MLAMG_REQUIRE(A, "A is NULL");
  if (n_rows) *n_rows = A->n_rows;
  if (n_cols) *n_cols = A->n_cols;
  if (nnz) *nnz = A->nnz;
  return MLAMG_OK;
}

int mlamg_csr_device_arrays(const mlamg_csr* A, int32_t** indptr, int32_t** indices,
                            double** data) {
  MLAMG_REQUIRE(A, "A is NULL");
  if (indptr) *indptr = A->indptr;
  if (indices) *indices = A->indices;
  if (data) *data = A->data;
  return MLAMG_OK;
}

int mlamg_csr_download(const mlamg_csr* A, int32_t* indptr_host, int32_t* indices_host,
                       double* data_host) {
  MLAMG_REQUIRE(A, "A is NULL");
  if (indptr_host)
    MLAMG_HIP(hipMemcpy(indptr_host, A->indptr, sizeof(int32_t) * (A->n_rows + 1),
                        hipMemcpyDeviceToHost));
  if (indices_host && A->nnz)
    MLAMG_HIP(hipMemcpy(indices_host, A->indices, sizeof(int32_t) * A->nnz,
                        hipMemcpyDeviceToHost));
  if (data_host && A->nnz)
    MLAMG_HIP(hipMemcpy(data_host, A->data, sizeof(double) * A->nnz, hipMemcpyDeviceToHost));
  return MLAMG_OK;
}

int mlamg_csr_copy_device(const mlamg_csr* A, int32_t* indptr, int32_t* indices, double* data,
                          void* stream) {
  MLAMG_REQUIRE(A, "A is NULL");
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (indptr)
    MLAMG_HIP(hipMemcpyAsync(indptr, A->indptr, sizeof(int32_t) * (A->n_rows + 1),
                             hipMemcpyDeviceToDevice, s));
  if (indices && A->nnz)
    MLAMG_HIP(hipMemcpyAsync(indices, A->indices, sizeof(int32_t) * A->nnz,
                             hipMemcpyDeviceToDevice, s));
  if (data && A->nnz)
    MLAMG_HIP(hipMemcpyAsync(data, A->data, sizeof(double) * A->nnz, hipMemcpyDeviceToDevice,
                             s));
  return MLAMG_OK;
}

}  // extern "C"

struct mlamg_timer {
  mlamg::LaunchTimer ev;
  bool used = false;
};

namespace mlamg {
static thread_local LaunchTimer* g_armed = nullptr;
LaunchTimer* take_armed_timer(hipStream_t s) {
  LaunchTimer* t = g_armed;
  if (!t) return nullptr;
  // a launch being captured into a graph must not carry the events
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &st) != hipSuccess || st != hipStreamCaptureStatusNone)
    return nullptr;
  g_armed = nullptr;
  t->taken = true;
  return t;
}
}  // namespace mlamg

extern "C" {
int mlamg_timer_create(mlamg_timer** out) {
  MLAMG_REQUIRE(out, "out is NULL");
  auto* t = new mlamg_timer();
  hipError_t e = hipEventCreate(&t->ev.start);
  if (e == hipSuccess) e = hipEventCreate(&t->ev.stop);
  if (e != hipSuccess) {
    if (t->ev.start) (void)hipEventDestroy(t->ev.start);
    delete t;
    set_error(std::string("mlamg_timer_create: ") + hipGetErrorString(e));
    return MLAMG_EHIP;
  }
  *out = t;
  return MLAMG_OK;
}
int mlamg_timer_destroy(mlamg_timer* t) {
  if (!t) return MLAMG_OK;
  if (g_armed == &t->ev) g_armed = nullptr;
  (void)hipEventDestroy(t->ev.start);
  (void)hipEventDestroy(t->ev.stop);
  delete t;
  return MLAMG_OK;
}
int mlamg_timer_arm(mlamg_timer* t) {
  MLAMG_REQUIRE(t, "t is NULL");
  t->used = true;
  t->ev.taken = false;
  g_armed = &t->ev;
  return MLAMG_OK;
}
int mlamg_timer_disarm(void) {
  g_armed = nullptr;
  return MLAMG_OK;
}
int mlamg_timer_elapsed_ms(mlamg_timer* t, float* ms) {
  MLAMG_REQUIRE(t && ms, "t / ms is NULL");
  MLAMG_REQUIRE(t->used && t->ev.taken && g_armed != &t->ev,
                "the timer was not armed, or no SpMV-family launch has consumed it");
  MLAMG_HIP(hipEventSynchronize(t->ev.stop));
  MLAMG_HIP(hipEventElapsedTime(ms, t->ev.start, t->ev.stop));
  return MLAMG_OK;
}
}  // extern "C"

namespace mlamg {
static std::atomic<uint64_t> g_format_epoch{0};
uint64_t format_epoch() { return g_format_epoch.load(); }
void bump_format_epoch() { g_format_epoch.fetch_add(1); }
}  // namespace mlamg

extern "C" int mlamg_device_cache_trim(size_t* freed_bytes) {
  const size_t n = mlamg::device_cache_trim();
  if (freed_bytes) *freed_bytes = n;
  return MLAMG_OK;
}

extern "C" int mlamg_device_cache_stats(size_t* cached_bytes, int64_t* hits, int64_t* misses) {
  mlamg::device_cache_stats(cached_bytes, hits, misses);
  return MLAMG_OK;
}
