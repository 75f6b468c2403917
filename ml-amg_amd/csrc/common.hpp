// Internal types and helpers of libmlamg_hip (gfx950 / MI355X).
//
// Device-resident CSR handle, error plumbing for the C-ABI (include/mlamg.h), launch helpers.
// Every floating-point kernel is compiled with -ffp-contract=off so that each multiply and add
// rounds exactly like scipy's sparsetools loops (no FMA contraction); this is what makes the
// SpMV / residual / Jacobi / restriction / prolongation results bitwise identical to the reference
// CPU path (ns/lib/multigrid.py:44,181,191; ns/preconditioner/MLAMG.py:145,191,194).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>
#include "../../include/mlamg.h"

namespace mlamg {

// ---------------------------------------------------------------- errors
void set_error(const std::string& msg);
const char* get_error();

#define MLAMG_HIP(call)                                                              \
  do {                                                                               \
    hipError_t _e = (call);                                                          \
    if (_e != hipSuccess) {                                                          \
      ::mlamg::set_error(std::string(#call) + " failed: " + hipGetErrorString(_e) +  \
                         " (" + __FILE__ + ":" + std::to_string(__LINE__) + ")");    \
      return MLAMG_EHIP;                                                             \
    }                                                                                \
  } while (0)

#define MLAMG_REQUIRE(cond, msg)                                                     \
  do {                                                                               \
    if (!(cond)) {                                                                   \
      ::mlamg::set_error(std::string(__func__) + ": " + (msg));                      \
      return MLAMG_EINVAL;                                                           \
    }                                                                                \
  } while (0)

#define MLAMG_TRY(call)                                                              \
  do {                                                                               \
    int _rc = (call);                                                                \
    if (_rc != MLAMG_OK) return _rc;                                                 \
  } while (0)

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ---------------------------------------------------------------- device allocations
// Every device buffer of the library comes from a size-class cache (runtime.cpp): a hipFree
// unmaps the pages, ~1 ms per buffer on MI355X, and one two-level amg_2_v call creates and
// drops ~60 buffers (55 ms of hipFree at 320^2 against a 95 ms call). A released block keeps
// hipFree's ordering (the device is synchronised before the block can be handed out again)
// and stays mapped for the next allocation of its size class; the cache holds at most
// MLAMG_DEVICE_CACHE_MB (default 8192) MiB and is flushed when an allocation fails; blocks above
// MLAMG_DEVICE_CACHE_MAX_BLOCK_MB (default 16) MiB are plain hipMalloc / hipFree.
hipError_t cached_malloc(void** p, size_t bytes);
hipError_t cached_free(void* p);
template <class T>
inline hipError_t cached_malloc_t(T** p, size_t bytes) {
  return cached_malloc(reinterpret_cast<void**>(p), bytes);
}
#define hipMalloc(p, bytes) ::mlamg::cached_malloc_t((p), (bytes))
#define hipFree(p) ::mlamg::cached_free((void*)(p))

// ---------------------------------------------------------------- CSR-stream geometry
// A row block = up to kBlockRows consecutive rows whose nonzeros (<= kBlockNnz) are staged
// through LDS by one 256-thread workgroup; a row longer than kBlockNnz gets a block of its own
// and is streamed in kBlockNnz chunks.
constexpr int kThreads = 256;
constexpr int kBlockRows = 256;
constexpr int kBlockNnz = 2048;   // 16 KiB of fp64 products in LDS per workgroup
// "sorted" format blocks: 512-thread workgroups, 32 KiB of products; 12 slot bits leave 20 bits
// of column offset, so a block's columns must span < 2^20
#ifndef MLAMG_SRT_THREADS  // build-time A/B knob (measured: 256 is 2-10 % slower than 512)
#define MLAMG_SRT_THREADS 512
#endif
#ifndef MLAMG_SRT_RPT  // rows per thread in the sorted kernel's phase 2 (2: C4 P0 102 -> 77 us; 1 for A/B)
#define MLAMG_SRT_RPT 2
#endif
constexpr int kSrtThreads = MLAMG_SRT_THREADS;
constexpr int kSrtRows = MLAMG_SRT_THREADS * MLAMG_SRT_RPT;
constexpr int kSrtNnz = 8 * MLAMG_SRT_THREADS;
constexpr int kSrtPosBits = 12;
// operators averaging at least this many entries per row take the sorted kernel's long-row
// instantiation (two rows summed side by side per thread)
#ifndef MLAMG_SRT_LONG_ROW  // build-time A/B knob
#define MLAMG_SRT_LONG_ROW 32.0
#endif
constexpr double kSrtLongRow = MLAMG_SRT_LONG_ROW;
// "long" format tiles (long-row coarse operators: Galerkin A_l, R = P^T): 256-thread
// workgroups, <= kLongNnz fp64 products in LDS, <= kLongRows rows per tile (one lane each)
constexpr int kLongNnz = 4096;
constexpr int kLongRows = 64;

// Row-pair pattern LDS windows (spmv.hip k_rowpair_win): cluster k of the wide entries' offsets
// is staged as rows [R0 + s[k], R0 + s[k] + len[k]) of x at window row base[k]
constexpr int kRpWinMax = 4;
constexpr int kRpWinNT = 256;        // pairs (threads) per workgroup
constexpr int kRpWinG = 2;           // global (unstaged) entries per kernel step at most
constexpr int kRpWinMaxRows = 4096;  // 32 KiB of LDS
struct RpWin {
  int32_t n = 0, rows = -1, nt = 256, woff0 = -1;
  int32_t s[kRpWinMax] = {0, 0, 0, 0}, len[kRpWinMax] = {0, 0, 0, 0},
          base[kRpWinMax] = {0, 0, 0, 0};
};

// Uniform row-pair stencils (spmv.hip k_rowpat_uni): every pattern entry is one of k <= 8
// column offsets with one value per (offset, row parity); offsets within +-halo rows read x from
// an LDS window of the workgroup's rows, the rest (at most kRpUniFar) are global loads
constexpr int kRpUniMax = 8;
constexpr int kRpUniFar = 2;
constexpr int kRpUniMaxHalo = 512;  // rows staged on each side of a workgroup's rows, at most
struct RpUni {
  int32_t k = 0;       // slots (0: not uniform)
  int32_t halo = 0;    // staged rows on each side (even)
  int32_t layout = 0;  // compile-time slot layout of k_rowpat_uni (0: run-time kinds)
  int32_t ch = 4;      // 256-pair chunks per workgroup (1, 2 or 4)
  int32_t off[kRpUniMax] = {0, 0, 0, 0, 0, 0, 0, 0};   // slot column offsets, ascending
  int32_t kind[kRpUniMax] = {0, 0, 0, 0, 0, 0, 0, 0};  // 0 even window offset, 1 offset -1,
                                                       // 2 offset +1, 3 global (far)
  double v0[kRpUniMax] = {0, 0, 0, 0, 0, 0, 0, 0};     // row 2i's value at each slot
  double v1[kRpUniMax] = {0, 0, 0, 0, 0, 0, 0, 0};     // row 2i+1's
  // far slot t (in slot order) reads x at pair offset alt_off[t] instead of its own offset for
  // the pairs [alt_lo[t], alt_hi[t]) — a row-partitioned slab's ghost plane (its x_ext position
  // is not the plane's global offset; build_rowpat). Empty range: none.
  int32_t alt_off[kRpUniFar] = {0, 0};
  int32_t alt_lo[kRpUniFar] = {0, 0};
  int32_t alt_hi[kRpUniFar] = {0, 0};
};

// Tolerance arguments: tol >= 0 arms the device stop flag with ||.|| <= tol (the reference's
// `e <= tol`, ns/lib/multigrid.py:197, MLAMG.py:194 — tol = 0 included: an exactly zero norm
// stops); a negative tol means "no tolerance" (run every requested cycle).
constexpr double kNoTol = -1.0;

}  // namespace mlamg

// Device CSR matrix. int32 indptr/indices, fp64 values (scipy's choice for these sizes:
// SURVEY.md §8a). Column indices are sorted within rows unless `sorted` is false.
struct mlamg_csr {
  int64_t n_rows = 0, n_cols = 0, nnz = 0;
  int32_t* indptr = nullptr;
  int32_t* indices = nullptr;
  double* data = nullptr;
  bool owns = true;
  int device = 0;
  // CSR-stream row-block partition (device + host copies)
  int32_t n_blocks = 0;
  int32_t* blk = nullptr;             // n_blocks+1 row boundaries
  std::vector<int32_t> blk_host;
  int32_t max_row_len = 0;
  double avg_row_len = 0.0;
  // optional SELL-64 copy (slices of 64 consecutive rows stored column-major, padded to the
  // slice's longest row with col = -1); used by the SpMV family when present
  int64_t n_slices = 0;
  int64_t* sell_ptr = nullptr;  // element offset of each slice (n_slices+1)
  int32_t* sell_col = nullptr;
  double* sell_val = nullptr;
  int32_t* sell_perm = nullptr;  // SELL-C-sigma row order (nullptr: natural order)
  int32_t sell_sigma = 0;
  int64_t sell_elems = 0;
  // optional dictionary-coded SELL ("sell_dict"): same slices, each element a uint16 code
  // (offset index | value index << 8) into <= 255 distinct column offsets (col - row) and <= 256
  // distinct values (bit patterns); code & 0xFF == 0xFF marks padding. Lossless: products and
  // their order are those of SELL. sell_col/sell_val are dropped while it is active.
  uint16_t* dict_code = nullptr;
  int64_t* dict_ptr = nullptr;   // code offset of each slice: rows padded to 8 codes, stored
                                 // [group of 8][lane][8] so a lane reads 8 codes in one 16-B load
  int32_t* dict_off = nullptr;   // 256 offsets
  double* dict_val = nullptr;    // 256 values
  int32_t dict_n_off = 0, dict_n_val = 0;
  // CSR-vector format (the canonical 512-virtual-lane order, spmv.hip k_csr_vcan): 0 = off,
  // else the number of lanes per row (64..512)
  int32_t vec_width = 0;
  // its column indices as 16-bit copies when n_cols <= 65536 (10 instead of 12 B per nonzero)
  uint16_t* vec_idx16 = nullptr;
  // optional gather-sorted copy ("sorted" format): row blocks of <= kSrtRows rows and
  // <= kSrtNnz nonzeros whose entries are stored in ascending column order, each packed as
  // (col - srt_base[block]) << kSrtPosBits | slot (its CSR position inside the block)
  int32_t srt_nb = 0;
  int32_t* srt_blk = nullptr;   // srt_nb+1 row boundaries
  int32_t* srt_base = nullptr;  // per block {r0, r1, e0, nnz, lo, hi, split, 0}: rows, entries
                                // and the column windows of the sorted entries
  uint32_t* srt_pk = nullptr;
  double* srt_val = nullptr;
  // value dictionary of the sorted copy (<= 256 distinct values, e.g. SA prolongators of
  // constant-coefficient stencils): srt_vi[e] indexes srt_vtab and srt_val is dropped
  uint8_t* srt_vi = nullptr;
  double* srt_vtab = nullptr;
  // block value dictionaries of the sorted copy (set_format(SORTED, 2): operators whose row
  // blocks repeat values, e.g. the Galerkin A_1 of a constant stencil, ~1,700 distinct values
  // per 4,096-entry block): block b's distinct values are srt_vtab[srt_vblk[2b] ..
  // + srt_vblk[2b+1]) and srt_vc[e] indexes them. srt_val is dropped.
  uint16_t* srt_vc = nullptr;
  int32_t* srt_vblk = nullptr;
  int64_t srt_vtab_n = 0;
  // optional row-pair pattern copy ("rowpat" format): every pair of rows (2i, 2i+1) is one of
  // <= 255 distinct pair patterns (the merge by column offset of the two rows' (col - row,
  // value) sequences), kept in LDS tables; the matrix stream is one byte per pair.
  // Constant-coefficient stencils only (C4: 27 pair patterns).
  uint8_t* rp_pid = nullptr;     // pattern id of each pair
  int32_t* rp_ptr = nullptr;     // 257 pattern starts into the entry arrays
  int32_t* rp_off = nullptr;     // per entry (column offset col - row, row 2i mask, row 2i+1
                                 // mask, flags: bit 0/1 = entry of row 2i/2i+1, bit 2 = "wide");
                                 // patterns padded to multiples of 8 entries
  double* rp_val = nullptr;      // per entry (row 2i's value, row 2i+1's value)
  int32_t rp_n_pat = 0, rp_n_ent = 0;
  int32_t rp_k = 8;                    // entries per kernel step (patterns padded to multiples)
  mlamg::RpWin rp_win;                 // LDS row windows of k_rowpair_win (rows < 0: none)
  uint16_t* rp_slot = nullptr;         // its slot order: pattern | local pair << 8, per workgroup
                                       // sorted by pattern
  std::vector<int32_t> rp_rep;         // representative pair of each pattern (host)
  mlamg::RpUni rp_uni;                 // uniform-stencil form (k_rowpat_uni; k == 0: none)
  uint16_t* rp_msk = nullptr;          // its per-pattern slot masks (row 2i | row 2i+1 << 8)
  int32_t rp_lds_pad = 0;              // extra LDS bytes per workgroup (occupancy cap, A/B knob)
  // plane-marching form of a uniform 3-D 7-point stencil (k_rowpat_march; rp_mF == 0: none):
  // far offset +-rp_mF (one grid plane), chunks per tile, planes per z segment
  int64_t rp_mF = 0;
  int32_t rp_mch = 4, rp_mseg = 0, rp_mpf = 1;
  // attached Jacobi weights (mlamg_csr_attach_dinv): an epilogue whose dinv pointer equals
  // rp_dinv_att reads the per-pattern values rp_dinv[2p], rp_dinv[2p+1] instead of memory
  const double* rp_dinv_att = nullptr;
  double* rp_dinv = nullptr;
  // optional long-row tiling ("long" format): tiles of consecutive rows (<= kLongRows rows,
  // <= kLongNnz nonzeros, or one longer row streamed in chunks) over the CSR arrays themselves;
  // every row summed left to right by one lane (scipy's order) from LDS products
  int32_t lg_nt = 0;
  int32_t* lg_tile = nullptr;  // lg_nt+1 row boundaries
  // number of per-block partial sums a NORM launch writes with the active format
  int32_t n_part = 0;
};

// Dense coarse-level inverse (dense.hip)
struct mlamg_dense {
  int64_t n = 0;
  double* inv = nullptr;  // row-major n x n
  int method = 0;  // 0 Gauss-Jordan, 1 inverse Cholesky factor (A^-1 = X^T X), 2 the factor X
                   // (lower) with X^T (strict upper) applied as two triangular passes (dense.hip)
  double* y = nullptr;  // method 2: the intermediate X b
};

namespace mlamg {
// s = p[start] + p[start+step] + ... in that order (bitwise a plain strided loop), with the loads
// issued 8 at a time: a one-workgroup reduction over tens of thousands of partials is otherwise
// a chain of dependent memory round trips.
__device__ __forceinline__ double strided_sum(const double* __restrict__ p, int n, int start,
                                              int step) {
  double s = 0.0;
  int i = start;
  for (; i + 7 * step < n; i += 8 * step) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = p[i + u * step];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; i < n; i += step) s += p[i];
  return s;
}
}  // namespace mlamg

namespace mlamg {
// Upper bound on the per-block partial sums a NORM launch of A can write, whatever format is
// active (CSR-stream: n_blocks; SELL-64: n/256; CSR-vector: n*VW/256 <= n/4), plus one slot.
// Wide CSR-vector widths (128..512 lanes per row, one workgroup of 512 lanes) write one partial
// per 512/VW rows; they are only accepted on operators with at most kWideMaxRows rows.
constexpr int64_t kWideMaxRows = int64_t(1) << 20;
inline int64_t part_capacity(const mlamg_csr* A) {
  int64_t c = std::max<int64_t>(std::max<int64_t>(A->n_blocks, A->srt_nb), (A->n_rows + 3) / 4);
  c = std::max<int64_t>(c, A->lg_nt);
  if (A->n_rows <= kWideMaxRows) c = std::max<int64_t>(c, A->n_rows);
  return c + 2;
}
// Allocate device arrays for an (n_rows x n_cols, nnz) CSR and the handle; no partition yet.
int csr_alloc(int64_t n_rows, int64_t n_cols, int64_t nnz, mlamg_csr** out);
// Build the CSR-stream row-block partition from the device indptr (syncs `stream`).
int csr_finalize(mlamg_csr* A, hipStream_t stream);
void csr_free(mlamg_csr* A);
int transpose_impl(const mlamg_csr* A, mlamg_csr** out, hipStream_t s);

// scratch buffer cache (per device); grows monotonically, freed at destroy/exit.
void* scratch(size_t bytes, int slot);

// bumped by every mlamg_csr_set_format: captured hipGraphs bake kernel choice and format
// arrays in, so graph caches compare it and re-capture after a change.
uint64_t format_epoch();
void bump_format_epoch();

// Dispatch-packet kernel timing (mlamg_timer_*, runtime.cpp): while a timer is armed on this
// thread, the next SpMV-family launch (MLAMG_LAUNCH) carries the timer's two events in its own
// dispatch packet (hipExtLaunchKernel) and disarms it. Their interval is then the kernel's
// execution alone — what rocprofv3's kernel trace reports — instead of event packet + dispatch
// + kernel, which is what a pair of stream events around the call measures.
struct LaunchTimer {
  hipEvent_t start = nullptr, stop = nullptr;
  bool taken = false;  // a launch recorded the events since the last arm
};
LaunchTimer* take_armed_timer(hipStream_t s);
#define MLAMG_LAUNCH(K, G, B, L, S, ...)                                             \
  do {                                                                               \
    if (::mlamg::LaunchTimer* lt_ = ::mlamg::take_armed_timer(S))                    \
      hipExtLaunchKernelGGL(K, G, B, L, S, lt_->start, lt_->stop, 0, __VA_ARGS__);   \
    else                                                                             \
      hipLaunchKernelGGL(K, G, B, L, S, __VA_ARGS__);                                \
  } while (0)

// generic kernels shared across translation units
int launch_spmv_plain(const mlamg_csr* A, const double* x, double* y, hipStream_t s);
int exclusive_scan_i64(const int64_t* in, int64_t* out, int64_t n, hipStream_t s);  // out[n] = total
int exclusive_scan_i32(const int32_t* in, int32_t* out, int64_t n, hipStream_t s);
// entries of a[0..n) outside [lo, hi) (device check before any kernel indexes with them); syncs
// V-cycle building blocks (spmv.hip, vec.hip, dense.hip, hier.hip), shared by the executors
int residual_impl(const mlamg_csr* A, const double* b, const double* x, double* r, double* norm2,
                  double* hist, int32_t* counter, int32_t* done, double tol, double* copy_to,
                  const double* copy_from, double* partial, hipStream_t s,
                  const double* smooth_dinv = nullptr);
int residual_partials(const mlamg_csr* A, const double* b, const double* x, double* r,
                      double* copy_to, const double* copy_from, double* partial,
                      const int32_t* done, hipStream_t s, const double* smooth_dinv = nullptr);
int jacobi_sweep(const mlamg_csr* A, const double* dinv, const double* b, const double* xin,
                 double* xout, bool explicit_form, const int32_t* done, hipStream_t s);
int spmv_add(const mlamg_csr* A, const double* x, double* y, const int32_t* done, hipStream_t s);
int spmv_fadd(const mlamg_csr* A, const int32_t* agg, const double* e, double* y,
              const double* dinv_w, const int32_t* done, hipStream_t s);
int spmv_set(const mlamg_csr* A, const double* x, double* y, const int32_t* done, hipStream_t s,
             double* smooth_x = nullptr, const double* smooth_dinv = nullptr);
int jacobi_from_residual(double* x, const double* dinv, const double* r, int64_t n,
                         const int32_t* done, hipStream_t s);
int jacobi_from_zero(double* x, const double* dinv, const double* b, int64_t n,
                     const int32_t* done, hipStream_t s);
int dense_solve_impl(const mlamg_dense* D, const double* b, double* x, const int32_t* done,
                     hipStream_t s);
// A^-1 of a dense row-major n x n operator (destroyed) through its inverse Cholesky factor on the
// whole GPU (dense.hip); *spd = false: not symmetric to rounding / not SPD, inv not written
int dense_chol_inverse(double* M, int64_t n, double* inv, bool* spd, hipStream_t s);
// the same for many operators in one launch sequence (Lp, Zd, flag filled in here); spd[j] per job
struct DenseJob {
  double* M;
  double* inv;
  double* Lp;
  double* Zd;
  int32_t* flag;
  int64_t n;
};
int dense_chol_inverse_batch(const DenseJob* jobs, int count, bool* spd, hipStream_t s);
int hier_coarse_cycle(mlamg_hier* H, const double* b, double** x_out, int use_graph,
                      hipStream_t s);
int32_t* hier_done_flag(mlamg_hier* H);
int64_t hier_fine_rows(const mlamg_hier* H);
// H's Krylov workspace of at least `bytes` (kept across calls, freed with H)
int hier_workspace(mlamg_hier* H, size_t bytes, void** out);
// coarsest solve by inner-hierarchy PCG (pcg.hip)
int pcg_solve_impl(mlamg_pcg* C, const double* b, double* x, const int32_t* outer_done,
                   hipStream_t s);
int64_t pcg_rows(const mlamg_pcg* C);
mlamg_hier* pcg_inner(mlamg_pcg* C);
// restarted left-preconditioned GMRES (scipy's algorithm) with one V-cycle of M as
// preconditioner (gmres.hip); rel_out (optional): final ||b - A x|| / ||b||
int gmres_impl(const mlamg_csr* A, mlamg_hier* M, const double* b, double* x, double rtol,
               int restart, int maxiter, bool x_zero, int* info_out, int* iters_out,
               double* presid_hist, int hist_cap, hipStream_t s, double* rel_out = nullptr);
int hier_prepare_ext(mlamg_hier* H);
int gs_sweep_impl(const mlamg_gs* G, double* x, const double* b, int iterations,
                  const int32_t* done, hipStream_t s);
int64_t gs_rows(const mlamg_gs* G);
// ||x||_2 of one cycle into hist[*counter] (+ tolerance flag), like the residual-norm path
int norm_hist_impl(const double* x, int64_t n, double* partial, double* hist, int32_t* counter,
                   int32_t* done, double tol, hipStream_t s);
int count_out_of_range(const int32_t* a, int64_t n, int64_t lo, int64_t hi, hipStream_t s,
                       int64_t* bad_out);
// Cycles are launched in batches; with a tolerance, the device-side stop flag is read back
// after each batch so the cycles after convergence are not launched at all (each would only
// check the flag and return, ~10 launches apiece). Batches grow 4, 4, 8, 16, 32, 32, ...: at
// most one batch of overshoot, a host sync per batch.
template <class F>
static int run_cycles(int n_cycles, double tol, int32_t* done_dev, int32_t* done_host,
                      hipStream_t s, F&& one) {
  if (!(tol >= 0.0) || !done_host) {
    for (int c = 0; c < n_cycles; ++c) MLAMG_TRY(one());
    return MLAMG_OK;
  }
  int c = 0, batch = 4, k = 0;
  while (c < n_cycles) {
    const int m = std::min(batch, n_cycles - c);
    for (int i = 0; i < m; ++i) MLAMG_TRY(one());
    c += m;
    if (c >= n_cycles) break;
    MLAMG_HIP(hipMemcpyAsync(done_host, done_dev, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    MLAMG_HIP(hipStreamSynchronize(s));
    if (*done_host) break;
    if (++k >= 2) batch = std::min(batch * 2, 32);
  }
  return MLAMG_OK;
}
}  // namespace mlamg
