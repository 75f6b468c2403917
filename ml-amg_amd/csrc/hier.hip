// Multilevel weighted-Jacobi V-cycle executor.
//
// Per level l < L (fine to coarse), one cycle is the reference two-level cycle
// (ns/preconditioner/MLAMG.py:189-195) with the coarse solve replaced by the next level:
//     x += Dinv_w (b - A x)          nu_pre times          MLAMG.py:143-146,190
//     b_{l+1} = R (b - A x)                                 MLAMG.py:191 (P.T @ (b - A@x))
//     x_{l+1} = cycle(l+1, x0 = 0)  / dense solve at L     MLAMG.py:191 (A_H_lu.solve)
//     x += P x_{l+1}                                        MLAMG.py:191
//     x += Dinv_w (b - A x)          nu_post times         MLAMG.py:192
// and at the finest level ||b - A x||_2 ends the cycle (MLAMG.py:194). That end-of-cycle
// residual is exactly what the next cycle's first pre-smoothing sweep recomputes, so it is kept
// and reused (same kernel, same bits), and the first sweep from a zero guess on coarse levels is
// x = Dinv_w b (0 + d*(b - A@0) bit for bit). The tolerance test runs on the device: the norm
// kernel raises a flag and every later kernel of the call returns immediately, so a whole batch
// of cycles is launched (or replayed from one captured hipGraph) without host round trips.
#include "common.hpp"

#include <hip/hip_runtime.h>

namespace {
struct Level {
  const mlamg_csr* A = nullptr;
  const double* dinv = nullptr;
  const mlamg_csr* P = nullptr;
  const mlamg_csr* R = nullptr;
  int64_t n = 0;
  double* x = nullptr;    // l > 0: iterate
  double* b = nullptr;    // l > 0: right-hand side
  double* r = nullptr;    // residual
  double* tmp = nullptr;  // ping-pong partner of x
  const mlamg_gs* gs = nullptr;  // Gauss-Seidel smoother (in place) instead of weighted Jacobi
  // factored prolongation (opt-in, mlamg_hier_set_factored_prolong): x += t - (w D^-1) A t with
  // t = Agg e, through fac_A (this level's A in the uniform row-pair format), instead of x += P e
  const mlamg_csr* fac_A = nullptr;
  const int32_t* fac_agg = nullptr;
  const double* fac_dinv = nullptr;
};

static int prolong_add(const Level& L, const double* e, double* x, const int32_t* done,
                       hipStream_t s) {
  if (L.fac_A) return mlamg::spmv_fadd(L.fac_A, L.fac_agg, e, x, L.fac_dinv, done, s);
  return mlamg::spmv_add(L.P, e, x, done, s);
}
}  // namespace

struct mlamg_hier {
  std::vector<Level> lv;
  const mlamg_csr* Ac = nullptr;
  const mlamg_dense* D = nullptr;
  mlamg_pcg* pcg = nullptr;  // coarse solve by inner-hierarchy PCG instead of a dense inverse
  // coarse solve by GMRES preconditioned by one V-cycle of an inner hierarchy of A_c (a coarse
  // operator that is not SPD and beyond the dense inverse's size: the reference's SuperLU
  // factors any nonsingular A_H, ns/lib/multigrid.py:165-170)
  mlamg_hier* gm_inner = nullptr;
  double gm_rtol = 1e-14, gm_fail_rtol = 1e-10;
  int gm_restart = 50, gm_maxiter = 20;
  int32_t gm_solves = 0, gm_last_iters = 0, gm_total_iters = 0, gm_not_converged = 0;
  double gm_worst_rel = 0.0;
  double* xc = nullptr;
  double* bc = nullptr;
  int nu_pre = 1, nu_post = 1;
  int norm_mode = 0;  // per-cycle history: 0 = ||b - A x||_2, 1 = ||x||_2 (amg_2_v error_tol)
  void* mem = nullptr;
  size_t mem_bytes = 0;
  double* partial = nullptr;
  int32_t* flags = nullptr;  // [0] counter, [1] done
  bool ready = false;
  // captured single cycle
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  const double* g_b = nullptr;
  double* g_x = nullptr;
  double* g_hist = nullptr;
  double g_tol = -1.0;
  hipStream_t cap_stream = nullptr;
  // captured coarse cycle (distributed executor: this hierarchy = replicated levels 1..L)
  hipGraph_t cgraph = nullptr;
  hipGraphExec_t cexec = nullptr;
  const double* cg_b = nullptr;
  uint64_t g_epoch = 0, cg_epoch = 0;
  double* cg_res = nullptr;
  int32_t* done_host = nullptr;  // pinned copy of flags[1], polled between batches of cycles
  // the stop flag the cycle's kernels test: flags + 1, or nullptr while a no-tolerance
  // mlamg_hier_vcycle runs (nothing can raise it, and every kernel would otherwise start with a
  // dependent load of it). done_check = 1 keeps it on every launch (A/B, mlamg_hier_set_done_check)
  int32_t* cur_done = nullptr;
  int done_check = 0;
  // a Krylov solver's workspace (gmres.hip), kept across calls and grown on demand: at C4 a
  // restart-100 GMRES needs 101 fine vectors (8 GB), too large for the allocation cache
  void* ws = nullptr;
  size_t ws_bytes = 0;
  // zero right-hand side for the paths that read b as a vector (Gauss-Seidel, coarse-only)
  double* zero_b = nullptr;
  bool zero_rhs = false;  // the last mlamg_hier_vcycle had b = NULL (cycle_bytes prices that)
};


using namespace mlamg;

static void hier_free_graph(mlamg_hier* H) {
  if (H->exec) (void)hipGraphExecDestroy(H->exec);
  if (H->graph) (void)hipGraphDestroy(H->graph);
  H->exec = nullptr;
  H->graph = nullptr;
  if (H->cexec) (void)hipGraphExecDestroy(H->cexec);
  if (H->cgraph) (void)hipGraphDestroy(H->cgraph);
  H->cexec = nullptr;
  H->cgraph = nullptr;
}

static int64_t coarse_rows(const mlamg_hier* H) {
  if (H->D) return H->D->n;
  if (H->gm_inner) return H->Ac->n_rows;
  return pcg_rows(H->pcg);
}

// a coarse solve that is driven from the host (PCG polls its flag, GMRES reads its status every
// step): the cycle runs eagerly, never from a captured graph
static bool host_driven_coarse(const mlamg_hier* H) { return H->pcg || H->gm_inner; }

// x = A_c^-1 b by GMRES from a zero guess to ||b - A_c x|| <= gm_rtol ||b||; every solve's
// outcome is counted (mlamg_hier_coarse_gmres_stats). Skipped once the outer tolerance flag is
// up (later kernels of the cycle then do nothing either)
static int gmres_coarse(mlamg_hier* H, const double* b, double* x, const int32_t* done,
                        hipStream_t s) {
  if (done) {
    int32_t d = 0;
    MLAMG_HIP(hipMemcpyAsync(&d, done, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    MLAMG_HIP(hipStreamSynchronize(s));
    if (d) return MLAMG_OK;
  }
  const int64_t n = H->Ac->n_rows;
  MLAMG_HIP(hipMemsetAsync(x, 0, sizeof(double) * n, s));
  int info = 0, it = 0;
  double rel = 0.0;
  MLAMG_TRY(gmres_impl(H->Ac, H->gm_inner, b, x, H->gm_rtol, H->gm_restart, H->gm_maxiter, true,
                       &info, &it, nullptr, 0, s, &rel));
  H->gm_solves += 1;
  H->gm_last_iters = it;
  H->gm_total_iters += it;
  if (info != 0) H->gm_not_converged += 1;
  H->gm_worst_rel = std::max(H->gm_worst_rel, rel);
  if (!(rel <= H->gm_fail_rtol)) {  // NaN included
    char msg[160];
    snprintf(msg, sizeof msg,
             "GMRES coarse solve did not converge (final relative residual %.3e > %.1e): the "
             "coarse operator may be singular", rel, H->gm_fail_rtol);
    set_error(msg);
    return MLAMG_EINVAL;
  }
  return MLAMG_OK;
}

// the coarsest solve: dense inverse GEMV, inner-hierarchy PCG (pcg.hip) or GMRES (gmres.hip)
static int coarse_solve(mlamg_hier* H, const double* b, double* x, const int32_t* done,
                        hipStream_t s) {
  if (H->D) return dense_solve_impl(H->D, b, x, done, s);
  if (H->gm_inner) return gmres_coarse(H, b, x, done, s);
  return pcg_solve_impl(H->pcg, b, x, done, s);
}

static int hier_prepare(mlamg_hier* H) {
  if (H->ready) return MLAMG_OK;
  MLAMG_REQUIRE(H->D != nullptr || H->pcg != nullptr || H->gm_inner != nullptr,
                "coarse solver not set (mlamg_hier_set_coarse / _pcg / _gmres)");
  size_t total = 0;
  auto add = [&](int64_t n) {
    size_t b = sizeof(double) * (size_t)std::max<int64_t>(n, 1);
    b = (b + 255) & ~size_t(255);
    total += b;
    return b;
  };
  for (size_t l = 0; l < H->lv.size(); ++l) {
    const int64_t n = H->lv[l].n;
    add(n);  // x: level 0 also needs it when this hierarchy serves as a coarse cycle
    add(n);
    add(n);
    add(n);
  }
  const int64_t nc = coarse_rows(H);
  add(nc);
  add(nc);
  int64_t maxblk = 1;
  for (auto& L : H->lv) maxblk = std::max<int64_t>(maxblk, part_capacity(L.A));
  add(maxblk);
  total += 256;
  MLAMG_HIP(hipMalloc(&H->mem, total));
  H->mem_bytes = total;
  char* p = static_cast<char*>(H->mem);
  auto take = [&](int64_t n) {
    double* q = reinterpret_cast<double*>(p);
    size_t b = sizeof(double) * (size_t)std::max<int64_t>(n, 1);
    p += (b + 255) & ~size_t(255);
    return q;
  };
  for (size_t l = 0; l < H->lv.size(); ++l) {
    Level& L = H->lv[l];
    L.x = take(L.n);
    L.b = take(L.n);
    L.r = take(L.n);
    L.tmp = take(L.n);
  }
  H->xc = take(nc);
  H->bc = take(nc);
  H->partial = take(maxblk);
  H->flags = reinterpret_cast<int32_t*>(p);
  H->cur_done = H->flags + 1;
  MLAMG_HIP(hipMemset(H->mem, 0, total));
  // hipMemset runs on the null stream and may return before it completes: a caller on a
  // non-blocking stream (one thread per rank, csrc/comm.hip's loopback) must not race it
  MLAMG_HIP(hipDeviceSynchronize());
  H->ready = true;
  return MLAMG_OK;
}

// smoothing sweeps starting from `cur` (x or tmp); returns buffer holding the result
static int smooth(const Level& L, const double* b, double*& cur, double* other, int nu,
                  const int32_t* done, hipStream_t s) {
  if (L.gs) return gs_sweep_impl(L.gs, cur, b, nu, done, s);  // in place, cur unchanged
  for (int i = 0; i < nu; ++i) {
    MLAMG_TRY(jacobi_sweep(L.A, L.dinv, b, cur, other, false, done, s));
    std::swap(cur, other);
  }
  return MLAMG_OK;
}

// one V-cycle below the finest level; result pointer returned through `res`. presmoothed: the
// caller's restriction kernel already wrote the first zero-guess sweep x = Dinv_w b into L.x.
static int cycle_coarse(mlamg_hier* H, size_t l, const double* b, double** res, hipStream_t s,
                        bool presmoothed = false) {
  const int32_t* done = H->cur_done;
  if (l == H->lv.size()) {
    MLAMG_TRY(coarse_solve(H, b, H->xc, done, s));
    *res = H->xc;
    return MLAMG_OK;
  }
  Level& L = H->lv[l];
  double* cur = L.x;
  double* other = L.tmp;
  if (H->nu_pre > 0 && L.gs) {
    MLAMG_HIP(hipMemsetAsync(cur, 0, sizeof(double) * L.n, s));
    MLAMG_TRY(smooth(L, b, cur, other, H->nu_pre, done, s));
    MLAMG_TRY(residual_impl(L.A, b, cur, L.r, nullptr, nullptr, nullptr, const_cast<int32_t*>(done),
                            kNoTol, nullptr, nullptr, nullptr, s));
  } else if (H->nu_pre > 0) {
    if (!presmoothed) MLAMG_TRY(jacobi_from_zero(cur, L.dinv, b, L.n, done, s));
    MLAMG_TRY(smooth(L, b, cur, other, H->nu_pre - 1, done, s));
    MLAMG_TRY(residual_impl(L.A, b, cur, L.r, nullptr, nullptr, nullptr, const_cast<int32_t*>(done),
                            kNoTol, nullptr, nullptr, nullptr, s));
  } else {
    MLAMG_HIP(hipMemsetAsync(cur, 0, sizeof(double) * L.n, s));
    MLAMG_HIP(hipMemcpyAsync(L.r, b, sizeof(double) * L.n, hipMemcpyDeviceToDevice, s));
  }
  const bool fuse_next = l + 1 < H->lv.size() && H->nu_pre > 0 && !H->lv[l + 1].gs;
  double* bn = (l + 1 < H->lv.size()) ? H->lv[l + 1].b : H->bc;
  if (fuse_next) {
    MLAMG_TRY(spmv_set(L.R, L.r, bn, done, s, H->lv[l + 1].x, H->lv[l + 1].dinv));
  } else {
    MLAMG_TRY(spmv_set(L.R, L.r, bn, done, s));
  }
  double* xn = nullptr;
  MLAMG_TRY(cycle_coarse(H, l + 1, bn, &xn, s, fuse_next));
  MLAMG_TRY(prolong_add(L, xn, cur, done, s));
  other = (cur == L.x) ? L.tmp : L.x;
  MLAMG_TRY(smooth(L, b, cur, other, H->nu_post, done, s));
  *res = cur;
  return MLAMG_OK;
}

// Fused mode (nu_pre >= 1 and an odd number of ping-pong sweeps after the first one, i.e.
// (nu_pre - 1 + nu_post) odd, so the cycle's result t lands in L0.tmp — V(1,1), V(2,2), V(1,3)
// but not V(2,1) or V(1,2), whose result ends in x itself): the
// end-of-cycle residual kernel r = b - A t also writes x = t + Dinv_w r, i.e. the NEXT cycle's
// first pre-smoothing sweep (same roundings), and the cycle starts from that. The caller applies
// the very first sweep before the first cycle and copies t back into x after the last one (t is
// still in tmp even when the tolerance flag stopped later cycles). Saves one pass over x, d, r.
static bool fused_presmooth(const mlamg_hier* H) {
  return !H->lv.empty() && H->nu_pre >= 1 && ((H->nu_pre - 1 + H->nu_post) & 1) &&
         !H->lv[0].gs && H->norm_mode == 0;
}

// one finest-level cycle; requires L0.r == b - A x on entry, leaves it so on exit (fused mode:
// x on entry is already pre-smoothed once, and on exit t is in L0.tmp, x = t + Dinv_w r)
static int cycle_top(mlamg_hier* H, const double* b, double* x, double* hist, double tol,
                     hipStream_t s) {
  int32_t* counter = H->flags;
  int32_t* done = H->cur_done;
  if (H->lv.empty()) {  // coarse-only hierarchy: x = A^-1 b
    MLAMG_TRY(coarse_solve(H, b, x, done, s));
    return MLAMG_OK;
  }
  Level& L = H->lv[0];
  const bool fused = fused_presmooth(H);
  double* cur = x;
  double* other = L.tmp;
  if (H->nu_pre > 0 && L.gs) {
    MLAMG_TRY(smooth(L, b, cur, other, H->nu_pre, done, s));
    MLAMG_TRY(residual_impl(L.A, b, cur, L.r, nullptr, nullptr, nullptr, done, kNoTol, nullptr,
                            nullptr, nullptr, s));
  } else if (H->nu_pre > 0) {
    if (!fused) MLAMG_TRY(jacobi_from_residual(cur, L.dinv, L.r, L.n, done, s));
    MLAMG_TRY(smooth(L, b, cur, other, H->nu_pre - 1, done, s));
    MLAMG_TRY(residual_impl(L.A, b, cur, L.r, nullptr, nullptr, nullptr, done, kNoTol, nullptr,
                            nullptr, nullptr, s));
  }
  const bool fuse_next = H->lv.size() > 1 && H->nu_pre > 0 && !H->lv[1].gs;
  double* bn = H->lv.size() > 1 ? H->lv[1].b : H->bc;
  if (fuse_next) {
    MLAMG_TRY(spmv_set(L.R, L.r, bn, done, s, H->lv[1].x, H->lv[1].dinv));
  } else {
    MLAMG_TRY(spmv_set(L.R, L.r, bn, done, s));
  }
  double* xn = nullptr;
  MLAMG_TRY(cycle_coarse(H, 1, bn, &xn, s, fuse_next));
  MLAMG_TRY(prolong_add(L, xn, cur, done, s));
  other = (cur == x) ? L.tmp : x;
  MLAMG_TRY(smooth(L, b, cur, other, H->nu_post, done, s));
  // end-of-cycle residual + norm (+ copy the iterate back into x when it sits in tmp)
  if (H->norm_mode == 1) {  // history of ||x||_2 (amg_2_v error_tol): residual kept for reuse
    MLAMG_TRY(residual_impl(L.A, b, cur, L.r, nullptr, nullptr, nullptr, done, 0.0,
                            cur != x ? x : nullptr, cur != x ? cur : nullptr, nullptr, s));
    MLAMG_TRY(norm_hist_impl(x, L.n, H->partial, hist, counter, done, tol, s));
    return MLAMG_OK;
  }
  // fused: nothing reads this r (the next cycle starts with its own residual), so it is not
  // stored — the kernel still forms it for the norm and the fused sweep x = t + Dinv_w r
  MLAMG_TRY(residual_impl(L.A, b, cur, fused ? nullptr : L.r, nullptr, hist, counter, done, tol,
                          cur != x ? x : nullptr, cur != x ? cur : nullptr, H->partial, s,
                          fused ? L.dinv : nullptr));
  return MLAMG_OK;
}

namespace mlamg {
// allocate the work buffers now (not capture-safe), so a later capture only records launches
int hier_prepare_ext(mlamg_hier* H) { return hier_prepare(H); }
// the device flag every kernel of a cycle checks (a PCG using H as preconditioner shares it)
int32_t* hier_done_flag(mlamg_hier* H) { return H->flags + 1; }
int hier_workspace(mlamg_hier* H, size_t bytes, void** out) {
  if (H->ws_bytes < bytes) {
    if (H->ws) (void)hipFree(H->ws);  // ordered after every earlier use (cache semantics)
    H->ws = nullptr;
    H->ws_bytes = 0;
    MLAMG_HIP(hipMalloc(&H->ws, bytes));
    H->ws_bytes = bytes;
  }
  *out = H->ws;
  return MLAMG_OK;
}
int64_t hier_fine_rows(const mlamg_hier* H) {
  return H->lv.empty() ? coarse_rows(H) : H->lv[0].n;
}

// One cycle from a zero guess on (b -> *x_out) treating level 0 of H as a coarse level
// (used by the distributed executor, whose H holds the replicated levels 1..L).
int hier_coarse_cycle(mlamg_hier* H, const double* b, double** x_out, int use_graph,
                      hipStream_t s) {
  MLAMG_TRY(hier_prepare(H));
  if (!use_graph || host_driven_coarse(H)) return cycle_coarse(H, 0, b, x_out, s);
  if (!(H->cexec && H->cg_b == b && H->cg_epoch == format_epoch())) {
    if (H->cexec) (void)hipGraphExecDestroy(H->cexec);
    if (H->cgraph) (void)hipGraphDestroy(H->cgraph);
    H->cexec = nullptr;
    H->cgraph = nullptr;
    if (!H->cap_stream) MLAMG_HIP(hipStreamCreateWithFlags(&H->cap_stream, hipStreamNonBlocking));
    MLAMG_HIP(hipStreamBeginCapture(H->cap_stream, hipStreamCaptureModeThreadLocal));
    double* res = nullptr;
    int rc = cycle_coarse(H, 0, b, &res, H->cap_stream);
    hipGraph_t g = nullptr;
    hipError_t e = hipStreamEndCapture(H->cap_stream, &g);
    if (rc != MLAMG_OK) {
      if (g) (void)hipGraphDestroy(g);
      return rc;
    }
    MLAMG_HIP(e);
    H->cgraph = g;
    MLAMG_HIP(hipGraphInstantiate(&H->cexec, g, nullptr, nullptr, 0));
    H->cg_b = b;
    H->cg_epoch = format_epoch();
    H->cg_res = res;
  }
  MLAMG_HIP(hipGraphLaunch(H->cexec, s));
  *x_out = H->cg_res;
  return MLAMG_OK;
}
}  // namespace mlamg

extern "C" {

int mlamg_hier_create(mlamg_hier** out) {
  MLAMG_REQUIRE(out, "out is NULL");
  *out = new mlamg_hier();
  return MLAMG_OK;
}

int mlamg_hier_destroy(mlamg_hier* H) {
  if (!H) return MLAMG_OK;
  hier_free_graph(H);
  if (H->cap_stream) (void)hipStreamDestroy(H->cap_stream);
  if (H->mem) (void)hipFree(H->mem);
  if (H->done_host) (void)hipHostFree(H->done_host);
  if (H->ws) (void)hipFree(H->ws);
  if (H->zero_b) (void)hipFree(H->zero_b);
  delete H;
  return MLAMG_OK;
}

int mlamg_hier_add_level(mlamg_hier* H, const mlamg_csr* A, const double* dinv_w,
                         const mlamg_csr* P, const mlamg_csr* R) {
  MLAMG_REQUIRE(H && A && dinv_w && P && R, "NULL argument");
  MLAMG_REQUIRE(!H->ready, "hierarchy already finalised");
  MLAMG_REQUIRE(A->n_rows == A->n_cols, "A must be square");
  MLAMG_REQUIRE(P->n_rows == A->n_rows, "P rows != A rows");
  MLAMG_REQUIRE(R->n_cols == A->n_rows && R->n_rows == P->n_cols, "R must be P^T");
  if (!H->lv.empty()) {
    MLAMG_REQUIRE(H->lv.back().P->n_cols == A->n_rows, "level sizes do not chain");
  }
  Level L;
  L.A = A;
  L.dinv = dinv_w;
  L.P = P;
  L.R = R;
  L.n = A->n_rows;
  H->lv.push_back(L);
  return MLAMG_OK;
}

int mlamg_hier_set_coarse(mlamg_hier* H, const mlamg_csr* A_coarse, const mlamg_dense* D) {
  MLAMG_REQUIRE(H && D, "NULL argument");
  MLAMG_REQUIRE(!H->ready, "hierarchy already finalised");
  if (!H->lv.empty())
    MLAMG_REQUIRE(H->lv.back().P->n_cols == D->n, "coarse size does not match last P");
  H->Ac = A_coarse;
  H->D = D;
  H->pcg = nullptr;
  H->gm_inner = nullptr;
  return MLAMG_OK;
}

int mlamg_hier_set_coarse_pcg(mlamg_hier* H, const mlamg_csr* A_coarse, mlamg_pcg* C) {
  MLAMG_REQUIRE(H && A_coarse && C, "NULL argument");
  MLAMG_REQUIRE(!H->ready, "hierarchy already finalised");
  MLAMG_REQUIRE(pcg_rows(C) == A_coarse->n_rows, "PCG solver of another size");
  if (!H->lv.empty())
    MLAMG_REQUIRE(H->lv.back().P->n_cols == A_coarse->n_rows, "coarse size does not match last P");
  H->Ac = A_coarse;
  H->D = nullptr;
  H->pcg = C;
  H->gm_inner = nullptr;
  return MLAMG_OK;
}

int mlamg_hier_set_coarse_gmres(mlamg_hier* H, const mlamg_csr* A_coarse, mlamg_hier* inner,
                                double rtol, double fail_rtol, int restart, int maxiter) {
  MLAMG_REQUIRE(H && A_coarse && inner, "NULL argument");
  MLAMG_REQUIRE(inner != H, "the preconditioner hierarchy must be another hierarchy");
  MLAMG_REQUIRE(!H->ready, "hierarchy already finalised");
  MLAMG_REQUIRE(A_coarse->n_rows == A_coarse->n_cols, "A_coarse must be square");
  MLAMG_REQUIRE(hier_fine_rows(inner) == A_coarse->n_rows,
                "preconditioner hierarchy does not match A_coarse");
  MLAMG_REQUIRE(rtol >= 0.0 && fail_rtol >= rtol && restart > 0 && maxiter > 0,
                "invalid GMRES parameters");
  if (!H->lv.empty())
    MLAMG_REQUIRE(H->lv.back().P->n_cols == A_coarse->n_rows, "coarse size does not match last P");
  H->Ac = A_coarse;
  H->D = nullptr;
  H->pcg = nullptr;
  H->gm_inner = inner;
  H->gm_rtol = rtol;
  H->gm_fail_rtol = fail_rtol;
  H->gm_restart = restart;
  H->gm_maxiter = maxiter;
  return MLAMG_OK;
}

int mlamg_hier_coarse_gmres_stats(const mlamg_hier* H, int32_t* solves, int32_t* last_iters,
                                  int32_t* total_iters, int32_t* not_converged,
                                  double* worst_rel) {
  MLAMG_REQUIRE(H, "NULL argument");
  MLAMG_REQUIRE(H->gm_inner, "the coarse solve is not GMRES");
  if (solves) *solves = H->gm_solves;
  if (last_iters) *last_iters = H->gm_last_iters;
  if (total_iters) *total_iters = H->gm_total_iters;
  if (not_converged) *not_converged = H->gm_not_converged;
  if (worst_rel) *worst_rel = H->gm_worst_rel;
  return MLAMG_OK;
}

int mlamg_hier_set_level_smoother(mlamg_hier* H, int level, const mlamg_gs* gs) {
  MLAMG_REQUIRE(H && level >= 0 && (size_t)level < H->lv.size(), "invalid level");
  MLAMG_REQUIRE(!gs || gs_rows(gs) == H->lv[level].n, "Gauss-Seidel handle of another size");
  H->lv[level].gs = gs;
  hier_free_graph(H);
  return MLAMG_OK;
}

int mlamg_hier_set_norm(mlamg_hier* H, int mode) {
  MLAMG_REQUIRE(H && (mode == 0 || mode == 1), "mode must be 0 (residual) or 1 (x)");
  H->norm_mode = mode;
  hier_free_graph(H);
  return MLAMG_OK;
}

int mlamg_hier_set_factored_prolong(mlamg_hier* H, int level, const mlamg_csr* A_uni,
                                    const int32_t* agg, const double* dinv_w) {
  MLAMG_REQUIRE(H && level >= 0 && (size_t)level < H->lv.size(), "invalid level");
  Level& L = H->lv[level];
  if (!A_uni) {
    L.fac_A = nullptr;
    L.fac_agg = nullptr;
    L.fac_dinv = nullptr;
    hier_free_graph(H);
    return MLAMG_OK;
  }
  MLAMG_REQUIRE(agg && dinv_w, "agg and dinv_w are required");
  MLAMG_REQUIRE(A_uni->n_rows == L.n && A_uni->n_cols == L.n, "A_uni is not this level's size");
  if (!(A_uni->rp_pid && A_uni->rp_uni.k > 0 && A_uni->rp_msk)) {
    set_error("factored prolongation: A_uni is not in the uniform row-pair format");
    return MLAMG_EUNSUPPORTED;
  }
  L.fac_A = A_uni;
  L.fac_agg = agg;
  L.fac_dinv = dinv_w;
  hier_free_graph(H);
  return MLAMG_OK;
}

int mlamg_hier_set_done_check(mlamg_hier* H, int always) {
  MLAMG_REQUIRE(H && (always == 0 || always == 1), "always must be 0 or 1");
  H->done_check = always;
  hier_free_graph(H);
  return MLAMG_OK;
}

int mlamg_hier_set_smoothing(mlamg_hier* H, int nu_pre, int nu_post) {
  MLAMG_REQUIRE(H && nu_pre >= 0 && nu_post >= 0, "invalid argument");
  H->nu_pre = nu_pre;
  H->nu_post = nu_post;
  hier_free_graph(H);
  return MLAMG_OK;
}

int mlamg_hier_vcycle(mlamg_hier* H, const double* b, double* x, int n_cycles, double tol,
                      double* res_hist, int32_t* cycles_done_host, int use_graph, void* stream) {
  MLAMG_REQUIRE(H && x, "NULL argument");
  MLAMG_REQUIRE(b != x, "b and x must differ");
  MLAMG_REQUIRE(n_cycles >= 0, "n_cycles < 0");
  MLAMG_TRY(hier_prepare(H));
  hipStream_t s = S(stream);
  // b NULL: a zero right-hand side (the reference's convergence-factor problems, b = 0). The
  // fine-level kernels then take b = +0.0 without reading a vector of zeros (the same bits:
  // 0.0 - A x); the paths that read b as a vector get a zero buffer
  H->zero_rhs = !b;
  if (!b && (H->lv.empty() || H->lv[0].gs)) {
    const int64_t n0 = hier_fine_rows(H);
    if (!H->zero_b) {
      MLAMG_HIP(hipMalloc(&H->zero_b, sizeof(double) * std::max<int64_t>(n0, 1)));
      MLAMG_HIP(hipMemsetAsync(H->zero_b, 0, sizeof(double) * std::max<int64_t>(n0, 1), s));
    }
    b = H->zero_b;
  }
  // a PCG coarse solve polls its convergence flag between iterations, GMRES reads its status
  // every step: cycles run eagerly
  if (host_driven_coarse(H)) use_graph = 0;
  MLAMG_HIP(hipMemsetAsync(H->flags, 0, 2 * sizeof(int32_t), s));
  // no tolerance: no kernel can raise the stop flag, so none tests it (restored on return: a
  // PCG that uses H as its preconditioner shares the flag, hier_done_flag)
  struct DoneScope {
    mlamg_hier* H;
    ~DoneScope() { H->cur_done = H->flags + 1; }
  } done_scope{H};
  H->cur_done = (tol >= 0.0 || H->done_check || H->pcg) ? H->flags + 1 : nullptr;
  const bool fused = fused_presmooth(H) && n_cycles > 0;
  if (!H->lv.empty()) {
    Level& L = H->lv[0];
    // r = b - A x for the first cycle's pre-smoothing sweep
    MLAMG_TRY(residual_impl(L.A, b, x, L.r, nullptr, nullptr, nullptr, nullptr, kNoTol, nullptr,
                            nullptr, nullptr, s));
    if (fused) MLAMG_TRY(jacobi_from_residual(x, L.dinv, L.r, L.n, nullptr, s));
  }
  if (use_graph && n_cycles > 0 && !H->lv.empty()) {
    if (!(H->exec && H->g_b == b && H->g_x == x && H->g_hist == res_hist && H->g_tol == tol &&
          H->g_epoch == format_epoch())) {
      hier_free_graph(H);
      if (!H->cap_stream) MLAMG_HIP(hipStreamCreateWithFlags(&H->cap_stream, hipStreamNonBlocking));
      MLAMG_HIP(hipStreamBeginCapture(H->cap_stream, hipStreamCaptureModeThreadLocal));
      int rc = cycle_top(H, b, x, res_hist, tol, H->cap_stream);
      hipGraph_t g = nullptr;
      hipError_t e = hipStreamEndCapture(H->cap_stream, &g);
      if (rc != MLAMG_OK) {
        if (g) (void)hipGraphDestroy(g);
        return rc;
      }
      MLAMG_HIP(e);
      H->graph = g;
      MLAMG_HIP(hipGraphInstantiate(&H->exec, g, nullptr, nullptr, 0));
      H->g_b = b;
      H->g_x = x;
      H->g_hist = res_hist;
      H->g_tol = tol;
      H->g_epoch = format_epoch();
    }
    if (!H->done_host) (void)hipHostMalloc(&H->done_host, sizeof(int32_t), hipHostMallocDefault);
    MLAMG_TRY(run_cycles(n_cycles, tol, H->flags + 1, H->done_host, s, [&]() -> int {
      MLAMG_HIP(hipGraphLaunch(H->exec, s));
      return MLAMG_OK;
    }));
  } else {
    if (!H->done_host) (void)hipHostMalloc(&H->done_host, sizeof(int32_t), hipHostMallocDefault);
    MLAMG_TRY(run_cycles(n_cycles, tol, H->flags + 1, H->done_host, s,
                         [&]() { return cycle_top(H, b, x, res_hist, tol, s); }));
  }
  if (fused)  // the iterate is t (in tmp); x holds t + Dinv_w r for a cycle that never ran
    MLAMG_HIP(hipMemcpyAsync(x, H->lv[0].tmp, sizeof(double) * H->lv[0].n,
                             hipMemcpyDeviceToDevice, s));
  MLAMG_HIP(hipGetLastError());
  if (cycles_done_host) {
    int32_t cnt = 0;
    MLAMG_HIP(hipMemcpyAsync(&cnt, H->flags, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    MLAMG_HIP(hipStreamSynchronize(s));
    *cycles_done_host = H->lv.empty() ? n_cycles : cnt;
  }
  return MLAMG_OK;
}

static double spmv_bytes(const mlamg_csr* A) {
  return 12.0 * A->nnz + 4.0 * (A->n_rows + 1) + 8.0 * A->n_cols + 8.0 * A->n_rows;
}

// Bytes of one V-cycle, summed over its launches. stored = false: every operator priced as
// CSR (SURVEY.md §8(d) model — a CSR-EQUIVALENT figure, which re-encoded operators beat);
// stored = true: every operator priced as the format it is stored in (mlamg_csr_format_bytes:
// matrix stream + x once + y once), Jacobi weights not read when attached to a rowpat operator,
// end-of-cycle r not written in fused mode — the bytes the cycle must move through HBM.
static int cycle_bytes(const mlamg_hier* H, bool stored, double* bytes) {
  double t = 0.0;
  auto op = [&](const mlamg_csr* M, double* b) -> int {
    if (!stored) {
      *b = spmv_bytes(M);
      return MLAMG_OK;
    }
    return mlamg_csr_format_bytes(M, b);
  };
  for (size_t l = 0; l < H->lv.size(); ++l) {
    const Level& L = H->lv[l];
    const double n = (double)L.n;
    double a = 0.0, r = 0.0, p = 0.0;
    MLAMG_TRY(op(L.A, &a));
    MLAMG_TRY(op(L.R, &r));
    MLAMG_TRY(op(L.P, &p));
    if (L.fac_A) {  // the factored form streams agg (4 B/row) and gathers e instead of P
      double fa = 0.0;
      MLAMG_TRY(op(L.fac_A, &fa));
      p = fa - 8.0 * n + 4.0 * n + 8.0 * (double)L.P->n_cols;
    }
    const double dv = (stored && L.A->rp_dinv_att) ? 0.0 : 8.0 * n;
    // + b (not read at the finest level when the right-hand side is zero), dinv
    const double bb = (l == 0 && H->zero_rhs && !L.gs) ? 0.0 : 8.0 * n;
    const double jac = a + bb + dv;
    const double res = a + bb;
    const bool fused = l == 0 && fused_presmooth(H);
    if (H->nu_pre > 0) {
      // first sweep: elementwise at the top (unless fused into the cycle end); below, fused
      // into the restriction kernel above (+ read dinv, write x)
      if (!fused) t += (l == 0) ? 32.0 * n : 16.0 * n;
      t += (H->nu_pre - 1) * jac + res;
    }
    t += r;
    t += p + 8.0 * n;  // + read x before the add
    t += H->nu_post * jac;
    // end-of-cycle residual norm, + x = t (read t, write x) or, fused, x = t + Dinv_w r
    // (fused: + read dinv, write x; r itself is not stored)
    const int swaps = L.gs ? 0 : std::max(H->nu_pre - 1, 0) + H->nu_post;
    if (l == 0) {
      if (stored && fused)
        t += res + dv;  // r's store replaced by x's
      else
        t += res + ((fused || (swaps & 1)) ? 16.0 * n : 0.0);
    }
  }
  if (H->D) t += 8.0 * H->D->n * H->D->n + 16.0 * H->D->n;
  if (H->pcg) {  // priced per PCG iteration of the last solve: A_c x + ~10 vector passes +
                 // one inner V-cycle
    int32_t it = 0;
    MLAMG_TRY(mlamg_pcg_stats(H->pcg, &it, nullptr, nullptr, nullptr, nullptr));
    double a = 0.0, inner = 0.0;
    MLAMG_TRY(stored ? mlamg_csr_format_bytes(H->Ac, &a) : (a = spmv_bytes(H->Ac), MLAMG_OK));
    MLAMG_TRY(cycle_bytes(pcg_inner(H->pcg), stored, &inner));
    t += (double)std::max(it, 1) * (a + 80.0 * (double)H->Ac->n_rows + inner);
  }
  if (H->gm_inner) {  // priced per GMRES step of the last solve: A_c x + one inner V-cycle +
                      // ~2 (k + 1) Gram-Schmidt vector passes, k ~ restart / 2 on average
    double a = 0.0, inner = 0.0;
    MLAMG_TRY(stored ? mlamg_csr_format_bytes(H->Ac, &a) : (a = spmv_bytes(H->Ac), MLAMG_OK));
    MLAMG_TRY(cycle_bytes(H->gm_inner, stored, &inner));
    t += (double)std::max(H->gm_last_iters, 1) *
         (a + inner + 8.0 * (double)(H->gm_restart + 2) * (double)H->Ac->n_rows);
  }
  *bytes = t;
  return MLAMG_OK;
}

int mlamg_hier_cycle_bytes(const mlamg_hier* H, double* bytes) {
  MLAMG_REQUIRE(H && bytes, "NULL argument");
  return cycle_bytes(H, false, bytes);
}

int mlamg_hier_cycle_format_bytes(const mlamg_hier* H, double* bytes) {
  MLAMG_REQUIRE(H && bytes, "NULL argument");
  return cycle_bytes(H, true, bytes);
}

}  // extern "C"
