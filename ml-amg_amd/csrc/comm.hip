// Multi-GPU V-cycle: RCCL communicator, halo exchange and the partitioned executor.
//
// One process per GPU. The first K levels are row-partitioned (mlamg/partition.py builds the
// maps: level 0 in near-equal blocks, level l+1 owned by the rank owning each aggregate's
// seed); the levels below are replicated on every rank (their setup is deterministic). Per
// partitioned level l of a cycle:
//   x  = Dinv b  (l > 0, zero guess)  |  x += Dinv r  (l = 0, reusing the end-of-cycle r)
//   halo_x(x); r = b - A_loc x_ext                    RCCL send/recv with the neighbours
//   halo_r(r); b_{l+1}[own] = R_own r_ext             coarse rows summed by their owner
//   l+1 partitioned: recurse; halo_p(x_{l+1}) ;  else: allgatherv(b_{l+1}), replicated cycle
//   x += P_loc x_{l+1,ext}
//   halo_x(x); t = x + Dinv(b - A x)                  post-smoothing
//   l = 0: halo_x(t); r = b - A t, ||r||^2 -> allreduce (MLAMG.py:194); x <- t
// Local rows keep their stored order and every coarse row is summed by one owner, so the
// iterate is bitwise the single-GPU iterate; only the norm's summation order differs.
#include "common.hpp"

#include <rccl/rccl.h>

#include <chrono>
#include <functional>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <tuple>

// In-process transport for testing the executor with several ranks on ONE device (RCCL refuses
// two ranks on one GPU): every rank is a host thread with its own stream; a send posts (buffer,
// ready event) into a shared mailbox, the receiver orders its stream after the ready event and
// copies device-to-device, and the sender's stream is then ordered after that copy (so it cannot
// overwrite its send buffer early). Same message order and grouping semantics as the RCCL calls
// it stands in for; never used by a communicator made with mlamg_comm_create.
struct LoopPost {
  const double* p = nullptr;
  size_t n = 0;
  hipEvent_t ready = nullptr;
  hipEvent_t done = nullptr;
  bool consumed = false;
  ~LoopPost() {
    if (ready) (void)hipEventDestroy(ready);
    if (done) (void)hipEventDestroy(done);
  }
};

struct LoopRound {  // one all-reduce: every rank's (buffer, ready), then (copied) events
  std::vector<const double*> buf;
  std::vector<hipEvent_t> ready, copied;
  int posted = 0, finished = 0, left = 0;
};

struct mlamg_loop_group {
  int W = 1;
  std::mutex mu;
  std::condition_variable cv;
  std::map<std::tuple<int, int, uint64_t>, std::shared_ptr<LoopPost>> box;
  std::vector<uint64_t> send_seq, recv_seq;  // [src * W + dst]
  std::map<uint64_t, LoopRound> rounds;
  int members = 0;
};

struct mlamg_comm {
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0;
  mlamg_loop_group* loop = nullptr;  // in-process test transport instead of RCCL
  bool null_transport = false;       // timing only: exchanges skipped (results are NOT valid)
  struct Recv {
    double* buf;
    size_t n;
    int peer;
  };
  std::vector<std::shared_ptr<LoopPost>> sends;  // posted in the open group
  std::vector<Recv> recvs;                       // completed at group end
  uint64_t ar_seq = 0;
  double* ar_stage = nullptr;
  size_t ar_cap = 0;
};

struct mlamg_halo {
  mlamg_comm* c = nullptr;
  int64_t n_own = 0, n_ghost = 0;
  std::vector<int> nbr;
  std::vector<int64_t> send_off, send_cnt, recv_off, recv_cnt;
  int32_t* send_idx = nullptr;  // device, concatenated per neighbour
  double* send_buf = nullptr;   // device
  int64_t n_send = 0;
};

#define MLAMG_NCCL(call)                                                            \
  do {                                                                              \
    ncclResult_t _r = (call);                                                       \
    if (_r != ncclSuccess) {                                                        \
      ::mlamg::set_error(std::string(#call) + " failed: " + ncclGetErrorString(_r)); \
      return MLAMG_ENCCL;                                                           \
    }                                                                               \
  } while (0)

namespace mlamg {

constexpr auto kLoopTimeout = std::chrono::seconds(120);

static int loop_wait(mlamg_loop_group* g, std::unique_lock<std::mutex>& lk,
                     const std::function<bool()>& ready, const char* what) {
  if (!g->cv.wait_for(lk, kLoopTimeout, ready)) {
    set_error(std::string("loopback transport: timed out waiting for ") + what);
    return MLAMG_ENCCL;
  }
  return MLAMG_OK;
}

static int xgroup_begin(mlamg_comm* c) {
  if (c->null_transport) return MLAMG_OK;
  if (!c->loop) MLAMG_NCCL(ncclGroupStart());
  return MLAMG_OK;
}

static int xsend(mlamg_comm* c, const double* buf, size_t n, int peer, hipStream_t s) {
  if (c->null_transport) return MLAMG_OK;
  if (!c->loop) {
    MLAMG_NCCL(ncclSend(buf, n, ncclFloat64, peer, c->comm, s));
    return MLAMG_OK;
  }
  auto post = std::make_shared<LoopPost>();
  post->p = buf;
  post->n = n;
  MLAMG_HIP(hipEventCreateWithFlags(&post->ready, hipEventDisableTiming));
  MLAMG_HIP(hipEventRecord(post->ready, s));
  mlamg_loop_group* g = c->loop;
  {
    std::lock_guard<std::mutex> lk(g->mu);
    const uint64_t seq = g->send_seq[c->rank * g->W + peer]++;
    g->box[std::make_tuple(c->rank, peer, seq)] = post;
  }
  g->cv.notify_all();
  c->sends.push_back(post);
  return MLAMG_OK;
}

static int xrecv(mlamg_comm* c, double* buf, size_t n, int peer, hipStream_t s) {
  if (c->null_transport) return MLAMG_OK;
  if (!c->loop) {
    MLAMG_NCCL(ncclRecv(buf, n, ncclFloat64, peer, c->comm, s));
    return MLAMG_OK;
  }
  c->recvs.push_back({buf, n, peer});
  return MLAMG_OK;
}

static int xgroup_end(mlamg_comm* c, hipStream_t s) {
  if (c->null_transport) return MLAMG_OK;
  if (!c->loop) {
    MLAMG_NCCL(ncclGroupEnd());
    return MLAMG_OK;
  }
  mlamg_loop_group* g = c->loop;
  std::vector<mlamg_comm::Recv> recvs;
  recvs.swap(c->recvs);
  std::vector<std::shared_ptr<LoopPost>> sends;
  sends.swap(c->sends);
  for (const auto& r : recvs) {
    std::shared_ptr<LoopPost> post;
    {
      std::unique_lock<std::mutex> lk(g->mu);
      const auto key = std::make_tuple(r.peer, c->rank, g->recv_seq[r.peer * g->W + c->rank]);
      MLAMG_TRY(loop_wait(g, lk, [&] { return g->box.count(key) != 0; }, "a matching send"));
      post = g->box[key];
      g->box.erase(key);
      ++g->recv_seq[r.peer * g->W + c->rank];
    }
    MLAMG_REQUIRE(post->n == r.n, "loopback transport: send/recv sizes differ");
    MLAMG_HIP(hipStreamWaitEvent(s, post->ready, 0));
    if (r.n) MLAMG_HIP(hipMemcpyAsync(r.buf, post->p, sizeof(double) * r.n, hipMemcpyDeviceToDevice, s));
    MLAMG_HIP(hipEventCreateWithFlags(&post->done, hipEventDisableTiming));
    MLAMG_HIP(hipEventRecord(post->done, s));
    {
      std::lock_guard<std::mutex> lk(g->mu);
      post->consumed = true;
    }
    g->cv.notify_all();
  }
  for (const auto& p : sends) {
    {
      std::unique_lock<std::mutex> lk(g->mu);
      MLAMG_TRY(loop_wait(g, lk, [&] { return p->consumed; }, "the receiver of a send"));
    }
    MLAMG_HIP(hipStreamWaitEvent(s, p->done, 0));
  }
  return MLAMG_OK;
}

__global__ void k_loop_sum(const double* __restrict__ stage, int W, int64_t n,
                           double* __restrict__ out) {
  const int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  double t = stage[i];
  for (int r = 1; r < W; ++r) t += stage[(int64_t)r * n + i];
  out[i] = t;
}

static int xallreduce_sum(mlamg_comm* c, double* buf, size_t n, hipStream_t s) {
  if (c->null_transport) return MLAMG_OK;
  if (!c->loop) {
    MLAMG_NCCL(ncclAllReduce(buf, buf, n, ncclFloat64, ncclSum, c->comm, s));
    return MLAMG_OK;
  }
  mlamg_loop_group* g = c->loop;
  const int W = g->W;
  if (c->ar_cap < (size_t)W * n) {
    MLAMG_HIP(hipStreamSynchronize(s));
    if (c->ar_stage) (void)hipFree(c->ar_stage);
    c->ar_stage = nullptr;
    MLAMG_HIP(hipMalloc(&c->ar_stage, sizeof(double) * std::max<size_t>((size_t)W * n, 1)));
    c->ar_cap = (size_t)W * n;
  }
  const uint64_t round = c->ar_seq++;
  hipEvent_t ready = nullptr, copied = nullptr;
  MLAMG_HIP(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
  MLAMG_HIP(hipEventRecord(ready, s));
  std::vector<const double*> bufs;
  std::vector<hipEvent_t> readies;
  {
    std::unique_lock<std::mutex> lk(g->mu);
    LoopRound& R = g->rounds[round];
    if (R.buf.empty()) {
      R.buf.assign(W, nullptr);
      R.ready.assign(W, nullptr);
      R.copied.assign(W, nullptr);
    }
    R.buf[c->rank] = buf;
    R.ready[c->rank] = ready;
    ++R.posted;
    g->cv.notify_all();
    MLAMG_TRY(loop_wait(g, lk, [&] { return g->rounds[round].posted == W; }, "all-reduce peers"));
    bufs = g->rounds[round].buf;
    readies = g->rounds[round].ready;
  }
  // every rank's buffer, in rank order, into this rank's staging area
  for (int r = 0; r < W; ++r) {
    MLAMG_HIP(hipStreamWaitEvent(s, readies[r], 0));
    if (n) MLAMG_HIP(hipMemcpyAsync(c->ar_stage + (size_t)r * n, bufs[r], sizeof(double) * n,
                                    hipMemcpyDeviceToDevice, s));
  }
  MLAMG_HIP(hipEventCreateWithFlags(&copied, hipEventDisableTiming));
  MLAMG_HIP(hipEventRecord(copied, s));
  std::vector<hipEvent_t> copies;
  {
    std::unique_lock<std::mutex> lk(g->mu);
    LoopRound& R = g->rounds[round];
    R.copied[c->rank] = copied;
    ++R.finished;
    g->cv.notify_all();
    MLAMG_TRY(loop_wait(g, lk, [&] { return g->rounds[round].finished == W; }, "all-reduce copies"));
    copies = g->rounds[round].copied;
  }
  // nobody reads this rank's buffer any more once every copy is done: overwrite it
  for (int r = 0; r < W; ++r) MLAMG_HIP(hipStreamWaitEvent(s, copies[r], 0));
  if (n) {
    hipLaunchKernelGGL(k_loop_sum, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                       c->ar_stage, W, (int64_t)n, buf);
    MLAMG_HIP(hipGetLastError());
  }
  {
    std::lock_guard<std::mutex> lk(g->mu);
    LoopRound& R = g->rounds[round];
    if (++R.left == W) {  // last one out: the events have all been waited on by every stream
      for (auto e : R.ready) (void)hipEventDestroy(e);
      for (auto e : R.copied) (void)hipEventDestroy(e);
      g->rounds.erase(round);
    }
  }
  return MLAMG_OK;
}

__global__ void k_pack(const double* __restrict__ x, const int32_t* __restrict__ idx, int64_t n,
                       double* __restrict__ out) {
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i < n) out[i] = x[idx[i]];
}

static int halo_pack(mlamg_halo* h, const double* x_ext, hipStream_t s) {
  if (h->n_send) {
    hipLaunchKernelGGL(k_pack, dim3((h->n_send + 255) / 256), dim3(256), 0, s, x_ext, h->send_idx,
                       h->n_send, h->send_buf);
    MLAMG_HIP(hipGetLastError());
  }
  return MLAMG_OK;
}

// the grouped send/recv of a packed halo, on stream s
static int halo_post(mlamg_halo* h, double* x_ext, hipStream_t s) {
  if (h->nbr.empty()) return MLAMG_OK;
  MLAMG_TRY(xgroup_begin(h->c));
  for (size_t q = 0; q < h->nbr.size(); ++q) {
    if (h->send_cnt[q])
      MLAMG_TRY(xsend(h->c, h->send_buf + h->send_off[q], (size_t)h->send_cnt[q], h->nbr[q], s));
    if (h->recv_cnt[q])
      MLAMG_TRY(xrecv(h->c, x_ext + h->n_own + h->recv_off[q], (size_t)h->recv_cnt[q],
                      h->nbr[q], s));
  }
  return xgroup_end(h->c, s);
}

int halo_exchange_impl(mlamg_halo* h, double* x_ext, hipStream_t s) {
  MLAMG_TRY(halo_pack(h, x_ext, s));
  return halo_post(h, x_ext, s);
}

// sum the residual partials of this rank into partial[n] (fixed order)
__global__ __launch_bounds__(1024) void k_local_sum(double* __restrict__ partial, int n) {
  __shared__ double red[16];
  double s = 0.0;
  s = strided_sum(partial, n, threadIdx.x, 1024);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int i = 0; i < 16; ++i) t += red[i];
    partial[n] = t;
  }
}

__global__ void k_norm_finish(const double* __restrict__ sum, double* hist, int32_t* counter,
                              int32_t* done, double tol) {
  if (*done) return;  // converged earlier: every rank saw the same global norm
  const double nrm = sqrt(*sum);
  const int c = *counter;
  if (hist) hist[c] = nrm;
  *counter = c + 1;
  if (tol >= 0.0 && nrm <= tol) *done = 1;
}

}  // namespace mlamg

using namespace mlamg;

namespace {
// An operator split by rows for overlapping its halo exchange: part 1 is a run
// of rows that read no ghost entry, parts 0 and 2 the rows before and after it (either may be
// empty). Part k holds rows [r0[k], r0[k] + rows) of the operator, stored in the same order and
// in an exact-order kernel format, so every row's sum is the unsplit operator's bit for bit.
struct OpSplit {
  const mlamg_csr* m[3] = {nullptr, nullptr, nullptr};
  int64_t r0[3] = {0, 0, 0};
  bool on() const { return m[1] != nullptr; }
};

struct DLevel {
  const mlamg_csr* A = nullptr;  // n_own x (n_own + ghosts_x)
  const mlamg_csr* P = nullptr;  // n_own x (next own + ghosts_p) | n_own x n_c (last level)
  const mlamg_csr* R = nullptr;  // next own x (n_own + ghosts_r)
  const double* dinv = nullptr;
  mlamg_halo* hx = nullptr;
  mlamg_halo* hr = nullptr;
  mlamg_halo* hp = nullptr;  // halo of x_{l+1} for P (nullptr on the last partitioned level)
  OpSplit sA, sR, sP;        // row splits behind hx, hr, hp (optional)
  int64_t n_own = 0;
  // work (l > 0: x_ext, b own; every level: r_ext, t_ext; xp_ext = x_{l+1} for P)
  double* x_ext = nullptr;
  double* b = nullptr;
  double* r_ext = nullptr;
  double* t_ext = nullptr;
  double* xp_ext = nullptr;
};
}  // namespace

struct mlamg_dhier {
  mlamg_comm* c = nullptr;
  std::vector<DLevel> lv;
  mlamg_hier* coarse = nullptr;  // replicated levels K..L
  std::vector<int64_t> c_lo_all, c_hi_all;  // owned segments of the replicated space
  int64_t nc = 0;
  double* bc = nullptr;
  double* partial = nullptr;
  int32_t* flags = nullptr;  // counter, done
  std::vector<void*> bufs;
  bool ready = false;
  int coarse_graph = 1;
  // whole-cycle hipGraph (kernels + RCCL calls captured together), keyed like mlamg_hier's
  int cycle_graph = 0;
  bool capturing = false;
  hipStream_t cap_stream = nullptr;
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  const double* g_b = nullptr;
  double* g_x = nullptr;
  double* g_hist = nullptr;
  double g_tol = -1.0;
  uint64_t g_epoch = 0;
  int32_t* done_host = nullptr;  // pinned copy of the stop flag (run_cycles)
  // halo / interior overlap: the RCCL group of a split operator's exchange runs on comm_s while
  // the interior rows run on the cycle's stream (events fork and join the two)
  int overlap = 1;
  hipStream_t comm_s = nullptr;
  std::vector<hipEvent_t> evs;
  size_t ev_next = 0;
  int64_t part_cap = 0;
};

// the exchange of halo h into buf followed by the operator `whole`, through op(M, row0, part):
// unsplit, the exchange then op(whole, 0, -1); split, the pack on s, the RCCL group on comm_s
// (forked from s after the pack, so every earlier reader of the ghost region is done), the
// interior rows on s meanwhile, then s joins comm_s and runs the boundary rows
template <class Op>
static int exchange_then(mlamg_dhier* D, mlamg_halo* h, double* buf, const mlamg_csr* whole,
                         const OpSplit& sp, hipStream_t s, Op&& op) {
  if (!(D->overlap && sp.on() && !h->nbr.empty())) {
    MLAMG_TRY(halo_exchange_impl(h, buf, s));
    return op(whole, (int64_t)0, -1);
  }
  if (D->ev_next + 2 > D->evs.size()) {
    for (int q = 0; q < 16; ++q) {
      hipEvent_t e;
      MLAMG_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      D->evs.push_back(e);
    }
  }
  hipEvent_t fork = D->evs[D->ev_next++], join = D->evs[D->ev_next++];
  MLAMG_TRY(halo_pack(h, buf, s));
  MLAMG_HIP(hipEventRecord(fork, s));
  MLAMG_HIP(hipStreamWaitEvent(D->comm_s, fork, 0));
  MLAMG_TRY(halo_post(h, buf, D->comm_s));
  MLAMG_HIP(hipEventRecord(join, D->comm_s));
  MLAMG_TRY(op(sp.m[1], sp.r0[1], 1));
  MLAMG_HIP(hipStreamWaitEvent(s, join, 0));
  if (sp.m[0]) MLAMG_TRY(op(sp.m[0], sp.r0[0], 0));
  if (sp.m[2]) MLAMG_TRY(op(sp.m[2], sp.r0[2], 2));
  return MLAMG_OK;
}

static void dhier_free_graph(mlamg_dhier* D) {
  if (D->exec) (void)hipGraphExecDestroy(D->exec);
  if (D->graph) (void)hipGraphDestroy(D->graph);
  D->exec = nullptr;
  D->graph = nullptr;
}

extern "C" {

int mlamg_comm_unique_id(void* id_out) {
  MLAMG_REQUIRE(id_out, "NULL argument");
  ncclUniqueId id;
  MLAMG_NCCL(ncclGetUniqueId(&id));
  std::memcpy(id_out, &id, sizeof(id));
  return MLAMG_OK;
}

int mlamg_comm_create(const void* id, int nranks, int rank, mlamg_comm** out) {
  MLAMG_REQUIRE(id && out && nranks >= 1 && rank >= 0 && rank < nranks, "invalid argument");
  auto* c = new mlamg_comm();
  c->nranks = nranks;
  c->rank = rank;
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  ncclResult_t r = ncclCommInitRank(&c->comm, nranks, uid, rank);
  if (r != ncclSuccess) {
    delete c;
    set_error(std::string("ncclCommInitRank failed: ") + ncclGetErrorString(r));
    return MLAMG_ENCCL;
  }
  *out = c;
  return MLAMG_OK;
}

int mlamg_comm_info(const mlamg_comm* c, int* nranks_out, int* rank_out, int* device_out,
                    int* transport_out) {
  MLAMG_REQUIRE(c && nranks_out && rank_out, "NULL argument");
  if (c->comm) {  // as RCCL itself reports them
    MLAMG_NCCL(ncclCommCount(c->comm, nranks_out));
    MLAMG_NCCL(ncclCommUserRank(c->comm, rank_out));
    if (device_out) MLAMG_NCCL(ncclCommCuDevice(c->comm, device_out));
  } else {
    *nranks_out = c->nranks;
    *rank_out = c->rank;
    if (device_out) MLAMG_HIP(hipGetDevice(device_out));
  }
  if (transport_out) *transport_out = c->comm ? 0 : (c->loop ? 1 : 2);
  return MLAMG_OK;
}

int mlamg_comm_destroy(mlamg_comm* c) {
  if (c) {
    if (c->comm) (void)ncclCommDestroy(c->comm);
    if (c->ar_stage) (void)hipFree(c->ar_stage);
    if (c->loop) {
      std::lock_guard<std::mutex> lk(c->loop->mu);
      --c->loop->members;
    }
    delete c;
  }
  return MLAMG_OK;
}

int mlamg_loop_group_create(int nranks, mlamg_loop_group** out) {
  MLAMG_REQUIRE(out && nranks >= 1, "invalid argument");
  auto* g = new mlamg_loop_group();
  g->W = nranks;
  g->send_seq.assign((size_t)nranks * nranks, 0);
  g->recv_seq.assign((size_t)nranks * nranks, 0);
  *out = g;
  return MLAMG_OK;
}

int mlamg_loop_group_destroy(mlamg_loop_group* g) {
  if (g) {
    {
      std::lock_guard<std::mutex> lk(g->mu);
      MLAMG_REQUIRE(g->members == 0, "loop group still has communicators");
    }
    delete g;
  }
  return MLAMG_OK;
}

int mlamg_comm_create_null(int nranks, int rank, mlamg_comm** out) {
  MLAMG_REQUIRE(out && nranks >= 1 && rank >= 0 && rank < nranks, "invalid argument");
  auto* c = new mlamg_comm();
  c->nranks = nranks;
  c->rank = rank;
  c->null_transport = true;
  *out = c;
  return MLAMG_OK;
}

int mlamg_comm_create_loopback(mlamg_loop_group* g, int rank, mlamg_comm** out) {
  MLAMG_REQUIRE(g && out && rank >= 0 && rank < g->W, "invalid argument");
  auto* c = new mlamg_comm();
  c->nranks = g->W;
  c->rank = rank;
  c->loop = g;
  {
    std::lock_guard<std::mutex> lk(g->mu);
    ++g->members;
  }
  *out = c;
  return MLAMG_OK;
}

int mlamg_comm_allreduce_sum(mlamg_comm* c, double* buf, int64_t n, void* stream) {
  MLAMG_REQUIRE(c && (n == 0 || buf), "NULL argument");
  return xallreduce_sum(c, buf, (size_t)n, S(stream));
}

int mlamg_halo_create(mlamg_comm* c, int64_t n_own, int32_t n_nbr, const int32_t* nbr,
                      const int64_t* send_cnt, const int32_t* send_idx_host,
                      const int64_t* recv_cnt, mlamg_halo** out) {
  MLAMG_REQUIRE(c && out && n_own >= 0 && n_nbr >= 0, "invalid argument");
  MLAMG_REQUIRE(n_nbr == 0 || (nbr && send_cnt && recv_cnt), "NULL argument");
  auto* h = new mlamg_halo();
  h->c = c;
  h->n_own = n_own;
  int64_t so = 0, ro = 0;
  for (int q = 0; q < n_nbr; ++q) {
    if (nbr[q] < 0 || nbr[q] >= c->nranks || nbr[q] == c->rank || send_cnt[q] < 0 || recv_cnt[q] < 0) {
      delete h;
      set_error("mlamg_halo_create: invalid neighbour entry");
      return MLAMG_EINVAL;
    }
    h->nbr.push_back(nbr[q]);
    h->send_off.push_back(so);
    h->send_cnt.push_back(send_cnt[q]);
    h->recv_off.push_back(ro);
    h->recv_cnt.push_back(recv_cnt[q]);
    so += send_cnt[q];
    ro += recv_cnt[q];
  }
  h->n_send = so;
  h->n_ghost = ro;
  for (int64_t i = 0; i < so; ++i)
    if (send_idx_host[i] < 0 || send_idx_host[i] >= n_own) {
      delete h;
      set_error("mlamg_halo_create: send index out of range");
      return MLAMG_EINVAL;
    }
  if (so) {
    if (hipMalloc(&h->send_idx, sizeof(int32_t) * so) != hipSuccess ||
        hipMalloc(&h->send_buf, sizeof(double) * so) != hipSuccess ||
        hipMemcpy(h->send_idx, send_idx_host, sizeof(int32_t) * so, hipMemcpyHostToDevice) !=
            hipSuccess) {
      if (h->send_idx) (void)hipFree(h->send_idx);
      if (h->send_buf) (void)hipFree(h->send_buf);
      delete h;
      set_error("mlamg_halo_create: device allocation failed");
      return MLAMG_ENOMEM;
    }
  }
  *out = h;
  return MLAMG_OK;
}

int mlamg_halo_destroy(mlamg_halo* h) {
  if (h) {
    if (h->send_idx) (void)hipFree(h->send_idx);
    if (h->send_buf) (void)hipFree(h->send_buf);
    delete h;
  }
  return MLAMG_OK;
}

int mlamg_halo_exchange(mlamg_halo* h, double* x_ext, void* stream) {
  MLAMG_REQUIRE(h && (h->n_own + h->n_ghost == 0 || x_ext), "NULL argument");
  return halo_exchange_impl(h, x_ext, S(stream));
}

int mlamg_dhier_create(mlamg_comm* c, mlamg_hier* coarse, int64_t nc, const int64_t* c_lo_all,
                       const int64_t* c_hi_all, mlamg_dhier** out) {
  MLAMG_REQUIRE(c && coarse && c_lo_all && c_hi_all && out, "NULL argument");
  auto* D = new mlamg_dhier();
  D->c = c;
  D->coarse = coarse;
  D->nc = nc;
  D->c_lo_all.assign(c_lo_all, c_lo_all + c->nranks);
  D->c_hi_all.assign(c_hi_all, c_hi_all + c->nranks);
  for (int q = 0; q < c->nranks; ++q)
    if (D->c_lo_all[q] < 0 || D->c_hi_all[q] < D->c_lo_all[q] || D->c_hi_all[q] > nc ||
        (q > 0 && D->c_lo_all[q] != D->c_hi_all[q - 1])) {
      delete D;
      set_error("mlamg_dhier_create: coarse segments must tile [0, nc) in rank order");
      return MLAMG_EINVAL;
    }
  *out = D;
  return MLAMG_OK;
}

int mlamg_dhier_add_level(mlamg_dhier* D, const mlamg_csr* A_loc, const double* dinv_w,
                          const mlamg_csr* P_loc, const mlamg_csr* R_own, mlamg_halo* halo_x,
                          mlamg_halo* halo_r, mlamg_halo* halo_p) {
  MLAMG_REQUIRE(D && A_loc && dinv_w && P_loc && R_own && halo_x && halo_r, "NULL argument");
  MLAMG_REQUIRE(!D->ready, "hierarchy already in use");
  const int64_t n = A_loc->n_rows;
  MLAMG_REQUIRE(A_loc->n_cols == n + halo_x->n_ghost, "A_loc columns != n_own + x ghosts");
  MLAMG_REQUIRE(halo_x->n_own == n && halo_r->n_own == n, "halo n_own mismatch");
  MLAMG_REQUIRE(P_loc->n_rows == n + halo_x->n_ghost, "P_loc rows != n_own + x ghosts");
  MLAMG_REQUIRE(R_own->n_cols == n + halo_r->n_ghost, "R_own columns != n_own + r ghosts");
  if (!D->lv.empty()) {
    DLevel& up = D->lv.back();
    MLAMG_REQUIRE(up.hp != nullptr, "previous level was declared the last partitioned level");
    MLAMG_REQUIRE(up.R->n_rows == n, "level rows != owned coarse rows of the level above");
    MLAMG_REQUIRE(up.hp->n_own == n, "P halo of the level above has a different n_own");
    MLAMG_REQUIRE(up.P->n_cols == n + up.hp->n_ghost, "P_loc columns != next own + p ghosts");
  }
  if (!halo_p) {
    const int me = D->c->rank;
    MLAMG_REQUIRE(P_loc->n_cols == D->nc, "last level P must have the replicated coarse columns");
    MLAMG_REQUIRE(R_own->n_rows == D->c_hi_all[me] - D->c_lo_all[me],
                  "R_own rows != owned coarse segment");
  }
  DLevel L;
  L.A = A_loc;
  L.P = P_loc;
  L.R = R_own;
  L.dinv = dinv_w;
  L.hx = halo_x;
  L.hr = halo_r;
  L.hp = halo_p;
  L.n_own = n;
  D->lv.push_back(L);
  return MLAMG_OK;
}

int mlamg_dhier_set_split(mlamg_dhier* D, int level, int which, const mlamg_csr* lo,
                          const mlamg_csr* mid, const mlamg_csr* hi) {
  MLAMG_REQUIRE(D && mid, "NULL argument");
  MLAMG_REQUIRE(!D->ready, "hierarchy already in use");
  MLAMG_REQUIRE(level >= 0 && (size_t)level < D->lv.size(), "level out of range");
  MLAMG_REQUIRE(which >= 0 && which <= 2, "which: 0 = A, 1 = R, 2 = P");
  DLevel& L = D->lv[level];
  MLAMG_REQUIRE(which != 2 || L.hp, "P is split only where a P halo precedes it");
  const mlamg_csr* whole = which == 0 ? L.A : which == 1 ? L.R : L.P;
  OpSplit sp;
  sp.m[0] = lo;
  sp.m[1] = mid;
  sp.m[2] = hi;
  int64_t r = 0;
  for (int k = 0; k < 3; ++k) {
    sp.r0[k] = r;
    if (!sp.m[k]) continue;
    MLAMG_REQUIRE(sp.m[k]->n_cols == whole->n_cols, "split part has other columns");
    // the row-pair kernels load epilogue vectors as 16-byte pairs: parts start on even rows
    MLAMG_REQUIRE(r % 2 == 0, "split parts must start on even rows");
    r += sp.m[k]->n_rows;
  }
  MLAMG_REQUIRE(r == whole->n_rows, "split parts do not cover the operator's rows");
  (which == 0 ? L.sA : which == 1 ? L.sR : L.sP) = sp;
  return MLAMG_OK;
}

int mlamg_dhier_set_overlap(mlamg_dhier* D, int on) {
  MLAMG_REQUIRE(D, "NULL argument");
  D->overlap = on ? 1 : 0;
  dhier_free_graph(D);
  return MLAMG_OK;
}

int mlamg_dhier_destroy(mlamg_dhier* D) {
  if (D) {
    dhier_free_graph(D);
    if (D->cap_stream) (void)hipStreamDestroy(D->cap_stream);
    if (D->comm_s) (void)hipStreamDestroy(D->comm_s);
    for (hipEvent_t e : D->evs) (void)hipEventDestroy(e);
    if (D->done_host) (void)hipHostFree(D->done_host);
    for (void* p : D->bufs)
      if (p) (void)hipFree(p);
    delete D;
  }
  return MLAMG_OK;
}

int mlamg_dhier_set_coarse_graph(mlamg_dhier* D, int use_graph) {
  MLAMG_REQUIRE(D, "NULL argument");
  D->coarse_graph = use_graph;
  return MLAMG_OK;
}

int mlamg_dhier_set_cycle_graph(mlamg_dhier* D, int use_graph) {
  MLAMG_REQUIRE(D, "NULL argument");
  D->cycle_graph = use_graph;
  dhier_free_graph(D);
  return MLAMG_OK;
}

static int dalloc(mlamg_dhier* D, double** p, int64_t n) {
  void* q = nullptr;
  MLAMG_HIP(hipMalloc(&q, sizeof(double) * std::max<int64_t>(n, 1)));
  MLAMG_HIP(hipMemset(q, 0, sizeof(double) * std::max<int64_t>(n, 1)));
  D->bufs.push_back(q);
  *p = static_cast<double*>(q);
  return MLAMG_OK;
}

static int dprepare(mlamg_dhier* D) {
  if (D->ready) return MLAMG_OK;
  MLAMG_REQUIRE(!D->lv.empty(), "no partitioned level");
  MLAMG_REQUIRE(D->lv.back().hp == nullptr, "last partitioned level must have halo_p = NULL");
  for (size_t l = 0; l < D->lv.size(); ++l) {
    DLevel& L = D->lv[l];
    const int64_t ext = L.n_own + std::max(L.hx->n_ghost, L.hr->n_ghost);
    if (l > 0) {
      MLAMG_TRY(dalloc(D, &L.x_ext, ext));
      MLAMG_TRY(dalloc(D, &L.b, L.n_own));
    }
    MLAMG_TRY(dalloc(D, &L.r_ext, ext));
    // t_ext of level l > 0 doubles as the P-halo buffer (xp_ext) of level l - 1
    const int64_t pg = l > 0 ? D->lv[l - 1].hp->n_ghost : 0;
    MLAMG_TRY(dalloc(D, &L.t_ext, std::max(ext, L.n_own + pg)));
    if (l > 0) D->lv[l - 1].xp_ext = L.t_ext;
  }
  MLAMG_TRY(dalloc(D, &D->bc, D->nc));
  int64_t pc = part_capacity(D->lv[0].A), ps = 0;
  for (int k = 0; k < 3; ++k)
    if (D->lv[0].sA.m[k]) ps += part_capacity(D->lv[0].sA.m[k]);
  MLAMG_TRY(dalloc(D, &D->partial, std::max(pc, ps)));
  if (!D->comm_s) MLAMG_HIP(hipStreamCreateWithFlags(&D->comm_s, hipStreamNonBlocking));
  double* f = nullptr;
  MLAMG_TRY(dalloc(D, &f, 1));
  D->flags = reinterpret_cast<int32_t*>(f);
  // the zero fills run on the null stream and may still be in flight: finish them before work
  // on the caller's (possibly non-blocking) stream touches these buffers
  MLAMG_HIP(hipDeviceSynchronize());
  D->ready = true;
  return MLAMG_OK;
}

// allgatherv of the owned coarse segments into the replicated b_c
static int allgather_segments(mlamg_dhier* D, hipStream_t s) {
  const int P = D->c->nranks, me = D->c->rank;
  if (P == 1) return MLAMG_OK;
  const int64_t lo = D->c_lo_all[me];
  const size_t mine = (size_t)(D->c_hi_all[me] - lo);
  MLAMG_TRY(xgroup_begin(D->c));
  for (int q = 0; q < P; ++q) {
    if (q == me) continue;
    if (mine) MLAMG_TRY(xsend(D->c, D->bc + lo, mine, q, s));
    const size_t theirs = (size_t)(D->c_hi_all[q] - D->c_lo_all[q]);
    if (theirs) MLAMG_TRY(xrecv(D->c, D->bc + D->c_lo_all[q], theirs, q, s));
  }
  return xgroup_end(D->c, s);
}

static int dcycle_below(mlamg_dhier* D, size_t l, double** x_out, hipStream_t s);

// coarse-grid correction of partitioned level l: b_{l+1} = R r, solve below, x += P x_{l+1}
static int correct(mlamg_dhier* D, size_t l, double* x_ext, const int32_t* done, hipStream_t s) {
  DLevel& L = D->lv[l];
  if (L.hp) {
    DLevel& N = D->lv[l + 1];
    // restriction fused with the next level's zero-guess sweep (x = Dinv_w b on owned rows)
    MLAMG_TRY(exchange_then(D, L.hr, L.r_ext, L.R, L.sR, s,
                            [&](const mlamg_csr* M, int64_t r0, int) {
                              return spmv_set(M, L.r_ext, N.b + r0, done, s, N.x_ext + r0,
                                              N.dinv + r0);
                            }));
    double* xn = nullptr;
    MLAMG_TRY(dcycle_below(D, l + 1, &xn, s));
    // xp_ext is the level below's t_ext: its owned part is the correction, the P-halo lands in
    // its (no longer needed) ghost region. P rows cover the owned AND the x-ghost rows: x_ext's
    // ghosts get the same update their owners compute (same row, same order, same inputs), so
    // no x halo is needed afterwards
    MLAMG_TRY(exchange_then(D, L.hp, L.xp_ext, L.P, L.sP, s,
                            [&](const mlamg_csr* M, int64_t r0, int) {
                              return spmv_add(M, L.xp_ext, x_ext + r0, done, s);
                            }));
  } else {
    const int me = D->c->rank;
    double* bo = D->bc + D->c_lo_all[me];
    MLAMG_TRY(exchange_then(D, L.hr, L.r_ext, L.R, L.sR, s,
                            [&](const mlamg_csr* M, int64_t r0, int) {
                              return spmv_set(M, L.r_ext, bo + r0, done, s);
                            }));
    MLAMG_TRY(allgather_segments(D, s));
    double* xc = nullptr;
    // inside a whole-cycle capture the coarse kernels are captured directly (no nested graph)
    MLAMG_TRY(hier_coarse_cycle(D->coarse, D->bc, &xc, D->coarse_graph && !D->capturing, s));
    MLAMG_TRY(spmv_add(L.P, xc, x_ext, done, s));
  }
  return MLAMG_OK;
}

// one cycle from a zero guess at partitioned level l > 0 (rhs in lv[l].b); result (own part)
// returned through x_out
static int dcycle_below(mlamg_dhier* D, size_t l, double** x_out, hipStream_t s) {
  const int32_t* done = D->flags + 1;
  DLevel& L = D->lv[l];
  // x = Dinv_w b was written by the restriction kernel of the level above (correct())
  MLAMG_TRY(exchange_then(D, L.hx, L.x_ext, L.A, L.sA, s,
                          [&](const mlamg_csr* M, int64_t r0, int) {
                            return residual_impl(M, L.b + r0, L.x_ext, L.r_ext + r0, nullptr,
                                                 nullptr, nullptr, const_cast<int32_t*>(done),
                                                 kNoTol, nullptr, nullptr, nullptr, s);
                          }));
  MLAMG_TRY(correct(D, l, L.x_ext, done, s));
  MLAMG_TRY(jacobi_sweep(L.A, L.dinv, L.b, L.x_ext, L.t_ext, false, done, s));
  *x_out = L.t_ext;
  return MLAMG_OK;
}

// Fused as in hier.hip: the end-of-cycle residual kernel also writes x = t + Dinv_w r (the next
// cycle's first pre-smoothing sweep); the caller applies the first sweep before the first cycle
// and copies t (still in t_ext) back into x after the last.
static int dcycle(mlamg_dhier* D, const double* b, double* x_ext, double* hist, double tol,
                  hipStream_t s) {
  int32_t* counter = D->flags;
  int32_t* done = D->flags + 1;
  DLevel& L = D->lv[0];
  const mlamg_csr* A = L.A;
  D->ev_next = 0;
  MLAMG_TRY(exchange_then(D, L.hx, x_ext, A, L.sA, s, [&](const mlamg_csr* M, int64_t r0, int) {
    return residual_impl(M, b ? b + r0 : nullptr, x_ext, L.r_ext + r0, nullptr, nullptr, nullptr,
                         done, kNoTol, nullptr, nullptr, nullptr, s);
  }));
  MLAMG_TRY(correct(D, 0, x_ext, done, s));
  MLAMG_TRY(jacobi_sweep(A, L.dinv, b, x_ext, L.t_ext, false, done, s));
  // r = b - A t with per-block ||r||^2 partials, x <- t; then the global norm
  // (r itself is not stored: the next cycle starts with its own residual). Split: the parts'
  // partials lie in part order (0, 1, 2), whatever order the parts ran in. The parts' row
  // blocks are cut differently from the unsplit operator's, so the NORM (history, tolerance
  // stop) matches overlap-off / single-GPU runs to rounding, not bitwise; the iterate itself is
  // bitwise unchanged (every row is summed in its stored order)
  int64_t poff[3] = {0, 0, 0};
  int nb = (int)A->n_part;
  if (D->overlap && L.sA.on() && !L.hx->nbr.empty()) {
    nb = 0;
    for (int k = 0; k < 3; ++k) {
      poff[k] = nb;
      if (L.sA.m[k]) nb += (int)L.sA.m[k]->n_part;
    }
  }
  MLAMG_TRY(exchange_then(D, L.hx, L.t_ext, A, L.sA, s,
                          [&](const mlamg_csr* M, int64_t r0, int part) {
                            return residual_partials(M, b ? b + r0 : nullptr, L.t_ext, nullptr,
                                                     x_ext + r0,
                                                     L.t_ext + r0,
                                                     D->partial + (part < 0 ? 0 : poff[part]),
                                                     done, s, L.dinv + r0);
                          }));
  hipLaunchKernelGGL(k_local_sum, dim3(1), dim3(1024), 0, s, D->partial, nb);
  MLAMG_HIP(hipGetLastError());
  if (D->c->nranks > 1) MLAMG_TRY(xallreduce_sum(D->c, D->partial + nb, 1, s));
  hipLaunchKernelGGL(k_norm_finish, dim3(1), dim3(1), 0, s, D->partial + nb, hist, counter, done,
                     tol);
  MLAMG_HIP(hipGetLastError());
  return MLAMG_OK;
}

int mlamg_dhier_vcycle(mlamg_dhier* D, const double* b, double* x_ext, int n_cycles, double tol,
                       double* res_hist, int32_t* cycles_done_host, void* stream) {
  // b NULL: this rank's part of the right-hand side is zero (as mlamg_hier_vcycle: the
  // fine-level kernels take +0.0 instead of reading b; same bits)
  MLAMG_REQUIRE(D && x_ext, "NULL argument");
  MLAMG_REQUIRE(n_cycles >= 0, "n_cycles < 0");
  MLAMG_TRY(dprepare(D));
  hipStream_t s = S(stream);
  DLevel& L = D->lv[0];
  MLAMG_HIP(hipMemsetAsync(D->flags, 0, 2 * sizeof(int32_t), s));
  MLAMG_TRY(halo_exchange_impl(L.hx, x_ext, s));
  MLAMG_TRY(residual_impl(L.A, b, x_ext, L.r_ext, nullptr, nullptr, nullptr, nullptr, kNoTol,
                          nullptr, nullptr, nullptr, s));
  if (n_cycles > 0) {
    // the first cycle's first pre-smoothing sweep (later ones are fused into the cycle end)
    MLAMG_TRY(jacobi_from_residual(x_ext, L.dinv, L.r_ext, L.n_own, nullptr, s));
    MLAMG_REQUIRE(!(D->cycle_graph && D->c->loop),
                  "the loopback transport cannot be captured into a graph");
    if (D->cycle_graph) {
      int c0 = 0;
      if (!(D->exec && D->g_b == b && D->g_x == x_ext && D->g_hist == res_hist &&
            D->g_tol == tol && D->g_epoch == format_epoch())) {
        // the first cycle runs eagerly: every RCCL peer connection (halo neighbours, the
        // allgather of coarse segments, the norm all-reduce) is set up outside the capture
        MLAMG_TRY(dcycle(D, b, x_ext, res_hist, tol, s));
        c0 = 1;
        dhier_free_graph(D);
        MLAMG_TRY(hier_prepare_ext(D->coarse));
        if (!D->cap_stream)
          MLAMG_HIP(hipStreamCreateWithFlags(&D->cap_stream, hipStreamNonBlocking));
        // order the capture stream after the work already queued on s
        hipEvent_t ev;
        MLAMG_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        MLAMG_HIP(hipEventRecord(ev, s));
        MLAMG_HIP(hipStreamWaitEvent(D->cap_stream, ev, 0));
        MLAMG_HIP(hipStreamSynchronize(D->cap_stream));
        (void)hipEventDestroy(ev);
        MLAMG_HIP(hipStreamBeginCapture(D->cap_stream, hipStreamCaptureModeThreadLocal));
        D->capturing = true;
        int rc = dcycle(D, b, x_ext, res_hist, tol, D->cap_stream);
        D->capturing = false;
        hipGraph_t g = nullptr;
        hipError_t e = hipStreamEndCapture(D->cap_stream, &g);
        if (rc != MLAMG_OK) {
          if (g) (void)hipGraphDestroy(g);
          return rc;
        }
        MLAMG_HIP(e);
        D->graph = g;
        MLAMG_HIP(hipGraphInstantiate(&D->exec, g, nullptr, nullptr, 0));
        D->g_b = b;
        D->g_x = x_ext;
        D->g_hist = res_hist;
        D->g_tol = tol;
        D->g_epoch = format_epoch();
      }
      if (!D->done_host) (void)hipHostMalloc(&D->done_host, sizeof(int32_t), hipHostMallocDefault);
      MLAMG_TRY(run_cycles(n_cycles - c0, tol, D->flags + 1, D->done_host, s, [&]() -> int {
        MLAMG_HIP(hipGraphLaunch(D->exec, s));
        return MLAMG_OK;
      }));
    } else {
      // every rank reads the same flag (set from the all-reduced norm) after the same batch,
      // so all ranks launch the same number of cycles and their collectives stay matched
      if (!D->done_host) (void)hipHostMalloc(&D->done_host, sizeof(int32_t), hipHostMallocDefault);
      MLAMG_TRY(run_cycles(n_cycles, tol, D->flags + 1, D->done_host, s,
                           [&]() { return dcycle(D, b, x_ext, res_hist, tol, s); }));
    }
    // the iterate is t; x holds t + Dinv_w r for a cycle that never ran
    MLAMG_HIP(hipMemcpyAsync(x_ext, L.t_ext, sizeof(double) * L.n_own, hipMemcpyDeviceToDevice, s));
  }
  if (cycles_done_host) {
    int32_t cnt = 0;
    MLAMG_HIP(hipMemcpyAsync(&cnt, D->flags, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    MLAMG_HIP(hipStreamSynchronize(s));
    *cycles_done_host = cnt;
  }
  return MLAMG_OK;
}

}  // extern "C"
