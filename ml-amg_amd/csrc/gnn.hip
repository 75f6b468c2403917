// GNN inference for learned aggregates and interpolation: the layers of
// ns/model/agg_interp.py FullAggNet.forward (:432-486) — AggNet's TAGConv/InstanceNorm/MLP
// node scorer, MPNN's NNConv/InstanceNorm/edge models (CNet, PNet) — on the device, fp32 like
// the reference (torch_geometric 2.x semantics, restated; torch_geometric is absent here).
//
// A graph is the CSR pattern of A (graph_from_matrix[_basic], ns/model/data.py:22-46): edge e =
// stored entry (i, j) in row-major order, source i = edge_index[0], target j = edge_index[1];
// messages flow source -> target and are summed at the target in edge order (the CSR of the
// transpose lists a target's incoming edges with ascending source), so every aggregation is
// deterministic. Dense layers use torch's Linear layout (weight [out, in], y = x W^T + b).
#include "common.hpp"

#include <rocprim/rocprim.hpp>

namespace mlamg {
namespace {

constexpr int kT = 256;

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
__device__ __forceinline__ float wsumf(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Y[m][n] = beta * Y[m][n] + sum_k X[m][k] W[n][k] (+ b[n]) -> act -> (+ R[m][n or 0]).
// A block stages W^T in LDS (K <= 160, N <= 64) and takes 256 / NP rows at a time, NP = N
// rounded up to a power of two; lane n of a row reads W^T[k][n] (consecutive: no conflicts) and
// the row's X[m][k] (one address: broadcast).
__global__ void k_linear(const float* __restrict__ X, int64_t M, int K, const float* __restrict__ W,
                         const float* __restrict__ b, int N, int NP, int act, float beta,
                         const float* __restrict__ R, int rc, float* __restrict__ Y) {
  extern __shared__ float wt[];  // K x N
  for (int q = threadIdx.x; q < K * N; q += kT) {
    const int k = q / N, n = q % N;
    wt[q] = W[(int64_t)n * K + k];
  }
  __syncthreads();
  const int rows = kT / NP;
  const int r = threadIdx.x / NP, n = threadIdx.x % NP;
  if (n >= N) return;
  for (int64_t m = (int64_t)blockIdx.x * rows + r; m < M; m += (int64_t)gridDim.x * rows) {
    const float* x = X + m * K;
    float acc = 0.0f;
    for (int k = 0; k < K; ++k) acc = fmaf(x[k], wt[k * N + n], acc);
    if (b) acc = acc + b[n];
    float y = beta != 0.0f ? beta * Y[m * N + n] + acc : acc;
    if (act == 1) y = fmaxf(y, 0.0f);
    if (R) y = y + R[m * rc + (rc == 1 ? 0 : n)];
    Y[m * N + n] = y;
  }
}

// y_i = sum over incoming edges e (tptr/teid: edges by target, ascending source) of
// w_e x_src(e); a wave per target, lane f < F
__global__ void k_propagate(const int32_t* __restrict__ tptr, const int32_t* __restrict__ teid,
                            const int32_t* __restrict__ src, const float* __restrict__ w,
                            const float* __restrict__ X, int64_t n, int F, float* __restrict__ Y) {
  const int64_t i = (int64_t)blockIdx.x * (kT / 64) + threadIdx.x / 64;
  const int f = threadIdx.x & 63;
  if (i >= n || f >= F) return;
  float acc = 0.0f;
  for (int32_t q = tptr[i]; q < tptr[i + 1]; ++q) {
    const int32_t e = teid[q];
    acc = fmaf(w[e], X[(int64_t)src[e] * F + f], acc);
  }
  Y[i * F + f] = acc;
}

// gcn_norm without self loops (TAGConv normalize=True): deg_j = sum of w over edges with
// target j; w'_e = deg^-1/2[src] w_e deg^-1/2[tgt] (inf -> 0)
__global__ void k_deg_isqrt(const int32_t* __restrict__ tptr, const int32_t* __restrict__ teid,
                            const float* __restrict__ w, int64_t n, float* __restrict__ dis) {
  const int64_t j = (int64_t)blockIdx.x * kT + threadIdx.x;
  if (j >= n) return;
  float d = 0.0f;
  for (int32_t q = tptr[j]; q < tptr[j + 1]; ++q) d += w[teid[q]];
  const float r = 1.0f / sqrtf(d);
  dis[j] = isinf(r) ? 0.0f : r;
}
__global__ void k_gcn_weight(const int32_t* __restrict__ src, const int32_t* __restrict__ tgt,
                             const float* __restrict__ w, int64_t E, int wstride,
                             const float* __restrict__ dis, float* __restrict__ wn) {
  const int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x;
  if (e >= E) return;
  wn[e] = (dis[src[e]] * w[e * wstride]) * dis[tgt[e]];
}

// instance norm over nodes, per channel (affine False, biased variance, eps): a block per channel
__global__ void k_inorm(const float* __restrict__ X, int64_t n, int F, float eps,
                        float* __restrict__ Y) {
  __shared__ double red[kT / 64];
  const int f = blockIdx.x;
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += kT) s += X[i * F + f];
  s = wsum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x / 64] = s;
  __syncthreads();
  double tot = 0.0;
  for (int w = 0; w < kT / 64; ++w) tot += red[w];
  const double mean = tot / (double)n;
  __syncthreads();
  double v = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += kT) {
    const double d = X[i * F + f] - mean;
    v += d * d;
  }
  v = wsum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x / 64] = v;
  __syncthreads();
  double vt = 0.0;
  for (int w = 0; w < kT / 64; ++w) vt += red[w];
  const float inv = (float)(1.0 / sqrt(vt / (double)n + (double)eps));
  const float mf = (float)mean;
  for (int64_t i = threadIdx.x; i < n; i += kT) Y[i * F + f] = (X[i * F + f] - mf) * inv;
}

// NNConv messages, the edge network fused in: per edge e (features ea[e][0..fe)),
//   h1 = relu(L1 ea + c1) (4), h2 = relu(L2 h1 + c2) (16), W_e = relu(L3 h2 + c3) [Fin x Fout],
//   msg[e][o] = sum_i x_src[i] W_e[i][o]   (NNConv.message: x_j @ weight.view(-1, in, out))
// A block: 64 edges (one per lane) x up to 4 output blocks of 16 (one per wave): every lane of a
// wave reads the same L3 row (broadcast), its own source row.
__global__ void k_nnconv_msg(const int32_t* __restrict__ src, const float* __restrict__ ea,
                             int64_t E, int fe, const float* __restrict__ L1,
                             const float* __restrict__ c1, const float* __restrict__ L2,
                             const float* __restrict__ c2, const float* __restrict__ L3,
                             const float* __restrict__ c3, const float* __restrict__ X, int Fin,
                             int Fout, float* __restrict__ msg) {
  const int lane = threadIdx.x & 63, ob = threadIdx.x >> 6;
  const int64_t e = (int64_t)blockIdx.x * 64 + lane;
  const int o0 = ob * 16;
  if (o0 >= Fout) return;
  const bool live = e < E;
  const int64_t ee = live ? e : 0;
  float h1[4], h2[16];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    float s = 0.0f;
    for (int t = 0; t < fe; ++t) s = fmaf(L1[a * fe + t], ea[ee * fe + t], s);
    h1[a] = fmaxf(s + c1[a], 0.0f);
  }
#pragma unroll
  for (int a = 0; a < 16; ++a) {
    float s = 0.0f;
#pragma unroll
    for (int t = 0; t < 4; ++t) s = fmaf(L2[a * 4 + t], h1[t], s);
    h2[a] = fmaxf(s + c2[a], 0.0f);
  }
  const float* xs = X + (int64_t)src[ee] * Fin;
  float acc[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) acc[u] = 0.0f;
  const int no = min(16, Fout - o0);
  for (int i = 0; i < Fin; ++i) {
    const float xi = xs[i];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if (u < no) {
        const int row = i * Fout + o0 + u;
        const float* l = L3 + (int64_t)row * 16;
        float s = 0.0f;
#pragma unroll
        for (int t = 0; t < 16; ++t) s = fmaf(l[t], h2[t], s);
        const float w = fmaxf(s + c3[row], 0.0f);
        acc[u] = fmaf(xi, w, acc[u]);
      }
    }
  }
  if (!live) return;
#pragma unroll
  for (int u = 0; u < 16; ++u)
    if (u < no) msg[e * Fout + o0 + u] = acc[u];
}

// out[i][o] = act(sum_{incoming e} msg[e][o] + root[i][o] + bias[o]) (+ R[i][o or 0])
__global__ void k_nnconv_aggr(const int32_t* __restrict__ tptr, const int32_t* __restrict__ teid,
                              const float* __restrict__ msg, const float* __restrict__ root,
                              const float* __restrict__ bias, int64_t n, int F, int act,
                              const float* __restrict__ R, int rc, float* __restrict__ Y) {
  const int64_t i = (int64_t)blockIdx.x * (kT / 64) + threadIdx.x / 64;
  const int f = threadIdx.x & 63;
  if (i >= n || f >= F) return;
  float s = 0.0f;
  for (int32_t q = tptr[i]; q < tptr[i + 1]; ++q) s += msg[(int64_t)teid[q] * F + f];
  float y = (s + root[i * F + f]) + bias[f];
  if (act == 1) y = fmaxf(y, 0.0f);
  if (R) y = y + R[i * rc + (rc == 1 ? 0 : f)];
  Y[i * F + f] = y;
}

// smallEdgeModel (agg_interp.py:37-55) and MPNN's post-ops (:124-141): a wave per edge,
//   in = [x_src (F) | x_tgt (F) | ea (fe)], h = relu(W1 in + b1) (H <= 64, lane o),
//   h = LayerNorm(h) * g + beta (eps 1e-5, biased variance), y_c = W2[c] . h + b2[c] (C <= 2),
//   out = act(y) (+ R[e][c or 0]).
__global__ void k_edge_mlp(const int32_t* __restrict__ src, const int32_t* __restrict__ tgt,
                           const float* __restrict__ X, int F, const float* __restrict__ ea,
                           int fe, int64_t E, const float* __restrict__ W1,
                           const float* __restrict__ b1, int H, const float* __restrict__ g,
                           const float* __restrict__ beta, const float* __restrict__ W2,
                           const float* __restrict__ b2, int C, int act,
                           const float* __restrict__ R, int rc, float* __restrict__ out) {
  extern __shared__ float w1t[];  // K x H, K = 2F + fe
  const int K = 2 * F + fe;
  for (int q = threadIdx.x; q < K * H; q += kT) w1t[q] = W1[(int64_t)(q % H) * K + q / H];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t e = (int64_t)blockIdx.x * (kT / 64) + threadIdx.x / 64;
  if (e >= E) return;
  const float* xs = X + (int64_t)src[e] * F;
  const float* xt = X + (int64_t)tgt[e] * F;
  const float* a = ea + e * fe;
  float h = 0.0f;
  if (lane < H) {
    for (int k = 0; k < F; ++k) h = fmaf(xs[k], w1t[k * H + lane], h);
    for (int k = 0; k < F; ++k) h = fmaf(xt[k], w1t[(F + k) * H + lane], h);
    for (int k = 0; k < fe; ++k) h = fmaf(a[k], w1t[(2 * F + k) * H + lane], h);
    h = fmaxf(h + b1[lane], 0.0f);
  }
  const float mean = wsumf(lane < H ? h : 0.0f) / (float)H;
  const float d = lane < H ? h - mean : 0.0f;
  const float var = wsumf(d * d) / (float)H;
  const float hn = lane < H ? (d / sqrtf(var + 1e-5f)) * g[lane] + beta[lane] : 0.0f;
  for (int c = 0; c < C; ++c) {
    float y = wsumf(lane < H ? hn * W2[c * H + lane] : 0.0f) + b2[c];
    if (act == 1) y = fmaxf(y, 0.0f);
    if (R) y = y + R[e * rc + (rc == 1 ? 0 : c)];
    if (lane == 0) out[e * C + c] = y;
  }
}

// top-k: keys ordered by descending score, then ascending node index
__global__ void k_topk_keys(const float* __restrict__ s, int64_t n, uint64_t* __restrict__ key) {
  const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  uint32_t u = __float_as_uint(s[i]);
  u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);  // ascending order of the float
  key[i] = ((uint64_t)(~u) << 32) | (uint64_t)i;
}
__global__ void k_topk_mark(const uint64_t* __restrict__ key, int64_t k, float* __restrict__ vec,
                            int32_t* __restrict__ idx) {
  const int64_t q = (int64_t)blockIdx.x * kT + threadIdx.x;
  if (q >= k) return;
  const int32_t i = (int32_t)(key[q] & 0xffffffffu);
  vec[i] = 1.0f;
  if (idx) idx[q] = i;
}

inline unsigned blocks(int64_t n, int per) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + per - 1) / per, 1 << 20));
}

}  // namespace
}  // namespace mlamg

using namespace mlamg;

extern "C" {

int mlamg_gnn_linear(const float* X, int64_t M, int K, const float* W, const float* b, int N,
                     int act, float beta, const float* R, int rc, float* Y, void* stream) {
  MLAMG_REQUIRE(M >= 0 && K >= 1 && K <= 160 && N >= 1 && N <= 64, "linear: K <= 160, N <= 64");
  MLAMG_REQUIRE(X && W && Y && (!R || rc == 1 || rc == N), "linear: bad arguments");
  if (M == 0) return MLAMG_OK;
  int NP = 1;
  while (NP < N) NP <<= 1;
  const int rows = kT / NP;
  hipLaunchKernelGGL(k_linear, dim3(blocks(M, rows)), dim3(kT), sizeof(float) * K * N, S(stream),
                     X, M, K, W, b, N, NP, act, beta, R, rc, Y);
  MLAMG_HIP(hipGetLastError());
  return MLAMG_OK;
}

int mlamg_gnn_gcn_norm(const int32_t* tptr, const int32_t* teid, const int32_t* src,
                       const int32_t* tgt, const float* w, int64_t n, int64_t E, float* dis_tmp,
                       float* wn, void* stream) {
  MLAMG_REQUIRE(tptr && teid && src && tgt && w && dis_tmp && wn, "NULL argument");
  hipStream_t s = S(stream);
  hipLaunchKernelGGL(k_deg_isqrt, dim3(blocks(n, kT)), dim3(kT), 0, s, tptr, teid, w, n, dis_tmp);
  if (E > 0)
    hipLaunchKernelGGL(k_gcn_weight, dim3(blocks(E, kT)), dim3(kT), 0, s, src, tgt, w, E, 1,
                       dis_tmp, wn);
  MLAMG_HIP(hipGetLastError());
  return MLAMG_OK;
}

int mlamg_gnn_propagate(const int32_t* tptr, const int32_t* teid, const int32_t* src,
                        const float* w, const float* X, int64_t n, int F, float* Y,
                        void* stream) {
  MLAMG_REQUIRE(F >= 1 && F <= 64, "propagate: F <= 64");
  hipLaunchKernelGGL(k_propagate, dim3(blocks(n, kT / 64)), dim3(kT), 0, S(stream), tptr, teid,
                     src, w, X, n, F, Y);
  MLAMG_HIP(hipGetLastError());
  return MLAMG_OK;
}

int mlamg_gnn_instance_norm(const float* X, int64_t n, int F, float eps, float* Y, void* stream) {
  MLAMG_REQUIRE(n >= 1 && F >= 1, "instance norm: empty input");
  hipLaunchKernelGGL(k_inorm, dim3(F), dim3(kT), 0, S(stream), X, n, F, eps, Y);
  MLAMG_HIP(hipGetLastError());
  return MLAMG_OK;
}

int mlamg_gnn_nnconv(const int32_t* tptr, const int32_t* teid, const int32_t* src,
                     const float* ea, int64_t E, int fe, const float* L1, const float* c1,
                     const float* L2, const float* c2, const float* L3, const float* c3,
                     const float* X, int64_t n, int Fin, int Fout, const float* root,
                     const float* bias, int act, const float* R, int rc, float* msg_tmp,
                     float* Y, void* stream) {
  MLAMG_REQUIRE(Fout >= 1 && Fout <= 64 && Fin >= 1 && fe >= 1, "nnconv: Fout <= 64");
  MLAMG_REQUIRE(root && bias && msg_tmp && Y, "NULL argument");
  hipStream_t s = S(stream);
  if (E > 0)
    hipLaunchKernelGGL(k_nnconv_msg, dim3(blocks(E, 64)), dim3(kT), 0, s, src, ea, E, fe, L1, c1,
                       L2, c2, L3, c3, X, Fin, Fout, msg_tmp);
  hipLaunchKernelGGL(k_nnconv_aggr, dim3(blocks(n, kT / 64)), dim3(kT), 0, s, tptr, teid,
                     msg_tmp, root, bias, n, Fout, act, R, rc, Y);
  MLAMG_HIP(hipGetLastError());
  return MLAMG_OK;
}

int mlamg_gnn_edge_mlp(const int32_t* src, const int32_t* tgt, const float* X, int F,
                       const float* ea, int fe, int64_t E, const float* W1, const float* b1,
                       int H, const float* g, const float* beta, const float* W2,
                       const float* b2, int C, int act, const float* R, int rc, float* out,
                       void* stream) {
  MLAMG_REQUIRE(H >= 1 && H <= 64 && C >= 1 && C <= 4 && 2 * F + fe <= 160, "edge mlp: sizes");
  if (E == 0) return MLAMG_OK;
  hipLaunchKernelGGL(k_edge_mlp, dim3(blocks(E, kT / 64)), dim3(kT),
                     sizeof(float) * (2 * F + fe) * H, S(stream), src, tgt, X, F, ea, fe, E, W1,
                     b1, H, g, beta, W2, b2, C, act, R, rc, out);
  MLAMG_HIP(hipGetLastError());
  return MLAMG_OK;
}

int mlamg_gnn_topk(const float* scores, int64_t n, int64_t k, float* vec, int32_t* idx,
                   void* stream) {
  MLAMG_REQUIRE(scores && vec && k >= 0 && k <= n, "topk: bad arguments");
  hipStream_t s = S(stream);
  uint64_t *k0 = nullptr, *k1 = nullptr;
  void* tmp = nullptr;
  size_t tb = 0;
  MLAMG_HIP(hipMalloc(&k0, sizeof(uint64_t) * std::max<int64_t>(n, 1)));
  hipError_t e = hipMalloc(&k1, sizeof(uint64_t) * std::max<int64_t>(n, 1));
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_topk_keys, dim3(blocks(n, kT)), dim3(kT), 0, s, scores, n, k0);
    e = rocprim::radix_sort_keys(nullptr, tb, k0, k1, (size_t)n, 0, 64, s);
  }
  if (e == hipSuccess) e = hipMalloc(&tmp, std::max<size_t>(tb, 1));
  if (e == hipSuccess) e = rocprim::radix_sort_keys(tmp, tb, k0, k1, (size_t)n, 0, 64, s);
  if (e == hipSuccess) e = hipMemsetAsync(vec, 0, sizeof(float) * n, s);
  if (e == hipSuccess && k > 0)
    hipLaunchKernelGGL(k_topk_mark, dim3(blocks(k, kT)), dim3(kT), 0, s, k1, k, vec, idx);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  (void)hipFree(tmp);
  (void)hipFree(k1);
  (void)hipFree(k0);
  if (e != hipSuccess) {
    set_error(std::string("topk: ") + hipGetErrorString(e));
    return MLAMG_EHIP;
  }
  return MLAMG_OK;
}

}  // extern "C"
