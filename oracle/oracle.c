/*
 * oracle.c — TEST INFRASTRUCTURE ONLY. CPU restatement of the reference hot-path loops that
 * live in compiled third-party code or in slow pure-Python loops, used by tests/ and by
 * bench.py's cpu_baseline leg as the checker. Never linked into, or called by, the product
 * (ml-amg_amd/mlamg). Built with -ffp-contract=off so every multiply and add rounds separately,
 * like scipy/pyamg on x86-64.
 *
 *   ref_csr_matvec          scipy sparsetools csr_matvec (A@x at ns/lib/multigrid.py:181,191)
 *   ref_gauss_seidel        pyamg 4.x amg_core gauss_seidel, forward sweep (multigrid.py:175,184)
 *   pyamg_gauss_seidel      the same in pyamg's three sweep directions (relaxation.gauss_seidel)
 *   ref_bellman_ford_torch  ns/lib/graph.py:28-53 modified_bellman_ford (fp32, sequential push
 *                           over coalesced COO order, strict <)
 *   canon_bellman_ford      same distances (order-independent fixed point) with the device's
 *                           order-independent label rule (min seed id over tight edges)
 *   pyamg_bellman_ford      pyamg 4.x graph.bellman_ford (ns/model/agg_interp.py:475): amg_core
 *                           pull sweeps over the rows in order, in place, strict <, in the
 *                           graph's dtype (float32: the CNet weights), until no distance changes
 *   ref_lloyd_cluster       pyamg 4.x amg_core lloyd_cluster + graph.lloyd_cluster driver loop
 *                           (called at ns/lib/graph.py:232), sequential
 *   canon_lloyd_cluster     same with the device's label rule (min cluster index over tight
 *                           pull neighbours)
 *   pyamg_symmetric_strength, pyamg_standard_aggregation, pyamg_block_gauss_seidel,
 *   pyamg_fit_candidates    pyamg 4.x/5.x amg_core symmetric_strength_of_connection,
 *                           standard_aggregation, block_gauss_seidel (1 x 1 blocks) and
 *                           fit_candidates_common (one candidate): the setup and smoother of
 *                           pyamg.aggregation.smoothed_aggregation_solver, which the reference's
 *                           PyAMG preconditioner builds (ns/preconditioner/PyAMG.py:94). pyamg is
 *                           absent: restated from its published algorithm, parity unpinned.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

void ref_csr_matvec(int64_t n, const int32_t* ip, const int32_t* ij, const double* ax,
                    const double* x, double* y) {
  for (int64_t i = 0; i < n; ++i) {
    double s = 0.0; /* Yx zero-initialised by A@x */
    for (int32_t k = ip[i]; k < ip[i + 1]; ++k) s += ax[k] * x[ij[k]];
    y[i] = s;
  }
}

/* device CSR-vector order (spmv.hip k_csr_vcan, every width 64..512 alike): 512 virtual lanes;
 * virtual lane v = 64 w + l sums the row's entries v, v + 512, ... left to right from +0.0; each
 * virtual wave w folds its 64 lanes with an xor butterfly (off = 32 .. 1: lane l becomes
 * a[l] + a[l ^ off]); the row is ((ws_0 + ws_1) + ...) + ws_7. */
void vec_matvec(int64_t n, const int32_t* ip, const int32_t* ij, const double* ax,
                const double* x, double* y) {
  double part[512], nxt[64];
  for (int64_t i = 0; i < n; ++i) {
    for (int v = 0; v < 512; ++v) {
      double s = 0.0;
      for (int32_t k = ip[i] + v; k < ip[i + 1]; k += 512) s += ax[k] * x[ij[k]];
      part[v] = s;
    }
    double r = 0.0;
    for (int w = 0; w < 8; ++w) {
      double* a = part + 64 * w;
      for (int off = 32; off > 0; off >>= 1) {
        for (int l = 0; l < 64; ++l) nxt[l] = a[l] + a[l ^ off];
        for (int l = 0; l < 64; ++l) a[l] = nxt[l];
      }
      r = w == 0 ? a[0] : r + a[0];
    }
    y[i] = r;
  }
}

void ref_gauss_seidel(int64_t n, const int32_t* ip, const int32_t* ij, const double* ax,
                      double* x, const double* b, int iterations) {
  for (int it = 0; it < iterations; ++it) {
    for (int64_t i = 0; i < n; ++i) {
      double rsum = 0.0, diag = 0.0;
      for (int32_t k = ip[i]; k < ip[i + 1]; ++k) {
        const int32_t j = ij[k];
        if (j == i) diag = ax[k];
        else rsum += ax[k] * x[j];
      }
      if (diag != 0.0) x[i] = (b[i] - rsum) / diag;
    }
  }
}

/* pyamg relaxation.gauss_seidel(A, x, b, iterations, sweep): amg_core gauss_seidel over rows
 * [row_start, row_stop) with row_step, the forward arithmetic above (a zero or missing diagonal
 * leaves x_i alone); sweep 0 forward, 1 backward (n-1 .. 0), 2 symmetric (forward then backward,
 * per iteration). */
static void gs_once(int64_t n, const int32_t* ip, const int32_t* ij, const double* ax, double* x,
                    const double* b, int backward) {
  for (int64_t t = 0; t < n; ++t) {
    const int64_t i = backward ? n - 1 - t : t;
    double rsum = 0.0, diag = 0.0;
    for (int32_t k = ip[i]; k < ip[i + 1]; ++k) {
      const int32_t j = ij[k];
      if (j == i) diag = ax[k];
      else rsum += ax[k] * x[j];
    }
    if (diag != 0.0) x[i] = (b[i] - rsum) / diag;
  }
}

void pyamg_gauss_seidel(int64_t n, const int32_t* ip, const int32_t* ij, const double* ax,
                        double* x, const double* b, int iterations, int sweep) {
  for (int it = 0; it < iterations; ++it) {
    if (sweep == 0 || sweep == 2) gs_once(n, ip, ij, ax, x, b, 0);
    if (sweep == 1 || sweep == 2) gs_once(n, ip, ij, ax, x, b, 1);
  }
}

/* graph.py:28-53. dist fp32 [n], nearest int64 [n]; returns number of sweeps */
int ref_bellman_ford_torch(int64_t n, const int32_t* ip, const int32_t* ij, const float* w,
                           const int64_t* centers, int64_t k, float* dist, int64_t* nearest) {
  for (int64_t i = 0; i < n; ++i) {
    dist[i] = INFINITY;
    nearest[i] = 0;
  }
  for (int64_t t = 0; t < k; ++t) {
    dist[centers[t]] = 0.0f;
    nearest[centers[t]] = centers[t];
  }
  int sweeps = 0;
  for (;;) {
    int finished = 1;
    ++sweeps;
    for (int64_t i = 0; i < n; ++i) {
      for (int32_t e = ip[i]; e < ip[i + 1]; ++e) {
        const int32_t j = ij[e];
        const float cand = dist[i] + w[e];
        if (cand < dist[j]) {
          dist[j] = cand;
          nearest[j] = nearest[i];
          finished = 0;
        }
      }
    }
    if (finished) break;
  }
  return sweeps;
}

/* device rule: same fixed-point distances; label = min seed node id over tight in-edges */
void canon_bellman_ford(int64_t n, const int32_t* ip, const int32_t* ij, const float* w,
                        const int32_t* seeds, int64_t k, float* dist, int32_t* label) {
  char* is_seed = (char*)calloc((size_t)n + 1, 1);
  for (int64_t i = 0; i < n; ++i) {
    dist[i] = INFINITY;
    label[i] = INT32_MAX;
  }
  for (int64_t t = 0; t < k; ++t) {
    dist[seeds[t]] = 0.0f;
    label[seeds[t]] = seeds[t];
    is_seed[seeds[t]] = 1;
  }
  int changed = 1;
  while (changed) {
    changed = 0;
    for (int64_t i = 0; i < n; ++i)
      for (int32_t e = ip[i]; e < ip[i + 1]; ++e) {
        const float cand = dist[i] + w[e];
        if (cand < dist[ij[e]]) {
          dist[ij[e]] = cand;
          changed = 1;
        }
      }
  }
  changed = 1;
  while (changed) {
    changed = 0;
    for (int64_t i = 0; i < n; ++i) {
      if (!(dist[i] < INFINITY) || label[i] == INT32_MAX) continue;
      for (int32_t e = ip[i]; e < ip[i + 1]; ++e) {
        const int32_t j = ij[e];
        if (is_seed[j]) continue;
        if (dist[i] + w[e] == dist[j] && label[i] < label[j]) {
          label[j] = label[i];
          changed = 1;
        }
      }
    }
  }
  for (int64_t i = 0; i < n; ++i)
    if (label[i] == INT32_MAX) label[i] = -1;
  free(is_seed);
}

/* pyamg amg_core bellman_ford (pull, in place); returns nonzero if anything changed */
static int pyamg_bf(int64_t n, const int32_t* ip, const int32_t* ij, const double* ax, double* x,
                    int32_t* z, int update_z) {
  int changed = 0;
  for (int64_t i = 0; i < n; ++i) {
    double xi = x[i];
    int32_t zi = z[i];
    for (int32_t jj = ip[i]; jj < ip[i + 1]; ++jj) {
      const int32_t j = ij[jj];
      const double d = ax[jj] + x[j];
      if (d < xi) {
        xi = d;
        zi = z[j];
      }
    }
    if (xi != x[i]) changed = 1;
    x[i] = xi;
    if (update_z) z[i] = zi;
  }
  return changed;
}

static void lloyd_boundary(int64_t n, const int32_t* ip, const int32_t* ij, const int32_t* c,
                           double* d) {
  for (int64_t i = 0; i < n; ++i) d[i] = DBL_MAX;
  for (int64_t i = 0; i < n; ++i)
    for (int32_t jj = ip[i]; jj < ip[i + 1]; ++jj)
      if (c[i] != c[ij[jj]]) {
        d[i] = 0.0;
        break;
      }
}

static void lloyd_recentre(int64_t n, const int32_t* c, const double* d, int32_t* s) {
  for (int64_t i = 0; i < n; ++i) {
    const int32_t seed = c[i];
    if (seed == -1) continue;
    if (d[s[seed]] < d[i]) s[seed] = (int32_t)i;
  }
}

/* one amg_core lloyd_cluster call; canon != 0 uses the order-independent label rule */
static void lloyd_once(int64_t n, const int32_t* ip, const int32_t* ij, const double* ax,
                       int32_t k, double* d, int32_t* c, int32_t* s, int canon, char* is_seed) {
  for (int64_t i = 0; i < n; ++i) {
    d[i] = DBL_MAX;
    c[i] = -1;
  }
  for (int32_t t = 0; t < k; ++t) {
    d[s[t]] = 0.0;
    c[s[t]] = t;
  }
  if (!canon) {
    while (pyamg_bf(n, ip, ij, ax, d, c, 1)) {
    }
  } else {
    memset(is_seed, 0, (size_t)n);
    for (int32_t t = 0; t < k; ++t) is_seed[s[t]] = 1;
    while (pyamg_bf(n, ip, ij, ax, d, c, 0)) {
    }
    int changed = 1;
    while (changed) {
      changed = 0;
      for (int64_t i = 0; i < n; ++i) {
        if (is_seed[i] || !(d[i] < DBL_MAX)) continue;
        int32_t best = c[i];
        for (int32_t jj = ip[i]; jj < ip[i + 1]; ++jj) {
          const int32_t j = ij[jj];
          if (ax[jj] + d[j] == d[i] && c[j] >= 0 && (best < 0 || c[j] < best)) best = c[j];
        }
        if (best != c[i]) {
          c[i] = best;
          changed = 1;
        }
      }
    }
  }
  lloyd_boundary(n, ip, ij, c, d);
  while (pyamg_bf(n, ip, ij, ax, d, c, canon ? 0 : 1)) {
  }
  lloyd_recentre(n, c, d, s);
}

/* pyamg.graph.lloyd_cluster driver: up to maxiter calls, stop when seeds do not move.
 * seeds updated in place; returns iterations run */
int lloyd_cluster(int64_t n, const int32_t* ip, const int32_t* ij, const double* ax, int32_t k,
                  int32_t* seeds, int maxiter, double* d, int32_t* c, int canon) {
  int32_t* last = (int32_t*)malloc(sizeof(int32_t) * (size_t)(k > 0 ? k : 1));
  char* is_seed = (char*)malloc((size_t)n + 1);
  int it = 0;
  for (; it < maxiter;) {
    memcpy(last, seeds, sizeof(int32_t) * (size_t)k);
    lloyd_once(n, ip, ij, ax, k, d, c, seeds, canon, is_seed);
    ++it;
    if (memcmp(last, seeds, sizeof(int32_t) * (size_t)k) == 0) break;
  }
  free(last);
  free(is_seed);
  return it;
}

/* pyamg 4.x pyamg.graph.bellman_ford(G, seeds) with its amg_core.bellman_ford kernel, for a
 * float32 G (ns/model/agg_interp.py:469-475 builds G from the CNet's float32 edge weights, so
 * amg_core runs its <int, float> instantiation: every sum rounds to float). distances start at
 * FLT_MAX (max_value(float32)), 0 at the seeds; nearest_seed starts at -1, seeds[s] at seeds;
 * each sweep visits rows 0..n-1 in order and, in place, takes the first strictly smaller
 * w_ij + d_j over the row's stored entries (and the nearest seed of that j); sweeps repeat
 * until a sweep leaves every distance unchanged. Returns the number of sweeps (>= 1). */
/* in the graph's dtype: float (the CNet weights as pyamg 4.x receives them) or double (a
 * pyamg build that binds only double would widen them first) */
#define PYAMG_BF(NAME, T, TMAX)                                                                \
  int NAME(int64_t n, const int32_t* ip, const int32_t* ij, const T* w, const int32_t* seeds,  \
           int64_t k, T* dist, int32_t* nearest) {                                             \
    for (int64_t i = 0; i < n; ++i) {                                                          \
      dist[i] = TMAX;                                                                          \
      nearest[i] = -1;                                                                         \
    }                                                                                          \
    for (int64_t s = 0; s < k; ++s) {                                                          \
      dist[seeds[s]] = 0;                                                                      \
      nearest[seeds[s]] = seeds[s];                                                            \
    }                                                                                          \
    int sweeps = 0, changed = 1;                                                               \
    while (changed) {                                                                          \
      changed = 0;                                                                             \
      for (int64_t i = 0; i < n; ++i) {                                                        \
        T xi = dist[i];                                                                        \
        int32_t zi = nearest[i];                                                               \
        for (int32_t jj = ip[i]; jj < ip[i + 1]; ++jj) {                                       \
          const int32_t j = ij[jj];                                                            \
          const T d = w[jj] + dist[j];                                                         \
          if (d < xi) {                                                                        \
            xi = d;                                                                            \
            zi = nearest[j];                                                                   \
          }                                                                                    \
        }                                                                                      \
        if (xi != dist[i]) changed = 1;                                                        \
        dist[i] = xi;                                                                          \
        nearest[i] = zi;                                                                       \
      }                                                                                        \
      ++sweeps;                                                                                \
    }                                                                                          \
    return sweeps;                                                                             \
  }
PYAMG_BF(pyamg_bellman_ford, float, FLT_MAX)
PYAMG_BF(pyamg_bellman_ford_f64, double, DBL_MAX)

/* ---------------------------------------------------------------- pyamg smoothed aggregation */
/* amg_core symmetric_strength_of_connection + pyamg's |.| and scale_rows_by_largest_entry.
 * sp (n+1), sj/sx (capacity nnz); returns nnz kept. */
int64_t pyamg_symmetric_strength(int64_t n, const int32_t* ip, const int32_t* ij,
                                 const double* ax, double theta, int32_t* sp, int32_t* sj,
                                 double* sx) {
  double* dg = (double*)malloc(sizeof(double) * (n ? n : 1));
  for (int64_t i = 0; i < n; ++i) {
    double d = 0.0;
    for (int32_t k = ip[i]; k < ip[i + 1]; ++k)
      if (ij[k] == i) d += ax[k];
    dg[i] = fabs(d);
  }
  int64_t nnz = 0;
  sp[0] = 0;
  for (int64_t i = 0; i < n; ++i) {
    const double eps = theta * theta * dg[i];
    for (int32_t k = ip[i]; k < ip[i + 1]; ++k) {
      const int32_t j = ij[k];
      const double a = ax[k];
      if (j == i || a * a >= eps * dg[j]) {
        sj[nnz] = j;
        sx[nnz] = a;
        ++nnz;
      }
    }
    sp[i + 1] = (int32_t)nnz;
  }
  for (int64_t i = 0; i < n; ++i) {
    double mx = 0.0;
    for (int32_t k = sp[i]; k < sp[i + 1]; ++k) mx = fmax(mx, fabs(sx[k]));
    const double inv = mx != 0.0 ? 1.0 / mx : 0.0;
    for (int32_t k = sp[i]; k < sp[i + 1]; ++k) sx[k] = fabs(sx[k]) * inv;
  }
  free(dg);
  return nnz;
}

/* amg_core standard_aggregation, literally: x[n] aggregate (-1 none), y[n] Cpts; returns the
 * number of aggregates */
int64_t pyamg_standard_aggregation(int64_t n, const int32_t* ip, const int32_t* ij, int32_t* x,
                                   int32_t* y) {
  for (int64_t i = 0; i < n; ++i) x[i] = 0;
  int32_t next = 1;
  for (int64_t i = 0; i < n; ++i) { /* pass 1 */
    if (x[i]) continue;
    int has_agg = 0, has_nb = 0;
    for (int32_t k = ip[i]; k < ip[i + 1]; ++k) {
      const int32_t j = ij[k];
      if (j != i) {
        has_nb = 1;
        if (x[j]) {
          has_agg = 1;
          break;
        }
      }
    }
    if (!has_nb) {
      x[i] = -(int32_t)n;
    } else if (!has_agg) {
      x[i] = next;
      y[next - 1] = (int32_t)i;
      for (int32_t k = ip[i]; k < ip[i + 1]; ++k) x[ij[k]] = next;
      ++next;
    }
  }
  for (int64_t i = 0; i < n; ++i) { /* pass 2 */
    if (x[i]) continue;
    for (int32_t k = ip[i]; k < ip[i + 1]; ++k) {
      const int32_t xj = x[ij[k]];
      if (xj > 0) {
        x[i] = -xj;
        break;
      }
    }
  }
  --next;
  for (int64_t i = 0; i < n; ++i) { /* pass 3 */
    const int32_t xi = x[i];
    if (xi != 0) {
      if (xi > 0) x[i] = xi - 1;
      else if (xi == -(int32_t)n) x[i] = -1;
      else x[i] = -xi - 1;
      continue;
    }
    x[i] = next;
    y[next] = (int32_t)i;
    for (int32_t k = ip[i]; k < ip[i + 1]; ++k)
      if (x[ij[k]] == 0) x[ij[k]] = next;
    ++next;
  }
  return next;
}

/* pyamg relaxation.block_gauss_seidel with blocksize 1 (amg_core block_gauss_seidel; Dinv from
 * get_block_diag + pinv_array: 1 / a_ii, 0 for a zero or missing diagonal). sweep 0 forward,
 * 1 backward, 2 symmetric (forward then backward, per iteration). */
static void bgs_once(int64_t n, const int32_t* ip, const int32_t* ij, const double* ax,
                     const double* dinv, double* x, const double* b, int backward) {
  for (int64_t t = 0; t < n; ++t) {
    const int64_t i = backward ? n - 1 - t : t;
    double rsum = b[i];
    for (int32_t k = ip[i]; k < ip[i + 1]; ++k) {
      const int32_t j = ij[k];
      if (j == i) continue;
      const double axl = 0.0 + ax[k] * x[j];
      rsum -= axl;
    }
    x[i] = 0.0 + dinv[i] * rsum;
  }
}

void pyamg_block_gauss_seidel(int64_t n, const int32_t* ip, const int32_t* ij, const double* ax,
                              double* x, const double* b, int iterations, int sweep) {
  double* dinv = (double*)malloc(sizeof(double) * (n ? n : 1));
  for (int64_t i = 0; i < n; ++i) {
    double d = 0.0;
    for (int32_t k = ip[i]; k < ip[i + 1]; ++k)
      if (ij[k] == i) d = ax[k]; /* the stored diagonal (the last one, as the sweeps read it) */
    dinv[i] = d != 0.0 ? 1.0 / d : 0.0;
  }
  for (int it = 0; it < iterations; ++it) {
    if (sweep == 0 || sweep == 2) bgs_once(n, ip, ij, ax, dinv, x, b, 0);
    if (sweep == 1 || sweep == 2) bgs_once(n, ip, ij, ax, dinv, x, b, 1);
  }
  free(dinv);
}

/* fit_candidates_common with K1 = K2 = 1: agg[n] (-1 none), k aggregates; T values (per row
 * with an aggregate, row order) into tx, Bc[k] */
void pyamg_fit_candidates(int64_t n, const int32_t* agg, int64_t k, const double* B, double tol,
                          double* tx, double* Bc) {
  double* s = (double*)calloc(k ? k : 1, sizeof(double));
  double* scale = (double*)malloc(sizeof(double) * (k ? k : 1));
  for (int64_t i = 0; i < n; ++i) /* AggOp.tocsc(): every column's rows ascending */
    if (agg[i] >= 0) s[agg[i]] += B[i] * B[i];
  for (int64_t j = 0; j < k; ++j) {
    const double nrm = sqrt(s[j]);
    const double thr = tol * nrm;
    scale[j] = nrm > thr ? 1.0 / nrm : 0.0;
    Bc[j] = nrm > thr ? nrm : 0.0;
  }
  int64_t o = 0;
  for (int64_t i = 0; i < n; ++i)
    if (agg[i] >= 0) tx[o++] = B[i] * scale[agg[i]];
  free(s);
  free(scale);
}
