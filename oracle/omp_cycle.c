/* TEST / BASELINE INFRASTRUCTURE ONLY — a multi-threaded (OpenMP) CPU restatement of the
 * weighted-Jacobi V-cycle kernels, used by bench.py's parallel CPU baseline leg (the bench's
 * `cpu_baseline` stays the 1-thread scipy port, the reference's own execution model).
 *
 * Rows are split across threads; each row is summed left to right in stored order with
 * separate multiply and add roundings (scipy sparsetools csr_matvec order, -ffp-contract=off),
 * so every vector except the norm is bitwise the sequential restatement's.
 *   omp_resid      r = b - A x                         (ns/lib/multigrid.py:181, MLAMG.py:191)
 *   omp_jacobi     x' = x + d * (b - A x)              (MLAMG.py:143-146, d = w / diag)
 *   omp_matvec     y = A x                             (restriction with R = P^T as CSR)
 *   omp_add_matvec x += A e                            (prolongation, MLAMG.py:191)
 *   omp_gemv       x = M b, M dense row-major          (coarse solve by the explicit inverse)
 *   omp_norm2      ||r||_2
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>

void omp_set_threads(int n) { omp_set_num_threads(n); }

static inline double row_sum(const int32_t* ip, const int32_t* ij, const double* ax,
                             const double* x, int64_t i) {
  double s = 0.0;
  for (int32_t k = ip[i]; k < ip[i + 1]; ++k) s += ax[k] * x[ij[k]];
  return s;
}

void omp_resid(int64_t n, const int32_t* ip, const int32_t* ij, const double* ax, const double* b,
               const double* x, double* r) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) r[i] = b[i] - row_sum(ip, ij, ax, x, i);
}

void omp_jacobi(int64_t n, const int32_t* ip, const int32_t* ij, const double* ax,
                const double* d, const double* b, const double* x, double* xout) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    const double r = b[i] - row_sum(ip, ij, ax, x, i);
    xout[i] = x[i] + d[i] * r;
  }
}

void omp_scale(int64_t n, const double* d, const double* b, double* x) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) x[i] = d[i] * b[i];  // zero-guess sweep: 0 + d*(b - 0)
}

void omp_matvec(int64_t n, const int32_t* ip, const int32_t* ij, const double* ax,
                const double* x, double* y) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) y[i] = row_sum(ip, ij, ax, x, i);
}

void omp_add_matvec(int64_t n, const int32_t* ip, const int32_t* ij, const double* ax,
                    const double* e, double* x) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) x[i] = x[i] + row_sum(ip, ij, ax, e, i);
}

void omp_gemv(int64_t n, const double* M, const double* b, double* x) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    double s = 0.0;
    const double* r = M + i * n;
    for (int64_t j = 0; j < n; ++j) s += r[j] * b[j];
    x[i] = s;
  }
}

double omp_norm2(int64_t n, const double* r) {
  double s = 0.0;
#pragma omp parallel for schedule(static) reduction(+ : s)
  for (int64_t i = 0; i < n; ++i) s += r[i] * r[i];
  return sqrt(s);
}
