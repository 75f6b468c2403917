/* TEST INFRASTRUCTURE ONLY (tests/test_markstein.py). The division the device's Gauss-Seidel
 * chains use (csrc/common.hpp mk_recip / mk_div: Markstein's correction of a * RN(1/b), with the
 * same range guards) against the IEEE division, bit for bit, on random operand pairs of several
 * exponent spreads, integer-valued pairs and the special values. Exit status = mismatches != 0.
 *   gcc -O2 -ffp-contract=off oracle/markstein_check.c -lm -o /tmp/mk && /tmp/mk 10000000 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t st = 88172645463325252ull;
static uint64_t rnd(void) {
  st ^= st << 13;
  st ^= st >> 7;
  st ^= st << 17;
  return st;
}
static double rd(int emin, int emax) {
  uint64_t m = rnd() & ((1ull << 52) - 1);
  int e = emin + (int)(rnd() % (uint64_t)(emax - emin + 1));
  uint64_t bits = ((uint64_t)(e + 1023) << 52) | m;
  if (rnd() & 1) bits |= 1ull << 63;
  double d;
  memcpy(&d, &bits, 8);
  return d;
}
static double mk_recip(double b) {
  const double ab = fabs(b);
  return (ab >= 0x1p-1000 && ab <= 0x1p1000) ? 1.0 / b : NAN;
}
static double mk_div(double a, double b, double y) {
  const double q = a * y;
  const double r = fma(-b, q, a);
  const double aq = fabs(q), aa = fabs(a);
  if (aq >= 0x1p-960 && aq <= 0x1p960 && aa >= 0x1p-960 && aa <= 0x1p960) return fma(r, y, q);
  return a / b;
}
static long check(double a, double b) {
  const double q1 = a / b, q2 = mk_div(a, b, mk_recip(b));
  uint64_t u1, u2;
  memcpy(&u1, &q1, 8);
  memcpy(&u2, &q2, 8);
  if (u1 == u2 || (isnan(q1) && isnan(q2))) return 0;
  printf("mismatch a=%a b=%a ieee=%a mk=%a\n", a, b, q1, q2);
  return 1;
}
int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 10000000L;
  long bad = 0;
  for (long i = 0; i < n && bad < 10; ++i) {
    switch (i % 5) {
      case 0: bad += check(rd(-30, 30), rd(-30, 30)); break;
      case 1: bad += check(rd(-4, 4), rd(-4, 4)); break;
      case 2: {
        double b = (double)((int64_t)(rnd() % 2001) - 1000);
        bad += check((double)((int64_t)(rnd() % 2000001) - 1000000), b == 0 ? 3.0 : b);
        break;
      }
      case 3: bad += check(rd(-1000, 1000), rd(-1010, 1010)); break;
      default: bad += check(rd(-1022, 1023), rd(-1022, 1023)); break;
    }
  }
  const double sp[] = {0.0, -0.0, 1.0, -1.0, 3.0, 0x1p-1022, 0x1.fffffffffffffp+1023, 0x1p-1074,
                       INFINITY, -INFINITY, NAN, 1e-300, 1e300, 0x1p-960, 0x1p960, 0x1p1000,
                       0x1p-1000, 0x1.fffffffffffffp-1, 0x1.0000000000001p+0};
  const int ns = (int)(sizeof(sp) / sizeof(sp[0]));
  for (int i = 0; i < ns; ++i)
    for (int j = 0; j < ns; ++j)
      if (sp[j] != 0.0) bad += check(sp[i], sp[j]);
  printf("checked %ld random pairs and %d specials: %ld mismatches\n", n, ns * ns, bad);
  return bad != 0;
}
