// Checks the walk kernel's division by a loop-invariant c (grf_philox.h div_by: q = x RN(1/c), one FMA
// correction, and the IEEE divide outside [2^-960, 2^960]) against x / c:
//   1. 320 M random normal x across exponents 2^-60 .. 2^60 over 16 divisors (1 - p_halt values, walk counts m);
//   2. the edges: zeros, subnormals, the smallest normals, values near the overflow threshold, inf and NaN
//      (the cumulative-load overflow case of ADVICE r04: fma(-inf, c, inf) alone would give NaN).
// build: gcc -O2 -o /tmp/div_check tools/div_check.c -lm   (prints "mismatches 0 of ..." twice)
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
static uint64_t st = 88172645463325252ull;
static inline uint64_t xr(void) { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; }

static double div_by(double x, double c, double y) {  // grf_philox.h, restated
    const double q = x * y;
    const double r = fma(fma(-q, c, x), y, q);
    const double ax = fabs(x), ar = fabs(r);
    if (!(ax >= 0x1p-960 && ax <= 0x1p960 && ar >= 0x1p-960 && ar <= 0x1p960)) return x / c;
    return r;
}

static int same(double a, double b) { return (isnan(a) && isnan(b)) || memcmp(&a, &b, 8) == 0; }

int main(void) {
    double cs[] = {0.9, 0.7, 0.95, 0.8, 0.85, 1.0, 0.5, 0.99, 0.75, 0.6, 7.0, 33.0, 128.0, 64.0, 3.0, 0.9 + 1e-9};
    const int nc = (int)(sizeof cs / sizeof *cs);
    long bad = 0, tot = 0;
    for (int ci = 0; ci < nc; ++ci) {
        const double c = cs[ci], y = 1.0 / c;
        for (long i = 0; i < 20000000; ++i) {
            uint64_t b = xr();
            uint64_t e = 1023 - 60 + (b >> 58) * 2;  // exponents
            uint64_t bits = (e << 52) | (xr() & ((1ull << 52) - 1));
            double x;
            memcpy(&x, &bits, 8);
            ++tot;
            if (!same(div_by(x, c, y), x / c)) {
                ++bad;
                if (bad < 5) printf("c=%.17g x=%.17g %.17g vs %.17g\n", c, x, div_by(x, c, y), x / c);
            }
        }
    }
    printf("mismatches %ld of %ld (random normal operands)\n", bad, tot);
    double edges[] = {0.0, -0.0, 0x1p-1074, -0x1p-1074, 0x1p-1060, 0x1p-1022, 0x1.8p-1022, 0x1p-1000, 0x1p-961,
                      0x1p-960, 0x1p960, 0x1p1000, 0x1.fffffffffffffp1023, -0x1.fffffffffffffp1023, INFINITY,
                      -INFINITY, NAN};
    long bad2 = 0, tot2 = 0;
    for (int ci = 0; ci < nc; ++ci) {
        const double c = cs[ci], y = 1.0 / c;
        for (int k = 0; k < (int)(sizeof edges / sizeof *edges); ++k) {
            for (int d = -40; d <= 40; ++d) {  // the edge and its neighbours
                double x = edges[k];
                for (int s = 0; s < (d < 0 ? -d : d) && isfinite(x); ++s) x = nextafter(x, d < 0 ? -INFINITY : INFINITY);
                ++tot2;
                if (!same(div_by(x, c, y), x / c)) {
                    ++bad2;
                    if (bad2 < 5) printf("edge c=%.17g x=%a %a vs %a\n", c, x, div_by(x, c, y), x / c);
                }
            }
        }
    }
    printf("mismatches %ld of %ld (edges: zero, subnormal, huge, inf, NaN)\n", bad2, tot2);
    return 0;
}
