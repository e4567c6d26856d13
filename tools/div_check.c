// Checks the walk kernel's division by a loop-invariant c (grf_philox.h Divisor: q = x RN(1/c), one FMA
// correction, and the IEEE divide outside the exponent window where |x|, |x / c| lie in [2^-959, 2^961)) against x / c:
//   1. 380 M random normal x across exponents 2^-60 .. 2^60 over 19 divisors (1 - p_halt values down to 2^-40, walk counts m);
//   2. the edges: zeros, subnormals, the smallest normals, values near the overflow threshold, inf and NaN
//      (the cumulative-load overflow case of ADVICE r04: fma(-inf, c, inf) alone would give NaN).
// build: gcc -O2 -o /tmp/div_check tools/div_check.c -lm   (prints "mismatches 0 of ..." twice)
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
static uint64_t st = 88172645463325252ull;
static inline uint64_t xr(void) { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; }

typedef struct { double c, y; uint32_t lo, span; } divisor;  // grf_philox.h Divisor, restated
static uint32_t hiword(double x) { uint64_t b; memcpy(&b, &x, 8); return (uint32_t)(b >> 32); }
static divisor make_divisor(double c) {
    divisor d = {c, 1.0 / c, 0, 0};
    const int32_t ec = (int32_t)((hiword(c) >> 20) & 0x7ff);
    const int32_t l = ec - 958 > 64 ? ec - 958 : 64, h = ec + 959 < 1983 ? ec + 959 : 1983;
    d.lo = (uint32_t)l;
    d.span = h >= l ? (uint32_t)(h - l) : 0u;
    if (h < l) d.lo = 0xffffffffu;
    return d;
}
static double div_by(double x, const divisor *d) {
    const uint32_t ex = (hiword(x) >> 20) & 0x7ffu;
    if (ex - d->lo > d->span) return x / d->c;
    const double q = x * d->y;
    return fma(fma(-q, d->c, x), d->y, q);
}

static int same(double a, double b) { return (isnan(a) && isnan(b)) || memcmp(&a, &b, 8) == 0; }

int main(void) {
    double cs[] = {0.9, 0.7, 0.95, 0.8, 0.85, 1.0, 0.5, 0.99, 0.75, 0.6, 7.0, 33.0, 128.0, 64.0, 3.0, 0.9 + 1e-9,
                  1e-3, 0x1p-40, 16384.0};
    const int nc = (int)(sizeof cs / sizeof *cs);
    long bad = 0, tot = 0;
    for (int ci = 0; ci < nc; ++ci) {
        const double c = cs[ci];
        const divisor dv = make_divisor(c);
        for (long i = 0; i < 20000000; ++i) {
            uint64_t b = xr();
            uint64_t e = 1023 - 60 + (b >> 58) * 2;  // exponents
            uint64_t bits = (e << 52) | (xr() & ((1ull << 52) - 1));
            double x;
            memcpy(&x, &bits, 8);
            ++tot;
            if (!same(div_by(x, &dv), x / c)) {
                ++bad;
                if (bad < 5) printf("c=%.17g x=%.17g %.17g vs %.17g\n", c, x, div_by(x, &dv), x / c);
            }
        }
    }
    printf("mismatches %ld of %ld (random normal operands)\n", bad, tot);
    double edges[] = {0.0, -0.0, 0x1p-1074, -0x1p-1074, 0x1p-1060, 0x1p-1022, 0x1.8p-1022, 0x1p-1000, 0x1p-961,
                      0x1p-960, 0x1p960, 0x1p1000, 0x1.fffffffffffffp1023, -0x1.fffffffffffffp1023, INFINITY,
                      -INFINITY, NAN};
    long bad2 = 0, tot2 = 0;
    for (int ci = 0; ci < nc; ++ci) {
        const double c = cs[ci];
        const divisor dv = make_divisor(c);
        for (int k = 0; k < (int)(sizeof edges / sizeof *edges); ++k) {
            for (int d = -40; d <= 40; ++d) {  // the edge and its neighbours
                double x = edges[k];
                for (int s = 0; s < (d < 0 ? -d : d) && isfinite(x); ++s) x = nextafter(x, d < 0 ? -INFINITY : INFINITY);
                ++tot2;
                if (!same(div_by(x, &dv), x / c)) {
                    ++bad2;
                    if (bad2 < 5) printf("edge c=%.17g x=%a %a vs %a\n", c, x, div_by(x, &dv), x / c);
                }
            }
        }
    }
    printf("mismatches %ld of %ld (edges: zero, subnormal, huge, inf, NaN)\n", bad2, tot2);
    return 0;
}
