// Checks the walk kernel's division by a loop-invariant c (grf_philox.h div_by: q = x RN(1/c), then one FMA
// correction) against x / c on 320 M random normal x over 16 divisors (1 - p_halt values and walk counts m).
// build: gcc -O2 -o /tmp/div_check tools/div_check.c -lm   (prints "mismatches 0 of 320000000")
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
static uint64_t st = 88172645463325252ull;
static inline uint64_t xr(void) { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; }
int main(void) {
    double cs[] = {0.9, 0.7, 0.95, 0.8, 0.85, 1.0, 0.5, 0.99, 0.75, 0.6, 7.0, 33.0, 128.0, 64.0, 3.0, 0.9 + 1e-9};
    long bad = 0, tot = 0;
    for (int ci = 0; ci < (int)(sizeof cs / sizeof *cs); ++ci) {
        const double c = cs[ci], y = 1.0 / c;
        for (long i = 0; i < 20000000; ++i) {
            uint64_t b = xr();
            // random normal doubles across exponents 2^-60 .. 2^60, random mantissa
            uint64_t e = 1023 - 60 + (b >> 58) * 2;  // exponents
            uint64_t bits = (e << 52) | (xr() & ((1ull << 52) - 1));
            double x; memcpy(&x, &bits, 8);
            const double q = x * y;
            const double r = fma(fma(-q, c, x), y, q);
            ++tot;
            if (r != x / c) { ++bad; if (bad < 5) printf("c=%.17g x=%.17g %.17g vs %.17g\n", c, x, r, x / c); }
        }
    }
    printf("mismatches %ld of %ld\n", bad, tot);
    return 0;
}
