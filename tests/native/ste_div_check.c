/* Host check of the STE division used by the HIP kernels (csrc/dqrm_internal.h, SteDiv):
 * q = RN(x*y), y = RN(1/s); two fma residual corrections; must equal the IEEE x/s bit for
 * bit on the fast range (|x|, s in [2^-60, 2^60]). Random x = g*s over many binades, plus
 * structured significands (all ones, powers of two, near-binade boundaries).
 * build: gcc -O2 -ffp-contract=off ste_div_check.c -lm;  run: ./a.out <n> <seed>
 * prints the number of mismatches (0 expected). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t st = 88172645463325252ull;
static uint64_t xr(void) { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; }
static float bits(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t ubits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

static float ste_fast(float x, float s, float y) {
    float q = x * y;
    float r = fmaf(-s, q, x);
    q = fmaf(r, y, q);
    r = fmaf(-s, q, x);
    return fmaf(r, y, q);
}

static float rand_float(int emin, int emax) {  /* random sign/significand, exponent in range */
    uint32_t e = (uint32_t)(127 + emin + (int)(xr() % (uint64_t)(emax - emin + 1)));
    uint32_t m;
    switch (xr() % 6) {
        case 0: m = 0x7FFFFF; break;                          /* all ones */
        case 1: m = 0; break;                                 /* power of two */
        case 2: m = (uint32_t)(xr() % 16); break;             /* just above a binade */
        case 3: m = 0x7FFFFF - (uint32_t)(xr() % 16); break;  /* just below the next */
        default: m = (uint32_t)(xr() & 0x7FFFFF);
    }
    return bits(((uint32_t)(xr() & 1) << 31) | (e << 23) | m);
}

int main(int argc, char** argv) {
    long n = argc > 1 ? atol(argv[1]) : 10000000;
    st ^= argc > 2 ? (uint64_t)atoll(argv[2]) * 0x9E3779B97F4A7C15ull : 0;
    long bad = 0;
    for (long i = 0; i < n; ++i) {
        const float s = fabsf(rand_float(-60, 60));
        const float y = 1.0f / s;
        /* x as the kernels see it: a product g*s (rounded), or any float in range */
        float x = (i & 1) ? rand_float(-60, 60) : rand_float(-30, 30) * s;
        if (!(fabsf(x) >= 0x1p-60f && fabsf(x) <= 0x1p60f)) continue;
        const float want = x / s, got = ste_fast(x, s, y);
        if (ubits(want) != ubits(got)) {
            if (bad < 5) printf("mismatch x=%a s=%a want=%a got=%a\n", x, s, want, got);
            ++bad;
        }
    }
    printf("%ld\n", bad);
    return 0;
}
