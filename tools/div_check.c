/* div_check -- CPU check of the search loop's division by a pre-computed
 * reciprocal (dis_search8.hip div_pre) against IEEE single division:
 * q0 = a*r, q1 = fma(fma(-b,q0,a),r,q0), q2 = fma(fma(-b,q1,a),r,q1),
 * r = RN(1/b), then q0's sign bit on q2's magnitude (the kernels' form since
 * r04; the same bits as "a = +-0 keeps q0"). Random a, b with exponents in [-60, 60]
 * (the patch sums and LU pivots of 8-bit images) and mantissas biased to the
 * edge cases (all ones, zero). Usage: div_check [samples]; exit 1 on a
 * mismatch. A second pass checks the output kernel's densify divisors
 * b = n / 2 (n = 1..16 covering patches) against numerators of exponent
 * [-100, 60] (k_output sends |a| < 2^-100 to IEEE division). Build: gcc -O2 -mfma -ffp-contract=off div_check.c -lm */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static float bf(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t fb(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static uint64_t s = 88172645463325252ull;
static uint64_t rnd(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }

static float div_pre(float a, float b, float r)
{
    const float q0 = a * r;
    const float q1 = fmaf(fmaf(-b, q0, a), r, q0);
    const float q2 = fmaf(fmaf(-b, q1, a), r, q1);
    return bf((fb(q0) & 0x80000000u) | (fb(q2) & 0x7fffffffu));
}

int main(int argc, char** argv)
{
    const long n = argc > 1 ? atol(argv[1]) : 400000000L;
    long bad = 0;
    for (long i = 0; i < n; i++) {
        const uint64_t x = rnd();
        const uint32_t ea = (uint32_t)(67 + (x % 121)), eb = (uint32_t)(67 + ((x >> 8) % 121));
        uint32_t ma = (uint32_t)(x >> 16) & 0x7fffff, mb = (uint32_t)(x >> 40) & 0x7fffff;
        if ((x >> 63) & 1) mb = (i & 1) ? 0x7fffff : ((i & 2) ? 0 : mb);
        if ((x >> 62) & 1) ma = (i & 4) ? 0x7fffff : ma;
        float a = bf(((uint32_t)(x >> 39 & 1) << 31) | ea << 23 | ma);
        const float b = bf(((uint32_t)(x >> 38 & 1) << 31) | eb << 23 | mb);
        if ((i & 1023) == 5) a = (i & 2048) ? -0.0f : 0.0f;
        volatile float bv = b, av = a;
        const float r = 1.0f / bv, ref = av / bv, got = div_pre(a, b, r);
        if (fb(got) != fb(ref)) {
            if (bad < 10) printf("a=%a b=%a ref=%a got=%a\n", a, b, ref, got);
            bad++;
        }
    }
    for (long i = 0; i < n / 4; i++) {  /* densify weights */
        const uint64_t x = rnd();
        const int nc = 1 + (int)(x % 16);
        const uint32_t ea = (uint32_t)(27 + ((x >> 8) % 161));
        uint32_t ma = (uint32_t)(x >> 16) & 0x7fffff;
        if ((x >> 62) & 1) ma = (i & 4) ? 0x7fffff : ma;
        const float a = bf(((uint32_t)(x >> 39 & 1) << 31) | ea << 23 | ma);
        volatile float bv = 0.5f * (float)nc, av = a;
        const float r = 1.0f / bv, ref = av / bv, got = div_pre(a, bv, r);
        if (fb(got) != fb(ref)) {
            if (bad < 10) printf("a=%a b=%a ref=%a got=%a\n", a, (float)bv, ref, got);
            bad++;
        }
    }
    printf("div_check: %ld + %ld samples, %ld mismatches\n", n, n / 4, bad);
    return bad != 0;
}
