/* check_div.c -- render.hip's div_by (Markstein's one-FMA correction from a correctly rounded
 * reciprocal) against IEEE x / d on random operand pairs in div_by's guarded range; prints the
 * number of differing results (must be 0). gcc -O2 -ffp-contract=off tools/check_div.c -lm */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t st = 88172645463325252ull;
static uint64_t xs(void) {
    st ^= st << 13;
    st ^= st >> 7;
    st ^= st << 17;
    return st;
}
static float fu(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t uf(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

int main(int argc, char **argv) {
    long n = argc > 1 ? atol(argv[1]) : 100000000L, bad = 0, used = 0;
    for (long i = 0; i < n; ++i) {
        uint64_t z = xs();
        uint32_t ex = 127 - 100 + (uint32_t)((z >> 40) % 201), ed = 127 - 60 + (uint32_t)((z >> 50) % 121);
        uint32_t mx = (uint32_t)z & 0x7fffff, md = (uint32_t)(z >> 23) & 0x7fffff;
        if ((i & 7) == 0) md = 0x7fffff - (uint32_t)(z % 8);  /* significands near all ones */
        if ((i & 7) == 1) md = (uint32_t)(z % 8);             /* and near powers of two */
        float x = fu((ex << 23) | mx), d = fu((ed << 23) | md);
        float inv = 1.0f / d, q = x * inv, r = fmaf(-d, q, x), q1 = fmaf(r, inv, q);
        float ax = fabsf(x), aq = fabsf(q1);
        if (!(ax >= 0x1p-100f && ax <= 0x1p100f && aq >= 0x1p-100f && aq <= 0x1p100f)) continue;
        ++used;
        if (uf(q1) != uf(x / d)) {
            if (++bad < 10) printf("x=%a d=%a x/d=%a got=%a\n", x, d, x / d, q1);
        }
    }
    printf("pairs %ld in range %ld differing %ld\n", n, used, bad);
    return bad != 0;
}
