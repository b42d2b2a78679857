/* Exhaustive check of the division identity quantize_fused_kernel relies on
 * (diffusion-llm-rs_amd/csrc/quant_kernels.hip, div_scale): with r = RN(1/s), q0 = RN(x r),
 * e = fma(-q0, s, x), q1 = fma(e, r, q0), q1 == RN(x / s) (Rust's `x / scale`, quantization.rs:61).
 * Both are scale-invariant in the normal range, so x runs over every significand of two
 * binades ([1, 4): the quotient's significand depends on whether x's significand is below s's)
 * and s over `nb` significands in [1, 2): the all-ones and all-zeros ones plus a seeded sample.
 * Usage: markstein_check NB SEED -> prints "checked N mismatches M". IEEE f32, no contraction. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static float f_of(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t u_of(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

int main(int argc, char **argv) {
    const int nb = argc > 1 ? atoi(argv[1]) : 64;
    uint64_t state = argc > 2 ? strtoull(argv[2], 0, 10) : 1;
    long long bad = 0, total = 0;
    for (int j = 0; j < nb; ++j) {
        uint32_t ms;
        if (j == 0) ms = 0x7fffff;
        else if (j == 1) ms = 0;
        else { state = state * 6364136223846793005ull + 1442695040888963407ull; ms = (uint32_t)(state >> 41) & 0x7fffff; }
        volatile float s = f_of((127u << 23) | ms), one = 1.0f;
        const float r = one / s;
        long long bad_j = 0;
#pragma omp parallel for reduction(+ : bad_j)
        for (uint32_t mx = 0; mx < (1u << 24); ++mx) {
            const float x = f_of(((126u + 1u + (mx >> 23)) << 23) | (mx & 0x7fffff));
            const float q = x / s;
            const float q0 = x * r;
            const float e = fmaf(-q0, s, x);
            const float q1 = fmaf(e, r, q0);
            bad_j += u_of(q1) != u_of(q);
        }
        bad += bad_j;
        total += 1ll << 24;
    }
    printf("checked %lld mismatches %lld\n", total, bad);
    return bad != 0;
}
