/*
 * dllm_sgemm.c -- TEST / BASELINE INFRASTRUCTURE ONLY (never linked by the product).
 *
 * A cache-blocked, packed AVX2/FMA f32 GEMM: the class of kernel the reference's linear layer
 * actually runs.  SimpleDiffusionModel::forward is `x.dot(&self.weights) + &self.bias`
 * (diffuse-llm-rs/src/lib.rs:806-813); ndarray 0.15's Array2::dot calls the `matrixmultiply`
 * crate's sgemm, a BLIS-style GEMM (packed A/B panels, MC/KC/NC cache blocking, an AVX/FMA
 * register-tile micro-kernel selected at run time).  The scalar i-k-j loop in dllm_oracle.c stays
 * the PARITY restatement; this file exists so bench.py's cpu_baseline times a CPU GEMM of the
 * same class as the reference's, instead of a scalar loop an order of magnitude slower.
 *
 * Blocking: NC = N (one B panel per KC slice), KC = 256, MC = 72; micro-tile MR x NR = 6 x 16
 * (12 ymm accumulators, 2 B loads + 6 broadcasts + 12 FMAs per k).  Threads split the MC blocks
 * of each KC slice (OpenMP); the B panel is packed once per slice by all threads.
 */
#include <immintrin.h>
#include <omp.h>
#include <stdlib.h>
#include <string.h>

#define MR 6
#define NR 16
#define KC 256
#define MC 72

/* Bp[j/NR][k][NR]: the KC x N slice starting at row k0, zero-padded to a multiple of NR. */
static void pack_b(const float *B, size_t N, size_t k0, size_t kc, float *Bp, int nthreads) {
    const size_t nsl = (N + NR - 1) / NR;
#pragma omp parallel for num_threads(nthreads) schedule(static)
    for (size_t s = 0; s < nsl; ++s) {
        float *dst = Bp + s * kc * NR;
        const size_t j0 = s * NR, w = (N - j0) < NR ? (N - j0) : NR;
        for (size_t k = 0; k < kc; ++k) {
            const float *src = B + (k0 + k) * N + j0;
            size_t j = 0;
            for (; j < w; ++j) dst[k * NR + j] = src[j];
            for (; j < NR; ++j) dst[k * NR + j] = 0.0f;
        }
    }
}

/* Ap[i/MR][k][MR] of the mc x kc block at (i0, k0), zero-padded to a multiple of MR. */
static void pack_a(const float *A, size_t K, size_t i0, size_t mc, size_t k0, size_t kc, float *Ap) {
    for (size_t s = 0; s < (mc + MR - 1) / MR; ++s) {
        float *dst = Ap + s * kc * MR;
        const size_t r0 = i0 + s * MR, h = (mc - s * MR) < MR ? (mc - s * MR) : MR;
        for (size_t k = 0; k < kc; ++k) {
            size_t r = 0;
            for (; r < h; ++r) dst[k * MR + r] = A[(r0 + r) * K + k0 + k];
            for (; r < MR; ++r) dst[k * MR + r] = 0.0f;
        }
    }
}

/* C[6][16] (+)= Ap-sliver . Bp-sliver over kc; partial tiles go through a local buffer. */
__attribute__((target("avx2,fma")))
static void micro_6x16(size_t kc, const float *a, const float *b, float *C, size_t ldc, size_t h, size_t w,
                       int accumulate) {
    __m256 c00 = _mm256_setzero_ps(), c01 = _mm256_setzero_ps(), c10 = _mm256_setzero_ps(),
           c11 = _mm256_setzero_ps(), c20 = _mm256_setzero_ps(), c21 = _mm256_setzero_ps(),
           c30 = _mm256_setzero_ps(), c31 = _mm256_setzero_ps(), c40 = _mm256_setzero_ps(),
           c41 = _mm256_setzero_ps(), c50 = _mm256_setzero_ps(), c51 = _mm256_setzero_ps();
    for (size_t k = 0; k < kc; ++k) {
        const __m256 b0 = _mm256_loadu_ps(b + k * NR), b1 = _mm256_loadu_ps(b + k * NR + 8);
        const float *ak = a + k * MR;
        __m256 av = _mm256_broadcast_ss(ak + 0);
        c00 = _mm256_fmadd_ps(av, b0, c00); c01 = _mm256_fmadd_ps(av, b1, c01);
        av = _mm256_broadcast_ss(ak + 1);
        c10 = _mm256_fmadd_ps(av, b0, c10); c11 = _mm256_fmadd_ps(av, b1, c11);
        av = _mm256_broadcast_ss(ak + 2);
        c20 = _mm256_fmadd_ps(av, b0, c20); c21 = _mm256_fmadd_ps(av, b1, c21);
        av = _mm256_broadcast_ss(ak + 3);
        c30 = _mm256_fmadd_ps(av, b0, c30); c31 = _mm256_fmadd_ps(av, b1, c31);
        av = _mm256_broadcast_ss(ak + 4);
        c40 = _mm256_fmadd_ps(av, b0, c40); c41 = _mm256_fmadd_ps(av, b1, c41);
        av = _mm256_broadcast_ss(ak + 5);
        c50 = _mm256_fmadd_ps(av, b0, c50); c51 = _mm256_fmadd_ps(av, b1, c51);
    }
    float t[MR * NR];
    _mm256_storeu_ps(t + 0, c00);  _mm256_storeu_ps(t + 8, c01);
    _mm256_storeu_ps(t + 16, c10); _mm256_storeu_ps(t + 24, c11);
    _mm256_storeu_ps(t + 32, c20); _mm256_storeu_ps(t + 40, c21);
    _mm256_storeu_ps(t + 48, c30); _mm256_storeu_ps(t + 56, c31);
    _mm256_storeu_ps(t + 64, c40); _mm256_storeu_ps(t + 72, c41);
    _mm256_storeu_ps(t + 80, c50); _mm256_storeu_ps(t + 88, c51);
    for (size_t r = 0; r < h; ++r) {
        float *c = C + r * ldc;
        if (accumulate)
            for (size_t j = 0; j < w; ++j) c[j] += t[r * NR + j];
        else
            for (size_t j = 0; j < w; ++j) c[j] = t[r * NR + j];
    }
}

/* Y[M][N] = X[M][K] . W[K][N] + bias (bias may be NULL).  Returns 0, or -1 on allocation failure
 * or a host without AVX2/FMA. */
int orc_sgemm_blocked(const float *X, size_t M, size_t K, const float *W, size_t N, const float *bias, float *Y,
                      int nthreads) {
    if (nthreads < 1) nthreads = 1;
    __builtin_cpu_init();
    if (!__builtin_cpu_supports("avx2") || !__builtin_cpu_supports("fma")) return -1;
    if (M == 0 || N == 0) return 0;
    const size_t nsl = (N + NR - 1) / NR;
    float *Bp = aligned_alloc(64, ((nsl * KC * NR * sizeof(float)) + 63) / 64 * 64);
    float *Ap = aligned_alloc(64, ((size_t)nthreads * MC * KC * sizeof(float) + 63) / 64 * 64);
    if (!Bp || !Ap) {
        free(Bp);
        free(Ap);
        return -1;
    }
    if (K == 0)
        for (size_t i = 0; i < M * N; ++i) Y[i] = 0.0f;
    for (size_t k0 = 0; k0 < K; k0 += KC) {
        const size_t kc = (K - k0) < KC ? (K - k0) : KC;
        pack_b(W, N, k0, kc, Bp, nthreads);
        const size_t nblk = (M + MC - 1) / MC;
#pragma omp parallel for num_threads(nthreads) schedule(static)
        for (size_t ib = 0; ib < nblk; ++ib) {
            const int tid = omp_get_thread_num();
            float *ap = Ap + (size_t)tid * MC * KC;
            const size_t i0 = ib * MC, mc = (M - i0) < MC ? (M - i0) : MC;
            pack_a(X, K, i0, mc, k0, kc, ap);
            for (size_t s = 0; s < nsl; ++s) {
                const size_t j0 = s * NR, w = (N - j0) < NR ? (N - j0) : NR;
                for (size_t r = 0; r < mc; r += MR) {
                    const size_t h = (mc - r) < MR ? (mc - r) : MR;
                    micro_6x16(kc, ap + (r / MR) * kc * MR, Bp + s * kc * NR, Y + (i0 + r) * N + j0, N, h, w,
                               k0 != 0);
                }
            }
        }
    }
    if (bias) {
#pragma omp parallel for num_threads(nthreads) schedule(static)
        for (size_t m = 0; m < M; ++m)
            for (size_t n = 0; n < N; ++n) Y[m * N + n] += bias[n];
    }
    free(Bp);
    free(Ap);
    return 0;
}
