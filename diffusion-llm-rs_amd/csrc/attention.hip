// attention.hip -- quantized-KV dequant-attention for gfx950 (a9, build-defined consumer).
//
// The reference dequantizes the per-tensor-quantized K and V of its cache every timestep
// (QuantizedKVCacheEntry::dequantize_keys/values, diffuse-llm-rs/src/quantization.rs:160-175) and
// hands them to DiffusionModel::forward_with_cache (diffuse-llm-rs/src/lib.rs:910-915).  Here the
// dequantization y = (q - zp) * scale (a2) is fused into a flash-style bidirectional SDPA,
// O = softmax(Q K^T / sqrt(D)) V per head.  Because K and V each carry ONE per-tensor scale,
//   Q K^T = s_k * (Q (q_k - z_k)^T)   and   P V = s_v * (P (q_v - z_v)),
// so only the exact integers (q - z) are staged (exact in f16) and the scales fold into the softmax
// exponent and the final normalisation: fewer roundings than dequantizing to f16 first.
//
// Layout: Q, O f16 [S][H][D]; K, V codes in the canonical packed bitstream of the flattened
// [S][H][D] tensor (one per-tensor {scale, zp} pair each, on the device), D = 128.
// Workgroup = 8 waves = 256 queries of one head; every 64-key block of K and V is staged once in
// LDS (K as [key][d], V transposed as [d][key]) and shared by the 8 waves; two LDS buffers, one
// barrier per block: block j+1's codes are loaded before block j's MFMAs and written to the other
// buffer after them.
// Per wave (32 queries): S^T = K Q^T with 32x32x16 f16 MFMA (keys in registers, the query on the
// lane, so the softmax row reductions are lane-local plus one cross-half shuffle), then O = P V with
// the S^T accumulator converted in place to the A operand (no LDS round trip for P).  The O rescale
// is skipped when no query's running max moved (exact: the factor is then 1).
#include "common.hpp"

typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef _Float16 half4_t __attribute__((ext_vector_type(4)));
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
typedef float float16_t __attribute__((ext_vector_type(16)));

namespace dllm {
namespace {

constexpr int kD = 128;          // head dim
constexpr int kKB = 64;          // keys per block
constexpr int kWaves = 8;
constexpr int kQT = 32 * kWaves; // queries per workgroup
constexpr int kKRow = kD + 8;    // K row stride (halves): 272 B, conflict-free b128 fragment reads
constexpr int kVRow = kKB + 8;   // Vt row stride (halves): 144 B

struct AttnBuf {
    _Float16 k[kKB][kKRow];       // 17 KiB
    _Float16 vt[kD][kVRow];       // 18 KiB
};
struct AttnSmem {
    AttnBuf buf[2];
    float bcast[kWaves][32];      // per-wave per-query factors (alpha, then 1/l)
};

// Codes of one thread's share of a block, loaded to registers ahead of the MFMAs.
// K: thread t < 256 owns key t>>2, dims 32*(t&3) .. +32 (one row chunk).
// V: thread t >= 256 owns keys 4*((t-256)>>4) .. +4, dims 8*((t-256)&15) .. +8 (a 4x8 micro-tile).
template <int BITS>
struct Raw {
    uint32_t w[BITS == 4 ? 4 : 8];
};

template <int BITS>
__device__ __forceinline__ void load_raw(Raw<BITS> &r, const uint8_t *__restrict__ Kq, const uint8_t *__restrict__ Vq,
                                         int tid, int j0, int S, int H, int h) {
    if (tid < 256) {
        const int key = tid >> 2, d0 = 32 * (tid & 3);
        const int s = min(j0 + key, S - 1);
        const size_t e = (static_cast<size_t>(s) * H + h) * kD + d0;
        if constexpr (BITS == 4) {
            const uint4 v = *reinterpret_cast<const uint4 *>(Kq + e / 2);   // 32 codes
            r.w[0] = v.x; r.w[1] = v.y; r.w[2] = v.z; r.w[3] = v.w;
        } else {
            const uint4 a = *reinterpret_cast<const uint4 *>(Kq + e), b = *reinterpret_cast<const uint4 *>(Kq + e + 16);
            r.w[0] = a.x; r.w[1] = a.y; r.w[2] = a.z; r.w[3] = a.w; r.w[4] = b.x; r.w[5] = b.y; r.w[6] = b.z; r.w[7] = b.w;
        }
    } else {
        const int t = tid - 256, k4 = 4 * (t >> 4), d0 = 8 * (t & 15);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int s = min(j0 + k4 + i, S - 1);
            const size_t e = (static_cast<size_t>(s) * H + h) * kD + d0;
            if constexpr (BITS == 4) {
                r.w[i] = *reinterpret_cast<const uint32_t *>(Vq + e / 2);          // 8 codes
            } else {
                const uint2 v = *reinterpret_cast<const uint2 *>(Vq + e);
                r.w[2 * i] = v.x; r.w[2 * i + 1] = v.y;
            }
        }
    }
}

// Code c (0..7) of an 8-code group of the thread's raw words, as the f16 pair trick input.
template <int BITS>
__device__ __forceinline__ half2_t pair_qz(uint32_t lo_word_codes, int shift, half2_t nz) {
    // (code_a at bit shift, code_b at bit shift + BITS) -> f16 pair (1024 + code) - (1024 + z)
    const uint32_t m = (1u << BITS) - 1u;
    const uint32_t a = (lo_word_codes >> shift) & m, b = (lo_word_codes >> (shift + BITS)) & m;
    const uint32_t t = (a | (b << 16)) | 0x64006400u;
    return __builtin_bit_cast(half2_t, t) + nz;   // exact
}

template <int BITS>
__device__ __forceinline__ void store_raw(const Raw<BITS> &r, AttnBuf &b, int tid, half2_t kz, half2_t vz) {
    constexpr int CPW = 32 / BITS;   // codes per word
    if (tid < 256) {
        const int key = tid >> 2, d0 = 32 * (tid & 3);
#pragma unroll
        for (int g = 0; g < 4; ++g) {   // 4 x 8 codes -> 4 x b128 stores
            half8_t out;
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const int c = 8 * g + 2 * p;   // code index within the 32
                const half2_t v = pair_qz<BITS>(r.w[c / CPW], BITS * (c % CPW), kz);
                out[2 * p] = v[0];
                out[2 * p + 1] = v[1];
            }
            *reinterpret_cast<half8_t *>(&b.k[key][d0 + 8 * g]) = out;
        }
    } else {
        const int t = tid - 256, k4 = 4 * (t >> 4), d0 = 8 * (t & 15);
        _Float16 v[4][8];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const int c = 2 * p;
                const uint32_t word = (BITS == 4) ? r.w[i] : r.w[2 * i + (c / CPW)];
                const half2_t x = pair_qz<BITS>(word, BITS * (c % CPW), vz);
                v[i][2 * p] = x[0];
                v[i][2 * p + 1] = x[1];
            }
#pragma unroll
        for (int dd = 0; dd < 8; ++dd)   // transposed: 4 consecutive keys of one dim per 8-B store
            *reinterpret_cast<half4_t *>(&b.vt[d0 + dd][k4]) = half4_t{v[0][dd], v[1][dd], v[2][dd], v[3][dd]};
    }
}

template <int BITS>
__global__ void __launch_bounds__(kWaves * 64)
kv_attention_kernel(const _Float16 *__restrict__ Q, const uint8_t *__restrict__ Kq, const float *__restrict__ kp,
                    const uint8_t *__restrict__ Vq, const float *__restrict__ vp, int S, int H,
                    _Float16 *__restrict__ O) {
    __shared__ __attribute__((aligned(16))) AttnSmem sm;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = blockIdx.y;
    const int q0 = blockIdx.x * kQT + wave * 32;
    const int ql = lane & 31, hh = lane >> 5;
    const float ks = kp[0], vs = vp[0];
    const _Float16 nkz = static_cast<_Float16>(-(1024.0f + kp[1]));   // zp is an integer <= 255: exact
    const _Float16 nvz = static_cast<_Float16>(-(1024.0f + vp[1]));
    const half2_t kz{nkz, nkz}, vz{nvz, nvz};
    // exp2 domain, K scale folded in: p = exp2(c * raw - m), c = log2(e) * s_k / sqrt(D).
    const float c = 1.4426950408889634f * ks / sqrtf(static_cast<float>(kD));

    // Q^T fragments (B operand of S^T = K Q^T): lane holds Q[q = q0 + ql][d = 16 t + 8 hh + j].
    half8_t qf[kD / 16];
    {
        const int qrow = min(q0 + ql, S - 1);
        const _Float16 *qp = Q + (static_cast<size_t>(qrow) * H + h) * kD + 8 * hh;
#pragma unroll
        for (int t = 0; t < kD / 16; ++t) qf[t] = *reinterpret_cast<const half8_t *>(qp + 16 * t);
    }

    float16_t o[kD / 32];   // O tiles: d-tile dt, lane = d (within tile), rows = query via regs
#pragma unroll
    for (int dt = 0; dt < kD / 32; ++dt)
#pragma unroll
        for (int e = 0; e < 16; ++e) o[dt][e] = 0.0f;
    float m_run = -INFINITY, l_run = 0.0f;   // for query q0 + ql (same in both lane halves)

    const int nkb = (S + kKB - 1) / kKB;
    Raw<BITS> raw;
    load_raw<BITS>(raw, Kq, Vq, tid, 0, S, H, h);
    store_raw<BITS>(raw, sm.buf[0], tid, kz, vz);
    __syncthreads();

    for (int kb = 0; kb < nkb; ++kb) {
        const int j0 = kb * kKB;
        AttnBuf &cur = sm.buf[kb & 1];
        const bool more = kb + 1 < nkb;
        if (more) load_raw<BITS>(raw, Kq, Vq, tid, j0 + kKB, S, H, h);   // in flight during the MFMAs

        // ---- S^T (2 x 32 keys x 32 queries) = (q_k - z_k) Q^T ----
        float16_t st[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
#pragma unroll
            for (int e = 0; e < 16; ++e) st[u][e] = 0.0f;
#pragma unroll
            for (int t = 0; t < kD / 16; ++t) {
                const half8_t kf = *reinterpret_cast<const half8_t *>(&cur.k[32 * u + ql][16 * t + 8 * hh]);
                st[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf, qf[t], st[u], 0, 0, 0);
            }
        }
        // st[u][r]: key = j0 + 32u + (r&3) + 8(r>>2) + 4 hh, query = q0 + ql.
        float mloc = -INFINITY;
        const bool tail = j0 + kKB > S;
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                if (tail) {
                    const int key = j0 + 32 * u + (r & 3) + 8 * (r >> 2) + 4 * hh;
                    st[u][r] = key < S ? st[u][r] : -INFINITY;
                }
                mloc = fmaxf(mloc, st[u][r]);
            }
        mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
        const float m_new = fmaxf(m_run, mloc * c);
        const float alpha = exp2f(m_run - m_new);   // exactly 1 when the max did not move
        float lsum = 0.0f;
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                st[u][r] = exp2f(fmaf(st[u][r], c, -m_new));
                lsum += st[u][r];
            }
        lsum += __shfl_xor(lsum, 32, 64);
        l_run = l_run * alpha + lsum;
        m_run = m_new;
        // ---- rescale O rows by their query's alpha, only if some query's max moved ----
        if (!__all(alpha == 1.0f)) {
            if (hh == 0) sm.bcast[wave][ql] = alpha;
            __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float4 a4 = *reinterpret_cast<const float4 *>(&sm.bcast[wave][8 * g + 4 * hh]);
#pragma unroll
                for (int dt = 0; dt < kD / 32; ++dt) {
                    o[dt][4 * g + 0] *= a4.x; o[dt][4 * g + 1] *= a4.y;
                    o[dt][4 * g + 2] *= a4.z; o[dt][4 * g + 3] *= a4.w;
                }
            }
        }
        // ---- O += P (q_v - z_v): P^T accumulator as the A operand (k-step s: keys 16s..16s+15) ----
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int u = s >> 1, sl = s & 1;
            half8_t pa;
#pragma unroll
            for (int j = 0; j < 8; ++j) pa[j] = static_cast<_Float16>(st[u][8 * sl + j]);
#pragma unroll
            for (int dt = 0; dt < kD / 32; ++dt) {
                // element j <-> key 16s + 8(j>>2) + 4hh + (j&3), d = 32dt + ql
                const _Float16 *vrow = &cur.vt[32 * dt + ql][16 * s + 4 * hh];
                const half4_t lo = *reinterpret_cast<const half4_t *>(vrow);
                const half4_t hi = *reinterpret_cast<const half4_t *>(vrow + 8);
                const half8_t vb = half8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(pa, vb, o[dt], 0, 0, 0);
            }
        }
        if (more) store_raw<BITS>(raw, sm.buf[(kb + 1) & 1], tid, kz, vz);
        __syncthreads();   // next block staged; this block's buffer free for block kb+2
    }

    // ---- normalise (1/l and the V scale) and store: o[dt][r] -> query q0 + (r&3) + 8(r>>2) + 4hh ----
    if (hh == 0) sm.bcast[wave][ql] = vs / l_run;
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const float4 inv = *reinterpret_cast<const float4 *>(&sm.bcast[wave][8 * g + 4 * hh]);
        const float iv[4] = {inv.x, inv.y, inv.z, inv.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int q = q0 + 8 * g + 4 * hh + i;
            if (q >= S) continue;
            _Float16 *op = O + (static_cast<size_t>(q) * H + h) * kD + ql;
#pragma unroll
            for (int dt = 0; dt < kD / 32; ++dt) op[32 * dt] = static_cast<_Float16>(o[dt][4 * g + i] * iv[i]);
        }
    }
}

}  // namespace
}  // namespace dllm

using namespace dllm;

extern "C" int dllm_kv_attention(const void *Q, const uint8_t *Kq, const float *k_params, const uint8_t *Vq,
                                 const float *v_params, uint8_t bits, size_t S, size_t H, size_t D, void *O,
                                 dllm_stream_t stream) {
    if (D != kD) return fail(DLLM_ERR_UNSUPPORTED, "dllm_kv_attention: head dim must be 128");
    if (bits != 4 && bits != 8) return fail(DLLM_ERR_UNSUPPORTED, "dllm_kv_attention: bits must be 4 or 8");
    if (S == 0 || H == 0) return DLLM_OK;
    if (!Q || !Kq || !Vq || !k_params || !v_params || !O) return fail(DLLM_ERR_INVALID_PARAMS, "null pointer");
    if (S > (1u << 28) || H > 65535) return fail(DLLM_ERR_SHAPE_MISMATCH, "S or H too large");
    if ((reinterpret_cast<uintptr_t>(Kq) & 15) || (reinterpret_cast<uintptr_t>(Vq) & 15) ||
        (reinterpret_cast<uintptr_t>(Q) & 15))
        return fail(DLLM_ERR_INVALID_PARAMS, "Q, K and V codes must be 16-byte aligned");
    dim3 grid(static_cast<unsigned>((S + kQT - 1) / kQT), static_cast<unsigned>(H));
    if (bits == 4)
        kv_attention_kernel<4><<<grid, kWaves * 64, 0, as_stream(stream)>>>(
            static_cast<const _Float16 *>(Q), Kq, k_params, Vq, v_params, (int)S, (int)H, static_cast<_Float16 *>(O));
    else
        kv_attention_kernel<8><<<grid, kWaves * 64, 0, as_stream(stream)>>>(
            static_cast<const _Float16 *>(Q), Kq, k_params, Vq, v_params, (int)S, (int)H, static_cast<_Float16 *>(O));
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}
