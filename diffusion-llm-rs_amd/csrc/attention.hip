// attention.hip -- quantized-KV dequant-attention for gfx950 (a9, build-defined consumer).
//
// The reference dequantizes the per-tensor-quantized K and V of its cache every timestep
// (QuantizedKVCacheEntry::dequantize_keys/values, diffuse-llm-rs/src/quantization.rs:160-175) and
// hands them to DiffusionModel::forward_with_cache (diffuse-llm-rs/src/lib.rs:910-915).  Here the
// dequantization (a2: y = (q - zp) * scale, exact f32, then rounded to f16) is fused into a
// flash-style bidirectional SDPA: O = softmax(Q K^T / sqrt(D)) V per head.
//
// Layout: Q, O f16 [S][H][D]; K, V codes in the canonical packed bitstream of the flattened
// [S][H][D] tensor (one per-tensor {scale, zp} pair each, on the device), D = 128.
// Block = 8 waves = 256 query rows of one head; every 32-key block of K and V is dequantized
// once into LDS (K as [key][d], V transposed as [d][key]) and shared by the 8 waves.
// Per wave (32 query rows): S^T = K Q^T with 32x32x16 f16 MFMA (keys in registers, the query on
// the lane, so the softmax row reductions are lane-local plus one cross-half shuffle), then
// O = P V with the S^T accumulator converted in place to the A operand (no LDS round trip for P).
#include "common.hpp"

typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef _Float16 half4_t __attribute__((ext_vector_type(4)));
typedef float float16_t __attribute__((ext_vector_type(16)));

namespace dllm {
namespace {

constexpr int kD = 128;          // head dim
constexpr int kKB = 32;          // keys per block
constexpr int kWaves = 8;
constexpr int kQT = 32 * kWaves; // query rows per workgroup

struct AttnSmem {
    _Float16 k[kKB][kD + 8];      // 8.5 KiB, K block [key][d] (+16 B pad per row: conflict-free b128 reads)
    _Float16 vt[kD][kKB + 8];     // ~10 KiB, V block transposed [d][key] (+8 pad: 80-B rows)
    float alpha[kWaves][32];      // per-wave per-query rescale factors
};

// Dequantizes 16 consecutive codes starting at element e of the packed stream into f16 (a2 in f32,
// then rounded).
template <int BITS>
__device__ __forceinline__ void dequant16(const uint8_t *__restrict__ q, size_t e, float scale, float zp,
                                          _Float16 (&out)[16]) {
    if constexpr (BITS == 4) {
        const uint2 v = *reinterpret_cast<const uint2 *>(q + e / 2);   // 16 nibbles
        const uint64_t w = (static_cast<uint64_t>(v.y) << 32) | v.x;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            float d = static_cast<float>((w >> (4 * i)) & 0xF) - zp;
            out[i] = static_cast<_Float16>(d * scale);
        }
    } else {
        const uint4 v = *reinterpret_cast<const uint4 *>(q + e);
        const uint32_t ww[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            float d = static_cast<float>((ww[i >> 2] >> (8 * (i & 3))) & 0xFF) - zp;
            out[i] = static_cast<_Float16>(d * scale);
        }
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
    const float ks = kp[0], kz = kp[1], vs = vp[0], vz = vp[1];
    // log2(e) / sqrt(D): scores kept in the exp2 domain.
    const float c = 1.4426950408889634f / sqrtf(static_cast<float>(kD));

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
    float m_run = -INFINITY, l_run = 0.0f;   // for query q0 + ql (duplicated in both lane halves)

    const int nkb = (S + kKB - 1) / kKB;
    for (int kb = 0; kb < nkb; ++kb) {
        const int j0 = kb * kKB;
        // ---- cooperative dequant of the K / V block into LDS: threads 0..255 K, 256..511 V,
        //      16 consecutive codes of one key row each ----
        {
            const int t = tid & 255;
            const int key = t >> 3;              // 0..31
            const int d0 = (t & 7) * 16;         // 0..112
            const int s = min(j0 + key, S - 1);
            const size_t e = (static_cast<size_t>(s) * H + h) * kD + d0;
            _Float16 vals[16];
            if (tid < 256) {
                dequant16<BITS>(Kq, e, ks, kz, vals);
                half8_t a, b;
#pragma unroll
                for (int i = 0; i < 8; ++i) { a[i] = vals[i]; b[i] = vals[8 + i]; }
                *reinterpret_cast<half8_t *>(&sm.k[key][d0]) = a;
                *reinterpret_cast<half8_t *>(&sm.k[key][d0 + 8]) = b;
            } else {
                dequant16<BITS>(Vq, e, vs, vz, vals);
#pragma unroll
                for (int i = 0; i < 16; ++i) sm.vt[d0 + i][key] = vals[i];
            }
        }
        __syncthreads();

        // ---- S^T (32 keys x 32 queries) = K Q^T ----
        float16_t st;
#pragma unroll
        for (int e = 0; e < 16; ++e) st[e] = 0.0f;
#pragma unroll
        for (int t = 0; t < kD / 16; ++t) {
            const half8_t kf = *reinterpret_cast<const half8_t *>(&sm.k[ql][16 * t + 8 * hh]);
            st = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf, qf[t], st, 0, 0, 0);
        }
        // st[r]: key = j0 + (r&3) + 8(r>>2) + 4 hh, query = q0 + ql.
        float mloc = -INFINITY;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int key = j0 + (r & 3) + 8 * (r >> 2) + 4 * hh;
            st[r] = (key < S) ? st[r] * c : -INFINITY;
            mloc = fmaxf(mloc, st[r]);
        }
        mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
        const float m_new = fmaxf(m_run, mloc);
        const float alpha = exp2f(m_run - m_new);   // exp2(-inf) = 0 on the first block
        float lsum = 0.0f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            st[r] = exp2f(st[r] - m_new);
            lsum += st[r];
        }
        lsum += __shfl_xor(lsum, 32, 64);
        l_run = l_run * alpha + lsum;
        m_run = m_new;
        // ---- rescale O rows by alpha of their query (broadcast through LDS) ----
        if (hh == 0) sm.alpha[wave][ql] = alpha;
        __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const float4 a4 = *reinterpret_cast<const float4 *>(&sm.alpha[wave][8 * g + 4 * hh]);
#pragma unroll
            for (int dt = 0; dt < kD / 32; ++dt) {
                o[dt][4 * g + 0] *= a4.x; o[dt][4 * g + 1] *= a4.y;
                o[dt][4 * g + 2] *= a4.z; o[dt][4 * g + 3] *= a4.w;
            }
        }
        // ---- O += P V: P^T accumulator as the A operand (k-step s = keys 16s..16s+15) ----
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            half8_t pa;
#pragma unroll
            for (int j = 0; j < 8; ++j) pa[j] = static_cast<_Float16>(st[8 * s + j]);
#pragma unroll
            for (int dt = 0; dt < kD / 32; ++dt) {
                // element j <-> key 16s + 8(j>>2) + 4hh + (j&3), d = 32dt + ql
                const _Float16 *vrow = &sm.vt[32 * dt + ql][16 * s + 4 * hh];
                const half4_t lo = *reinterpret_cast<const half4_t *>(vrow);
                const half4_t hi = *reinterpret_cast<const half4_t *>(vrow + 8);
                const half8_t vb = half8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(pa, vb, o[dt], 0, 0, 0);
            }
        }
        __syncthreads();   // K/V block consumed by every wave before it is overwritten
    }

    // ---- normalise and store: o[dt][r] -> query q0 + (r&3) + 8(r>>2) + 4hh, d = 32dt + ql ----
    if (hh == 0) sm.alpha[wave][ql] = 1.0f / l_run;
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const float4 inv = *reinterpret_cast<const float4 *>(&sm.alpha[wave][8 * g + 4 * hh]);
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
