// attention.h — single-token decode attention on gfx950 (the reference's score_cal / safe_softmax /
// score_value_mul trio, source/kernel/cuda/mha_kernel.cu:63-169, and CPU mha_kernel.cpp:36-77,
// re-designed as split-context flash-decoding):
//
//   * one wave64 owns one (kv head, context slice of PPW positions): a 16-byte vector per lane, LPR
//     lanes per cached row, so every K/V row of the slice is read exactly once, straight to VGPRs,
//     K and V loads all issued before the first use;
//   * the G query heads that share the kv head (GQA, mha_kernel.cpp:52,71 `h / group`) reuse the same
//     K/V registers;
//   * per-slice softmax state (m, l, o[hd]) goes to a small fp32 workspace and a one-wave-per-head
//     combine kernel merges the slices (m = max, l = sum e^{m_i-M} l_i, o = sum e^{m_i-M} o_i / l).
// Cache addressing is strided so the same kernel serves the reference layout [L][T][KV] (op API) and
// the engine's head-major layout [L][Hkv][T][hd].
#pragma once
#include "common.h"

namespace sli {

template <typename KT>
struct AttnArgs {
    const float* q;         // [hq * hd]
    const KT* k;            // this layer's cache base
    const KT* v;
    long long pos_stride;   // elements between positions
    long long head_stride;  // elements between kv heads
    float* part;            // [hq][max_splits][hd + 2]
    const int32_t* pos_dev; // nullable: then pos_host
    int pos_host;
    int n_kv_heads;
    int max_splits;
    float scale;            // 1/sqrt(hd) (mha_kernel.cpp:41)
};

constexpr int kAttnNit = 16;  // 16-byte vectors per lane per operand per wave (K and V each)

template <typename KT, int HD>
struct AttnGeom {
    static constexpr int EPV = Vec16<KT>::N;
    static constexpr int LPR = HD / EPV;     // lanes per cached row
    static constexpr int RPI = 64 / LPR;     // rows per wave-instruction
    static constexpr int PPW = kAttnNit * RPI;  // positions per wave (context slice)
    static_assert(LPR >= 1 && LPR <= 64 && (64 % LPR) == 0, "head_dim / vector shape");
};

template <typename KT, int HD, int G>
__global__ void __launch_bounds__(256) attn_partial_kernel(AttnArgs<KT> a) {
    using Geo = AttnGeom<KT, HD>;
    constexpr int EPV = Geo::EPV, LPR = Geo::LPR, RPI = Geo::RPI, PPW = Geo::PPW;
    const int lane = threadIdx.x & 63;
    const int wid = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int kvh = wid / a.max_splits;
    const int split = wid - kvh * a.max_splits;
    if (kvh >= a.n_kv_heads) return;
    const int pos = a.pos_dev ? *a.pos_dev : a.pos_host;
    const int t0 = split * PPW;
    if (t0 > pos) return;  // slice beyond the live context: the combine never reads it
    const int t_end = min(t0 + PPW, pos + 1);
    const int sub = lane / LPR;
    const int li = lane - sub * LPR;

    const KT* kb = a.k + (long long)kvh * a.head_stride + li * EPV;
    const KT* vb = a.v + (long long)kvh * a.head_stride + li * EPV;
    u32x4 kr[kAttnNit], vr[kAttnNit];
#pragma unroll
    for (int it = 0; it < kAttnNit; ++it) {
        const int t = min(t0 + it * RPI + sub, t_end - 1);  // clamp, never branch around a load
        kr[it] = load16<false>(kb + (long long)t * a.pos_stride);
    }
#pragma unroll
    for (int it = 0; it < kAttnNit; ++it) {
        const int t = min(t0 + it * RPI + sub, t_end - 1);
        vr[it] = load16<false>(vb + (long long)t * a.pos_stride);
    }

    float qv[G][EPV];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int e = 0; e < EPV; ++e) qv[g][e] = a.q[(size_t)(kvh * G + g) * HD + li * EPV + e];

    float s[kAttnNit][G];
    float m[G];
#pragma unroll
    for (int g = 0; g < G; ++g) m[g] = -INFINITY;
#pragma unroll
    for (int it = 0; it < kAttnNit; ++it) {
        float kf[EPV];
        Vec16<KT>::unpack(kr[it], kf);
        const bool live = (t0 + it * RPI + sub) < t_end;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            float d = 0.0f;
#pragma unroll
            for (int e = 0; e < EPV; ++e) d = fmaf(qv[g][e], kf[e], d);
            d = group_sum<LPR>(d);
            s[it][g] = live ? d * a.scale : -INFINITY;
            m[g] = fmaxf(m[g], s[it][g]);
        }
    }
    float l[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
#pragma unroll
        for (int o = LPR; o < 64; o <<= 1) m[g] = fmaxf(m[g], __shfl_xor(m[g], o, kWave));
        l[g] = 0.0f;
    }
    float ov[G][EPV];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int e = 0; e < EPV; ++e) ov[g][e] = 0.0f;
#pragma unroll
    for (int it = 0; it < kAttnNit; ++it) {
        float vf[EPV];
        Vec16<KT>::unpack(vr[it], vf);
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const float p = expf(s[it][g] - m[g]);  // 0 for masked rows
            l[g] += p;
#pragma unroll
            for (int e = 0; e < EPV; ++e) ov[g][e] = fmaf(p, vf[e], ov[g][e]);
        }
    }
    // l was accumulated once per lane of a row group (LPR copies of each row): reduce across row groups only
#pragma unroll
    for (int g = 0; g < G; ++g) {
#pragma unroll
        for (int o = LPR; o < 64; o <<= 1) {
            l[g] += __shfl_xor(l[g], o, kWave);
#pragma unroll
            for (int e = 0; e < EPV; ++e) ov[g][e] += __shfl_xor(ov[g][e], o, kWave);
        }
    }
    if (sub == 0) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            float* dst = a.part + ((size_t)(kvh * G + g) * a.max_splits + split) * (HD + 2);
#pragma unroll
            for (int e = 0; e < EPV; ++e) dst[li * EPV + e] = ov[g][e];
            if (li == 0) {
                dst[HD] = m[g];
                dst[HD + 1] = l[g];
            }
        }
    }
}

// One wave per query head: merge the live slices.
template <int HD>
__global__ void __launch_bounds__(64)
    attn_combine_kernel(const float* __restrict__ part, float* __restrict__ out, const int32_t* pos_dev,
                        int pos_host, int max_splits, int ppw) {
    const int h = blockIdx.x;
    const int lane = threadIdx.x;
    const int pos = pos_dev ? *pos_dev : pos_host;
    const int ns = pos / ppw + 1;
    const float* ph = part + (size_t)h * max_splits * (HD + 2);
    float mx = -INFINITY;
    for (int i = lane; i < ns; i += 64) mx = fmaxf(mx, ph[(size_t)i * (HD + 2) + HD]);
    mx = wave_max(mx);
    constexpr int DPL = (HD + 63) / 64;
    float o[DPL];
#pragma unroll
    for (int j = 0; j < DPL; ++j) o[j] = 0.0f;
    float L = 0.0f;
    for (int i = 0; i < ns; ++i) {
        const float* pi = ph + (size_t)i * (HD + 2);
        const float w = expf(pi[HD] - mx);
        L = fmaf(w, pi[HD + 1], L);
#pragma unroll
        for (int j = 0; j < DPL; ++j) {
            const int d = lane + 64 * j;
            if (d < HD) o[j] = fmaf(w, pi[d], o[j]);
        }
    }
#pragma unroll
    for (int j = 0; j < DPL; ++j) {
        const int d = lane + 64 * j;
        if (d < HD) out[(size_t)h * HD + d] = o[j] / L;
    }
}

}  // namespace sli
