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

// A byte range that extra workgroups of a latency-bound launch pull into the Infinity Cache (and L2)
// for the NEXT launch, which then streams it at cache speed: decode attention reads 1/12 of a layer's
// bytes and leaves HBM under-used, and the wo weights it precedes do not depend on it.
struct StreamPrefetch {
    const char* p = nullptr;
    long long bytes = 0;
    int blocks = 0;  // extra 256-thread workgroups appended to the grid
};

// Workgroup `b` of `pf.blocks` reads its contiguous share with default-policy (allocating) 16-byte loads.
__device__ __forceinline__ void stream_prefetch_block(const StreamPrefetch& pf, int b) {
    constexpr int U = 8;
    const long long per = ((pf.bytes / pf.blocks) + 15) & ~15ll;
    const long long lo = per * b, hi = min(pf.bytes, lo + per);
    unsigned sink = 0;
    for (long long o = lo + (long long)threadIdx.x * 16; o < hi; o += (long long)U * blockDim.x * 16) {
        u32x4 w[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const long long a = min(o + (long long)j * blockDim.x * 16, hi - 16);
            w[j] = *reinterpret_cast<const u32x4*>(pf.p + a);
        }
#pragma unroll
        for (int j = 0; j < U; ++j) sink ^= w[j].x;
    }
    if (sink == 0x9e3779b9u && pf.blocks < 0) asm volatile("" ::"v"(sink));  // keep the loads
}

template <typename KT>
struct AttnArgs {
    const float* q;         // [hq * hd]
    const KT* k;            // this layer's cache base
    const KT* v;
    long long pos_stride;   // elements between positions
    long long head_stride;  // elements between kv heads
    float* part;            // [hq][max_splits][hd + kAttnPartPad]: o[hd], m, l, pad
    const int32_t* pos_dev; // nullable: then pos_host
    int pos_host;
    int n_kv_heads;
    int max_splits;
    float scale;            // 1/sqrt(hd) (mha_kernel.cpp:41)
    StreamPrefetch pf;      // optional: workgroups past n_kv_heads * max_splits prefetch this range
};

// A workgroup covers kAttnSlots wave-instructions of K (and of V) per lane-row group: WAVES waves of
// NIT = kAttnSlots / WAVES vectors each. The split geometry (positions per workgroup) is therefore the
// same for every WAVES; WAVES trades registers for latency hiding: 16 waves of 4 (MHA, GQA-2: each
// wave starts computing as soon as its own few rows land, 4 waves per SIMD overlap) or 4 waves of 16
// (GQA-4/8, whose G query heads need the register room of one wave per SIMD).
constexpr int kAttnSlots = 64;
constexpr int kAttnMaxWgSplits = 128;  // combine-kernel capacity

template <typename KT, int HD>
struct AttnGeom {
    static constexpr int EPV = Vec16<KT>::N;
    static constexpr int LPR = HD / EPV;     // lanes per cached row
    static constexpr int RPI = 64 / LPR;     // rows per wave-instruction
    static constexpr int PPWG = kAttnSlots * RPI;  // positions per workgroup (context split)
    static_assert(LPR >= 1 && LPR <= 64 && (64 % LPR) == 0, "head_dim / vector shape");
};

__host__ __device__ constexpr int attn_waves(int g) { return g <= 2 ? 16 : 4; }

// grid: n_kv_heads * wg_splits workgroups; wave w of workgroup (kvh, s) owns the w-th slice of split s.
// The WAVES slice states are merged in LDS, so one partial per (q head, workgroup) reaches the workspace.
template <typename KT, int HD, int G>
__global__ void __launch_bounds__(64 * attn_waves(G)) attn_partial_kernel(AttnArgs<KT> a) {
    using Geo = AttnGeom<KT, HD>;
    constexpr int WAVES = attn_waves(G), kAttnNit = kAttnSlots / WAVES;
    constexpr int EPV = Geo::EPV, LPR = Geo::LPR, RPI = Geo::RPI, PPW = kAttnNit * RPI;
    __shared__ float sh[WAVES][G][HD + 2];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    if ((int)blockIdx.x >= a.n_kv_heads * a.max_splits) {
        stream_prefetch_block(a.pf, (int)blockIdx.x - a.n_kv_heads * a.max_splits);
        return;
    }
    const int kvh = blockIdx.x / a.max_splits;  // max_splits counts workgroup splits here
    const int wgs = blockIdx.x - kvh * a.max_splits;
    const int pos = a.pos_dev ? *a.pos_dev : a.pos_host;
    if (wgs * WAVES * PPW > pos) return;  // whole workgroup past the live context (uniform exit)
    const int t0 = (wgs * WAVES + wave) * PPW;
    const bool live_wave = t0 <= pos;
    const int t_end = min(t0 + PPW, pos + 1);
    const int sub = lane / LPR;
    const int li = lane - sub * LPR;

    float m[G], l[G], ov[G][EPV];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        m[g] = -INFINITY;
        l[g] = 0.0f;
#pragma unroll
        for (int e = 0; e < EPV; ++e) ov[g][e] = 0.0f;
    }
    if (live_wave) {
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
                s[it][g] = live ? d * a.scale : -INFINITY;  // mha_kernel.cpp:51-60 (sum * scale)
                m[g] = fmaxf(m[g], s[it][g]);
            }
        }
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int o = LPR; o < 64; o <<= 1) m[g] = fmaxf(m[g], __shfl_xor(m[g], o, kWave));
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
        // every lane of a row group holds the same p: reduce across row groups only
#pragma unroll
        for (int g = 0; g < G; ++g) {
#pragma unroll
            for (int o = LPR; o < 64; o <<= 1) {
                l[g] += __shfl_xor(l[g], o, kWave);
#pragma unroll
                for (int e = 0; e < EPV; ++e) ov[g][e] += __shfl_xor(ov[g][e], o, kWave);
            }
        }
    }
    if (sub == 0) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
#pragma unroll
            for (int e = 0; e < EPV; ++e) sh[wave][g][li * EPV + e] = ov[g][e];
            if (li == 0) {
                sh[wave][g][HD] = m[g];
                sh[wave][g][HD + 1] = l[g];
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < G * HD; i += blockDim.x) {
        const int g = i / HD, d = i - g * HD;
        float M = -INFINITY;
#pragma unroll
        for (int w = 0; w < WAVES; ++w) M = fmaxf(M, sh[w][g][HD]);
        float o = 0.0f, L = 0.0f;
#pragma unroll
        for (int w = 0; w < WAVES; ++w) {
            const float c = expf(sh[w][g][HD] - M);  // dead waves: m = -inf -> 0
            o = fmaf(c, sh[w][g][d], o);
            L = fmaf(c, sh[w][g][HD + 1], L);
        }
        float* dst = a.part + ((size_t)(kvh * G + g) * a.max_splits + wgs) * (HD + kAttnPartPad);
        dst[d] = o;
        if (d == 0) {
            dst[HD] = M;
            dst[HD + 1] = L;
        }
    }
}

// One workgroup per query head: merge the live workgroup partials (independent loads per split).
template <int HD>
__global__ void __launch_bounds__(256)
    attn_combine_kernel(const float* __restrict__ part, float* __restrict__ out, const int32_t* pos_dev,
                        int pos_host, int max_splits, int ppw_wg) {
    __shared__ float sw[kAttnMaxWgSplits];
    __shared__ float sL;
    const int h = blockIdx.x;
    const int tid = threadIdx.x;
    const int pos = pos_dev ? *pos_dev : pos_host;
    const int ns = pos / ppw_wg + 1;
    constexpr int PS = HD + kAttnPartPad;
    const float* ph = part + (size_t)h * max_splits * PS;
    if (tid < 64) {
        float mx = -INFINITY;
        for (int i = tid; i < ns; i += 64) mx = fmaxf(mx, ph[(size_t)i * PS + HD]);
        mx = wave_max(mx);
        float L = 0.0f;
        for (int i = tid; i < ns; i += 64) {
            const float w = expf(ph[(size_t)i * PS + HD] - mx);
            sw[i] = w;
            L = fmaf(w, ph[(size_t)i * PS + HD + 1], L);
        }
        L = wave_sum(L);
        if (tid == 0) sL = L;
    }
    __syncthreads();
    const float L = sL;
    for (int d = tid; d < HD; d += blockDim.x) {
        float o = 0.0f;
#pragma unroll 8
        for (int i = 0; i < ns; ++i) o = fmaf(sw[i], ph[(size_t)i * PS + d], o);
        out[(size_t)h * HD + d] = o / L;
    }
}

}  // namespace sli
