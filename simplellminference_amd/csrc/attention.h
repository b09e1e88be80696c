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
    float* out;             // [hq * hd] merged attention output
    unsigned* counters;     // [n_kv_heads] arrival counters, zero between launches (the last arriver resets)
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
    // Workgroup partial: the WAVES slice states merged in LDS, published write-through (sc1) so the
    // head's last-arriving workgroup can read it from any XCD without a fence pair
    // (MI355X_MICROARCH.md, hand-off table row 1: sc1 stores, drained, one agent-scope add per
    // workgroup behind a workgroup barrier, sc1 loads by the last adder after the barrier it joins).
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
        __hip_atomic_store(dst + d, o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (d == 0) {
            __hip_atomic_store(dst + HD, M, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(dst + HD + 1, L, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains before the arrival
    __syncthreads();
    __shared__ int last;
    const int ns = min(pos / (WAVES * PPW) + 1, a.max_splits);  // live workgroups of this kv head
    if (threadIdx.x == 0) {
        const unsigned prev = __hip_atomic_fetch_add(a.counters + kvh, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = prev == (unsigned)(ns - 1);
        if (last) __hip_atomic_store(a.counters + kvh, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!last) return;
    // Last arriver: merge the head's ns partials in split order (deterministic whatever the arrival
    // order): M = max m_i, w_i = e^{m_i - M}, out = (sum_i w_i o_i) / (sum_i w_i l_i).
    float* ml = &sh[0][0][0];  // reuse: [G][ns][2]
    for (int i = threadIdx.x; i < G * ns; i += blockDim.x) {
        const int g = i / ns, sp = i - g * ns;
        const float* src = a.part + ((size_t)(kvh * G + g) * a.max_splits + sp) * (HD + kAttnPartPad);
        ml[2 * i] = __hip_atomic_load(src + HD, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ml[2 * i + 1] = __hip_atomic_load(src + HD + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < G * HD; i += blockDim.x) {
        const int g = i / HD, d = i - g * HD;
        const float* src = a.part + (size_t)(kvh * G + g) * a.max_splits * (HD + kAttnPartPad) + d;
        const float* mlg = ml + 2 * g * ns;
        float M = -INFINITY;
        for (int sp = 0; sp < ns; ++sp) M = fmaxf(M, mlg[2 * sp]);
        float o = 0.0f, L = 0.0f;
        for (int sp = 0; sp < ns; ++sp) {
            const float w = expf(mlg[2 * sp] - M);
            const float ov = __hip_atomic_load(src + (size_t)sp * (HD + kAttnPartPad), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
            o = fmaf(w, ov, o);
            L = fmaf(w, mlg[2 * sp + 1], L);
        }
        a.out[(size_t)(kvh * G + g) * HD + d] = o / L;
    }
}

}  // namespace sli
