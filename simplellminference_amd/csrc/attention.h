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
    float* part;            // [hq][max_splits][hd + kAttnPartPad]: o[hd], m, l, pad
    float* out;             // [hq * hd] merged attention output
    unsigned* counters;     // [n_kv_heads] arrival counters, zero between launches (the last arriver resets)
    const int32_t* pos_dev; // nullable: then pos_host
    int pos_host;
    int n_kv_heads;
    int max_splits;
    float scale;            // 1/sqrt(hd) (mha_kernel.cpp:41)
    int seq_heads;          // kv heads per sequence: a batch is B sequences of seq_heads kv heads each
    int pos_seq_stride;     // int32s between consecutive sequences' positions at pos_dev
    unsigned long long* stamps = nullptr;  // diagnostic (tools/attn_lab): per-workgroup s_memrealtime x4
    int cache_heads = 0;    // > 0: the cache holds cache_heads kv heads shared by every sequence (prefill lanes
                            // of one sequence): kv head kvh reads cache head kvh % cache_heads
    int ppwg = 0;           // context positions per workgroup split (0: AttnGeom's PPWG; attn_stream.h sets it)
    int kv_group = 1;       // > 1: kv head kvh reads cache head kvh / kv_group (a GQA head group run as kv_group
                            // narrower groups that share each K/V row through the L2, ops.hip mha_launch_hd)
    int defer_merge = 0;    // != 0: only write the workgroup partials (plain stores); the splits are merged
                            // after the launch: 1 by the consumer (the wo GEMV's input staging, gemv.h
                            // XStageMerge), 2 by attn_merge_kernel (mha_launch launches it)
    // HAND (the fused q/k/v + attention launch, qkv_attn.h): q and this step's K/V rows are produced by the q/k/v
    // workgroups of the same launch, stored write-through (sc1) and counted per kv head
    const float* hand_kv = nullptr;  // [2][n_kv_heads][hd]: this step's k rows, then its v rows (cache-rounded)
    unsigned* hand_count = nullptr;  // attn_hand_bytes: q/k/v units landed per kv head (kAttnHandSub counters, one
                                     // per 128-byte line), then live workgroups done per kv head (the last resets)
    unsigned hand_expect = 0;        // units per kv head: (G + 2) * hd / 2
    int* hand_err = nullptr;         // DevState::error: a bounded wait that gave up sets kAttnErrHand
};

constexpr int kAttnErrHand = 8;               // DevState::error bit (oneshot.h 4)
constexpr unsigned kAttnHandSpin = 1u << 22;  // bounded wait (~seconds)
// A kv head's arrivals are spread over kAttnHandSub counters on separate 128-byte lines (producer workgroup b
// adds to counter b % kAttnHandSub): same-line device-scope atomics serialise (measured: one add per q/k/v unit on
// one line cost 23 / 45 us per TP-8 / TP-4 launch).
constexpr int kAttnHandSub = 16;
constexpr int kAttnHandLine = 32;  // unsigned per 128-byte line
__host__ __device__ constexpr size_t attn_hand_words(int n_kv_heads) {
    return (size_t)n_kv_heads * (kAttnHandSub + 1) * kAttnHandLine;
}
__host__ __device__ __forceinline__ unsigned* attn_hand_sub(unsigned* c, int kvh, int sub) {
    return c + ((size_t)kvh * kAttnHandSub + sub) * kAttnHandLine;
}
__host__ __device__ __forceinline__ unsigned* attn_hand_done(unsigned* c, int n_kv_heads, int kvh) {
    return c + ((size_t)n_kv_heads * kAttnHandSub + kvh) * kAttnHandLine;
}

// HAND: a wave's wait for its kv head's q / k / v units: lanes 0..kAttnHandSub-1 read one counter each, summed
// across the wave (the first read also waits for the K/V rows issued ahead of it, which the wave needs next anyway).
template <typename KT>
__device__ __forceinline__ void attn_hand_wait(const AttnArgs<KT>& a, int kvh) {
    const int lane = threadIdx.x & 63;
    unsigned* c = attn_hand_sub(a.hand_count, kvh, min(lane, kAttnHandSub - 1));
    for (unsigned spins = 0;; ++spins) {
        const unsigned v = __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((unsigned)wave_sum(lane < kAttnHandSub ? (float)v : 0.0f) >= a.hand_expect) break;  // exact below 2^24
        if (spins >= kAttnHandSpin) {
            __hip_atomic_fetch_or(a.hand_err, kAttnErrHand, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}
// HAND: one sc1 element of a handed-off vector
__device__ __forceinline__ float attn_hand_ld(const float* p) {
    return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Position of the sequence that owns (batched) kv head kvh.
template <typename KT>
__device__ __forceinline__ int attn_pos(const AttnArgs<KT>& a, int kvh) {
    return a.pos_dev ? a.pos_dev[(size_t)(kvh / a.seq_heads) * a.pos_seq_stride] : a.pos_host;
}

// A workgroup covers kAttnSlots wave-instructions of K (and of V) per lane-row group: WAVES waves of
// NIT = kAttnSlots / WAVES vectors each. The split geometry (positions per workgroup) is therefore the
// same for every WAVES; WAVES trades registers for latency hiding: 16 waves of 4 (MHA, GQA-2: each
// wave starts computing as soon as its own few rows land, 4 waves per SIMD overlap), 8 waves of 8
// (GQA-4) or 4 waves of 16 (GQA-8, whose G query heads need the register room of one wave per SIMD).
// K/V rows are read once per step: non-temporal loads (MI355X_MICROARCH.md nt-weights row), round 3: C1
// attention 8.89 -> 8.40 us (367.5 vs 362.5 tok/s), C4 37.4 -> 35.4 us (1737 vs 1720 tok/s); variant A/B in
// profiles/r3_attn_nt_ab.txt. SLI_ATTN_NT=0: default cache policy.
#ifndef SLI_ATTN_NT
#define SLI_ATTN_NT 1
#endif
#ifndef SLI_ATTN_SLOTS
#define SLI_ATTN_SLOTS 64
#endif
constexpr int kAttnSlots = SLI_ATTN_SLOTS;
constexpr int kAttnMaxWgSplits = 128;  // combine-kernel capacity

template <typename KT, int HD>
struct AttnGeom {
    static constexpr int EPV = Vec16<KT>::N;
    static constexpr int LPR = HD / EPV;     // lanes per cached row
    static constexpr int RPI = 64 / LPR;     // rows per wave-instruction
    static constexpr int PPWG = kAttnSlots * RPI;  // positions per workgroup (context split)
    static_assert(LPR >= 1 && LPR <= 64 && (64 % LPR) == 0, "head_dim / vector shape");
};

// tools/attn_lab (profiles/r03_attn_lab.txt): MHA / GQA-2 16 waves, GQA-4 8, GQA-8 4; V loaded after the
// scores (K and V never live together) for GQA-2 and GQA-4. MHA (57 VGPRs either way) issues K and V
// together: C1 attention 9.17 -> 8.92 us in the step (round 2, tools/ab_variants.sh).
// A/B knobs (variant builds, tools/ab_variants.sh); the defaults are the measured best.
#ifndef SLI_ATTN_WAVES_MHA
#define SLI_ATTN_WAVES_MHA 16
#endif
#ifndef SLI_ATTN_LATE_V_MHA
#define SLI_ATTN_LATE_V_MHA 0
#endif
__host__ __device__ constexpr int attn_waves(int g) { return g == 1 ? SLI_ATTN_WAVES_MHA : g <= 2 ? 16 : g == 4 ? 8 : 4; }
__host__ __device__ constexpr bool attn_late_v(int g) { return g == 1 ? SLI_ATTN_LATE_V_MHA != 0 : g <= 4; }

// grid: n_kv_heads * wg_splits workgroups; wave w of workgroup (kvh, s) owns the w-th slice of split s.
// The WAVES slice states are merged in LDS, so one partial per (q head, workgroup) reaches the workspace.
// The split work of workgroup (kvh, wgs): partial state published write-through, arrival counted.
// Returns true in the head's last-arriving workgroup (which must then merge the head: attn_merge).
// Every return is uniform over the workgroup.
template <typename KT, int HD, int G, int WAVES = attn_waves(G), bool LATE_V = attn_late_v(G), bool HAND = false>
__device__ __forceinline__ bool attn_publish(const AttnArgs<KT>& a, int kvh, int wgs) {
    using Geo = AttnGeom<KT, HD>;
    constexpr int kAttnNit = kAttnSlots / WAVES;
    constexpr int EPV = Geo::EPV, LPR = Geo::LPR, RPI = Geo::RPI, PPW = kAttnNit * RPI;
    __shared__ float sh[WAVES][G][HD + 2];
    __shared__ int last;
    __shared__ float hs[HAND ? (G + 2) * HD : 1];  // HAND: q (G heads), then this step's k and v rows
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int pos = attn_pos(a, kvh);
    if (wgs * WAVES * PPW > pos) return false;  // whole workgroup past the live context (uniform exit)
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
    if (HAND || live_wave) {  // HAND: every wave (the workgroup barrier below); a dead wave's state is reset after
        const int ch = a.cache_heads > 0 ? kvh % a.cache_heads : kvh / a.kv_group;
        const KT* kb = a.k + (long long)ch * a.head_stride + li * EPV;
        const KT* vb = a.v + (long long)ch * a.head_stride + li * EPV;
        u32x4 kr[kAttnNit], vr[kAttnNit];
#pragma unroll
        for (int it = 0; it < kAttnNit; ++it) {
            const int t = min(t0 + it * RPI + sub, t_end - 1);  // clamp, never branch around a load
            kr[it] = load16<SLI_ATTN_NT != 0>(kb + (long long)t * a.pos_stride);
        }
        auto load_v = [&]() {
#pragma unroll
            for (int it = 0; it < kAttnNit; ++it) {
                const int t = min(t0 + it * RPI + sub, t_end - 1);
                vr[it] = load16<SLI_ATTN_NT != 0>(vb + (long long)t * a.pos_stride);
            }
        };
        // LATE_V: V is loaded once the scores are done, so K and V never occupy registers together
        // (GQA-4/8 carry G query heads per lane: fewer registers = more resident workgroups)
        if constexpr (!LATE_V) load_v();
        // HAND: the rows below pos (earlier launches) are in flight. Wave 0 waits for the kv head's q / k / v units
        // and stages q and this step's K/V rows (sc1, one batch) into LDS for the workgroup; the row at pos then
        // replaces the (stale) cache row the clamped loads fetched. (One reader per workgroup: sc1 reads of the same
        // lines by every wave, and every wave polling, measured 16.6 -> 23 us per TP-8 launch.)
        auto hand_row = [&](u32x4(&r)[kAttnNit], const float* f) {
#pragma unroll
            for (int it = 0; it < kAttnNit; ++it) {
                if (min(t0 + it * RPI + sub, t_end - 1) == pos) {
                    float x[EPV];
#pragma unroll
                    for (int e = 0; e < EPV; ++e) x[e] = f[li * EPV + e];
                    r[it] = Vec16<KT>::pack(x);
                }
            }
        };
        if constexpr (HAND) {
            if (wave == 0) {
                attn_hand_wait(a, kvh);
                constexpr int NQ = G * HD, NJ = (G + 2) * HD / 64;
                float x[NJ];
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    const int i = j * 64 + lane;
                    const float* src = i < NQ        ? a.q + (size_t)kvh * NQ + i
                                       : i < NQ + HD ? a.hand_kv + (size_t)kvh * HD + (i - NQ)
                                                     : a.hand_kv + ((size_t)a.n_kv_heads + kvh) * HD + (i - NQ - HD);
                    x[j] = attn_hand_ld(src);
                }
#pragma unroll
                for (int j = 0; j < NJ; ++j) hs[j * 64 + lane] = x[j];
            }
            __syncthreads();
        }
        float qv[G][EPV];
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int e = 0; e < EPV; ++e)
                qv[g][e] = HAND ? hs[g * HD + li * EPV + e] : a.q[(size_t)(kvh * G + g) * HD + li * EPV + e];
        if constexpr (HAND) {
            hand_row(kr, hs + G * HD);
            if constexpr (!LATE_V) hand_row(vr, hs + (G + 1) * HD);
        }
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
        if constexpr (LATE_V) {
            load_v();
            if constexpr (HAND) hand_row(vr, hs + (G + 1) * HD);
        }
#pragma unroll
        for (int g = 0; g < G; ++g)
            m[g] = stride_max<LPR>(m[g]);
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
            l[g] = stride_sum<LPR>(l[g]);
#pragma unroll
            for (int e = 0; e < EPV; ++e) ov[g][e] = stride_sum<LPR>(ov[g][e]);
        }
        if (HAND && !live_wave) {  // (its rows were all masked: the empty state, as a dead wave's)
#pragma unroll
            for (int g = 0; g < G; ++g) {
                m[g] = -INFINITY;
                l[g] = 0.0f;
#pragma unroll
                for (int e = 0; e < EPV; ++e) ov[g][e] = 0.0f;
            }
        }
    }
    if (a.stamps && threadIdx.x == 0) a.stamps[blockIdx.x * 4 + 1] = __builtin_amdgcn_s_memrealtime();
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
    if constexpr (HAND) {  // every wave of the workgroup is past its wait: the head's last live workgroup resets
        if (threadIdx.x < 64) {
            const int ns = min(pos / (WAVES * PPW) + 1, a.max_splits);
            unsigned* done = attn_hand_done(a.hand_count, a.n_kv_heads, kvh);
            unsigned prev = 0;
            if (threadIdx.x == 0) prev = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (__builtin_amdgcn_readfirstlane(prev) == (unsigned)(ns - 1)) {
                if (threadIdx.x < kAttnHandSub)
                    __hip_atomic_store(attn_hand_sub(a.hand_count, kvh, threadIdx.x), 0u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                if (threadIdx.x == 0) __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    if (a.defer_merge) {  // partials for the next launch (the kernel boundary publishes them): plain stores
        for (int i = threadIdx.x; i < G * HD; i += 64 * WAVES) {
            const int g = i / HD, d = i - g * HD;
            float M = -INFINITY;
#pragma unroll
            for (int w = 0; w < WAVES; ++w) M = fmaxf(M, sh[w][g][HD]);
            float o = 0.0f, L = 0.0f;
#pragma unroll
            for (int w = 0; w < WAVES; ++w) {
                const float c = expf(sh[w][g][HD] - M);
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
        return false;
    }
    // Workgroup partial: the WAVES slice states merged in LDS, published write-through (sc1) so the
    // head's last-arriving workgroup can read it from any XCD without a fence pair
    // (MI355X_MICROARCH.md, hand-off table row 1: sc1 stores, drained, one agent-scope add per
    // workgroup behind a workgroup barrier, sc1 loads by the last adder after the barrier it joins).
    for (int i = threadIdx.x; i < G * HD; i += 64 * WAVES) {
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
    const int ns = min(pos / (WAVES * PPW) + 1, a.max_splits);  // live workgroups of this kv head
    if (threadIdx.x == 0) {
        const unsigned prev = __hip_atomic_fetch_add(a.counters + kvh, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = prev == (unsigned)(ns - 1);
        if (last) __hip_atomic_store(a.counters + kvh, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (a.stamps && threadIdx.x == 0) a.stamps[blockIdx.x * 4 + 2] = __builtin_amdgcn_s_memrealtime();
    return last != 0;
}

// sc1 (L2-coherent across XCDs, L1 bypassed) 4-byte load, counted by the compiler like any other load.
__device__ __forceinline__ float load_sc1(const float* base, unsigned bytes, unsigned off) {
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, bytes, 0x00020000);
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, off, 0, 16 /* sc1 */));
}

// Merge kv head kvh's ns live split partials into out (sc1 stores), by threads [t0, t0 + nthr) of the
// workgroup, one output (q head g, dim d) per thread per pass, in split order whatever the arrival
// order: M = max m_i, w_i = e^{m_i - M}, out = (sum_i w_i o_i) / (sum_i w_i l_i). Up to NS splits every
// load of a thread (its head's NS (m, l) pairs, its NS partial values) is issued in ONE batch: one
// round trip to the write-through copies; more splits take two passes in batches of NS. Ends with
// the storing threads drained; no barrier.
template <int HD, int G, int NS = 16>
__device__ __forceinline__ void attn_merge(const float* part, float* out, int kvh, int max_splits, int ns, int t0,
                                           int nthr) {
    constexpr int PS = HD + kAttnPartPad;
    const unsigned bytes = (unsigned)(sizeof(float) * (size_t)G * max_splits * PS);
    const float* base = part + (size_t)kvh * G * max_splits * PS;
    for (int i = (int)threadIdx.x - t0; i >= 0 && i < G * HD; i += nthr) {
        const int g = i / HD, d = i - g * HD;
        const unsigned row0 = (unsigned)(g * max_splits) * PS;
        float M = -INFINITY;
        if (ns > NS) {  // first pass: the max alone
            for (int s0 = 0; s0 < ns; s0 += NS) {
                float mv[NS];
#pragma unroll
                for (int j = 0; j < NS; ++j)
                    mv[j] = load_sc1(base, bytes, 4u * (row0 + (unsigned)min(s0 + j, ns - 1) * PS + HD));
#pragma unroll
                for (int j = 0; j < NS; ++j) M = fmaxf(M, mv[j]);
            }
        }
        float o = 0.0f, L = 0.0f;
        for (int s0 = 0; s0 < ns; s0 += NS) {
            float mv[NS], lv[NS], ov[NS];
#pragma unroll
            for (int j = 0; j < NS; ++j) {
                const unsigned r = row0 + (unsigned)min(s0 + j, ns - 1) * PS;
                mv[j] = load_sc1(base, bytes, 4u * (r + HD));
                lv[j] = load_sc1(base, bytes, 4u * (r + HD + 1));
                ov[j] = load_sc1(base, bytes, 4u * (r + d));
            }
            if (ns <= NS) {
#pragma unroll
                for (int j = 0; j < NS; ++j) M = fmaxf(M, mv[j]);  // clamped duplicates leave the max
            }
#pragma unroll
            for (int j = 0; j < NS; ++j) {
                if (s0 + j < ns) {
                    const float w = expf(mv[j] - M);
                    o = fmaf(w, ov[j], o);
                    L = fmaf(w, lv[j], L);
                }
            }
        }
        __hip_atomic_store(out + (size_t)(kvh * G + g) * HD + d, o / L, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Live split count of a kv head at position pos (workgroups that run attn_publish to the end).
template <typename KT, int HD, int G>
__device__ __forceinline__ int attn_live_splits(const AttnArgs<KT>& a, int kvh) {
    const int ppwg = a.ppwg > 0 ? a.ppwg : AttnGeom<KT, HD>::PPWG;
    return min(attn_pos(a, kvh) / ppwg + 1, a.max_splits);
}

// grid: n_kv_heads * wg_splits workgroups of 64 * WAVES threads
template <typename KT, int HD, int G, int WAVES = attn_waves(G), bool LATE_V = attn_late_v(G)>
// Stagger (C4: 1024 workgroups, two per CU, two residency rounds): each round is a K burst, the scores, a V burst
// and the merge, with HBM idle between the bursts. Workgroups 256..511 (the second of each CU in the first
// round, under the dispatcher's order) start SLI_ATTN_STAGGER x 0.85 us later, so their K burst overlaps the
// first workgroup's scores; later rounds stagger by themselves. Measured at C4 (profiles/r4_attn_stagger_ab.txt):
// 0 / 1.7 / 3.4 / 6.8 / 13.6 us = attention 34.95 / 34.24 / 34.18 / 35.09 / 44.56 us. 0: off.
#ifndef SLI_ATTN_STAGGER
#define SLI_ATTN_STAGGER 4
#endif
__global__ void __launch_bounds__(64 * WAVES) attn_partial_kernel(AttnArgs<KT> a) {
    if (a.stamps && threadIdx.x == 0) a.stamps[blockIdx.x * 4] = __builtin_amdgcn_s_memrealtime();
#if SLI_ATTN_STAGGER
    if (G == 4 && gridDim.x >= 1024 && blockIdx.x >= 256 && blockIdx.x < 512)
        for (int i = 0; i < SLI_ATTN_STAGGER; ++i) __builtin_amdgcn_s_sleep(32);
#endif
    const int kvh = blockIdx.x / a.max_splits;  // max_splits counts workgroup splits here
    if (attn_publish<KT, HD, G, WAVES, LATE_V>(a, kvh, blockIdx.x - kvh * a.max_splits)) {
        attn_merge<HD, G>(a.part, a.out, kvh, a.max_splits, attn_live_splits<KT, HD, G>(a, kvh), 0, 64 * WAVES);
        if (a.stamps && threadIdx.x == 0) a.stamps[blockIdx.x * 4 + 3] = __builtin_amdgcn_s_memrealtime();
    }
}

// The split merge as its own launch after an attention launch with defer_merge (batched decode: the
// consumer is the MFMA projection, whose every workgroup stages the whole activation, so merging in its
// staging would re-read the partials once per workgroup). Freed of the merge, the attention workgroups
// end right after their partial store: at C4 the 1024 workgroups run in two residency rounds, and the
// first round's slots free sooner. grid: n_kv_heads * attn_merge_wgs(G * HD) workgroups of
// kAttnMergeThreads: every thread merges ONE output (q head g, dim d), so the launch is one round trip to
// the partials (C4: two passes of 256 threads per kv head took 5.9 us).
constexpr int kAttnMergeThreads = 256;
__host__ __device__ constexpr int attn_merge_wgs(int outputs) {
    return (outputs + kAttnMergeThreads - 1) / kAttnMergeThreads;
}
template <typename KT, int HD, int G>
__global__ void __launch_bounds__(kAttnMergeThreads) attn_merge_kernel(AttnArgs<KT> a) {
    constexpr int MS = attn_merge_wgs(G * HD);
    const int kvh = blockIdx.x / MS, j = blockIdx.x - kvh * MS;
    attn_merge<HD, G>(a.part, a.out, kvh, a.max_splits, attn_live_splits<KT, HD, G>(a, kvh), -j * kAttnMergeThreads,
                      MS * kAttnMergeThreads);
}

}  // namespace sli
