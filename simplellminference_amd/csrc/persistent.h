// persistent.h — the whole decode step (or a phase range of it, under tensor parallelism) as ONE
// persistent launch: one 1024-thread workgroup per CU walks the phases
//     per layer: QKV (RMSNorm ⊕ [wq;wk;wv] ⊕ RoPE ⊕ K/V write) | ATTN (split-context partials) |
//                WO (split combine ⊕ wo ⊕ residual) | GU (RMSNorm ⊕ [gate;up] ⊕ SwiGLU) | DOWN (down ⊕ residual)
//     then LM (RMSNorm ⊕ tied head ⊕ argmax keys) and, when the range ends the step, key reduce + finalize,
// separated by a grid barrier. Before arriving at a barrier every wave issues the first weight chunk of
// its next GEMV phase (the weights never depend on activations), so the HBM stream keeps running
// through the barrier and the next phase's x staging (MI355X_MICROARCH.md price list: prefetch-credit).
//
// Hand-off protocol (cdna_hip_programming.md §6 Guideline 16, "Valid forms"): every storing wave drains
// (s_waitcnt vmcnt(0)), workgroup barrier, ONE lane agent-release, arrive on an XCD-group counter (the
// last arriver of a group bumps the top counter, the last group publishes the generation), relaxed poll
// of the generation, ONE agent-acquire, workgroup barrier, then plain loads. Counters are monotonic
// within a launch (epoch = barrier index + 1) and zeroed by a memset node before every launch; every
// spin is bounded and sets DevState::error on timeout.
#pragma once
#include "attention.h"
#include "gemv.h"

namespace sli {

struct DevState {
    int32_t pos;          // position of the token being fed
    int32_t token;        // token fed at pos
    int32_t n_forced;     // prompt length (teacher forcing while pos < n_forced)
    int32_t last_argmax;  // greedy argmax of the last step's logits
    int32_t advance;      // 1: finalize advances pos/token; 0: idempotent step (bench)
    int32_t error;        // bit 2: a grid barrier timed out
    unsigned long long key;  // argmax key of the last step (0 between steps)
};

// model.cpp:157-183: next position; teacher-forced prompt token while inside the prompt, else greedy.
__device__ __forceinline__ void finalize_state(DevState* st, const int32_t* prompt, int32_t* hist, int T) {
    const unsigned long long k = st->key;
    const int next = (int)argmax_key_index(k);
    st->last_argmax = next;
    st->key = 0;
    if (st->advance) {
        const int p = st->pos + 1;
        if (p < T) {
            st->pos = p;
            st->token = p < st->n_forced ? prompt[p] : next;
            hist[p] = st->token;
        }
    }
}

struct LayerPtrs {
    const void* qkv;
    const float* qkv_s;
    const void* wo;
    const float* wo_s;
    const void* gu;
    const float* gu_s;
    const void* down;
    const float* down_s;
};

struct StepParams {
    int D, L, T, hd, hq, hkv, Il, v_lo, v_n, V;
    int silu, partial, rank;
    float eps;
    const void* emb;
    const float* emb_s;
    const float* norms;
    const LayerPtrs* layers;  // device array [L]
    void* kc;
    void* vc;
    float *x, *xpart, *q, *act, *logits, *part;
    const float* sin_t;
    const float* cos_t;
    unsigned long long* keys;
    DevState* st;
    const int32_t* prompt;
    int32_t* hist;
    unsigned* bar;    // barrier words: 8 group counters, top counter, generation (128 B apart)
    int attn_splits;  // workgroup-level context splits per kv head (workspace capacity)
    int debug_flags;             // diagnostic (SLI_DEBUG_BARRIER): 1 no release, 2 no acquire, 4 no barrier
    unsigned long long* stamps;  // diagnostic (nullable): workgroup 0's s_memrealtime at phase start /
                                 // barrier arrival, 3 per phase (SLI_DEBUG_STAMPS=1)
};

constexpr int kPhasesPerLayer = 5;
enum { kPhQKV = 0, kPhATTN = 1, kPhWO = 2, kPhGU = 3, kPhDOWN = 4 };
constexpr int kBarStride = 32;        // unsigned words between barrier counters (one 128-B line each)
constexpr int kBarWords = 10 * kBarStride;
constexpr int kPartStride = kAttnPartPad;  // partial row = hd + 4 floats (attention.h layout)
constexpr int kPR = 2, kPU = 8;       // GEMV unit rows and 16-B vectors per row in flight (main loop)
constexpr int kPF = 4;                // vectors per row prefetched across a phase barrier

// Attention-phase geometry inside the persistent kernel (VGPR budget 128 at 16 waves/CU): NIT 16-B
// vectors per lane per operand, so K+V in flight = 2*NIT*4 VGPRs.
__host__ __device__ constexpr int pattn_nit(int g) { return g >= 4 ? 4 : 8; }
__host__ __device__ constexpr int pattn_ppw_wg(int hd, int kv_elem_bytes, int g) {
    return kAttnWaves * pattn_nit(g) * (64 / (hd / (16 / kv_elem_bytes)));
}

// ---------------------------------------------------------------- grid barrier
__device__ __forceinline__ void grid_arrive_wait(unsigned* bar, unsigned epoch, DevState* st, int dbg = 0) {
    if (dbg & 4) return;
    // caller: every wave drained its stores, workgroup barrier passed, lane 0 released (agent)
    const unsigned G = gridDim.x;
    const unsigned g = blockIdx.x & 7u;
    const unsigned gsize = (G - g + 7u) / 8u;
    const unsigned ngroups = G < 8u ? G : 8u;
    const unsigned t = __hip_atomic_fetch_add(&bar[g * kBarStride], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == epoch * gsize - 1u) {
        const unsigned t2 = __hip_atomic_fetch_add(&bar[8 * kBarStride], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (t2 == epoch * ngroups - 1u) __hip_atomic_store(&bar[9 * kBarStride], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    unsigned spins = 0;
    while (__hip_atomic_load(&bar[9 * kBarStride], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < epoch) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1u << 25)) {  // ~1 s: never hang the GPU; the host sees DevState::error
            __hip_atomic_fetch_or(&st->error, 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
    }
    if (!(dbg & 2)) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

// ---------------------------------------------------------------- x staging into LDS
// RMS-normalised copy of a global fp32 vector (rms_kernel.cpp:5-23), one round trip per thread.
__device__ __forceinline__ void stage_norm(float* smem, const float* x, const float* w, float eps, int cols) {
    GemvIn in{x, w, eps, cols};
    gemv_stage_x(smem, in);
}

// Layer-0 input: x = E[token] (emb_kernel.cpp:4-21), normalised into LDS; workgroup 0 also publishes x
// (the residual stream) to global memory.
template <typename WT>
__device__ __forceinline__ void stage_embed_norm(float* smem, const StepParams& P) {
    float* red = smem;
    float* xs = smem + kGemvLdsHead;
    const int tid = threadIdx.x, nt = blockDim.x, D = P.D;
    const int tok = P.st->token;
    const bool ok = tok >= 0 && tok < P.V;
    const float s = (ok && P.emb_s) ? P.emb_s[tok] : 1.0f;
    const WT* row = reinterpret_cast<const WT*>(P.emb) + (size_t)(ok ? tok : 0) * D;
    float ss = 0.0f;
    for (int c = tid; c < D; c += nt) {
        const float v = ok ? to_f32(row[c]) * s : 0.0f;
        xs[c] = v;
        ss += v * v;
        if (blockIdx.x == 0) P.x[c] = v;
    }
    ss = wave_sum(ss);
    if ((tid & 63) == 0) red[tid >> 6] = ss;
    __syncthreads();
    if (tid == 0) {
        float t = 0.0f;
        for (int w = 0; w < (nt >> 6); ++w) t += red[w];
        red[32] = 1.0f / sqrtf(t / (float)D + P.eps);
    }
    __syncthreads();
    const float inv = red[32];
    const float* nw = P.norms;  // attention norm of layer 0
    for (int c = tid; c < D; c += nt) xs[c] = (xs[c] * inv) * nw[c];
}

__device__ __forceinline__ void stage_plain(float* smem, const float* src, int cols) {
    GemvIn in{src, nullptr, 0.0f, cols};
    gemv_stage_x(smem, in);
}

// Split-context combine of every local head into LDS (the WO input): thread t owns dims [4t, 4t+4).
__device__ __forceinline__ void stage_combine(float* smem, const StepParams& P, int ppw_wg) {
    float* xs = smem + kGemvLdsHead;
    const int hd = P.hd, n = P.hq * hd;
    const int pos = P.st->pos;
    const int ns = pos / ppw_wg + 1;
    const int ps = hd + kPartStride;
    for (int d0 = 4 * threadIdx.x; d0 < n; d0 += 4 * blockDim.x) {
        const int h = d0 / hd, dd = d0 - h * hd;
        const float* ph = P.part + (size_t)h * P.attn_splits * ps;
        float M = -INFINITY;
        for (int s = 0; s < ns; ++s) M = fmaxf(M, ph[(size_t)s * ps + hd]);
        float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
        float Lsum = 0.0f;
        for (int s = 0; s < ns; ++s) {
            const float* p = ph + (size_t)s * ps;
            const float c = expf(p[hd] - M);
            const float4 v = *reinterpret_cast<const float4*>(p + dd);
            o.x = fmaf(c, v.x, o.x);
            o.y = fmaf(c, v.y, o.y);
            o.z = fmaf(c, v.z, o.z);
            o.w = fmaf(c, v.w, o.w);
            Lsum = fmaf(c, p[hd + 1], Lsum);
        }
        const float r = 1.0f / Lsum;
        *reinterpret_cast<float4*>(xs + d0) = make_float4(o.x * r, o.y * r, o.z * r, o.w * r);
    }
}

// ---------------------------------------------------------------- GEMV phase (balanced static schedule)
__device__ __forceinline__ void wave_units(int nunits, int& u_begin, int& u_end) {
    const long long gw = (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const long long nw = (long long)gridDim.x * (blockDim.x >> 6);
    u_begin = (int)(gw * nunits / nw);
    u_end = (int)((gw + 1) * nunits / nw);
}

template <typename WT, class Epi>
__device__ __forceinline__ bool gemv_prefetch(const WT* W, int cols, const Epi& epi, u32x4 (&pre)[kPF][kPR]) {
    constexpr int EPV = Vec16<WT>::N;
    const int lane = threadIdx.x & 63;
    const int nvec = cols / EPV;
    int u0, u1;
    wave_units(epi.units(), u0, u1);
    if (!(u0 < u1 && lane + (kPF - 1) * 64 < nvec)) return false;
    int rows[kPR];
    epi.rows(u0, rows);
    const size_t row_bytes = (size_t)cols * sizeof(WT);
#pragma unroll
    for (int j = 0; j < kPF; ++j)
#pragma unroll
        for (int r = 0; r < kPR; ++r)
            pre[j][r] = load16<true>(reinterpret_cast<const char*>(W) + (size_t)rows[r] * row_bytes +
                                     (size_t)(lane + j * 64) * 16);
    return true;
}

template <typename WT, class Epi>
__device__ __forceinline__ void gemv_run(const WT* W, const float* xs, int cols, Epi& epi,
                                         const u32x4 (&pre)[kPF][kPR], bool have_pre) {
    constexpr int EPV = Vec16<WT>::N, R = kPR, U = kPU;
    const int lane = threadIdx.x & 63;
    const int nvec = cols / EPV;
    const size_t row_bytes = (size_t)cols * sizeof(WT);
    int u_begin, u_end;
    wave_units(epi.units(), u_begin, u_end);
    float acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = 0.0f;
    if (have_pre) gemv_chunk<WT, R, kPF>(pre, xs, lane, acc);
    for (int u = u_begin; u < u_end; ++u) {
        int rows[R];
        epi.rows(u, rows);
        const char* wp[R];
#pragma unroll
        for (int r = 0; r < R; ++r) wp[r] = reinterpret_cast<const char*>(W) + (size_t)rows[r] * row_bytes;
        int v = (u == u_begin && have_pre) ? lane + kPF * 64 : lane;
        for (; v + (U - 1) * 64 < nvec; v += U * 64) {
            u32x4 w[U][R];
#pragma unroll
            for (int j = 0; j < U; ++j)
#pragma unroll
                for (int r = 0; r < R; ++r) w[j][r] = load16<true>(wp[r] + (size_t)(v + j * 64) * 16);
            gemv_chunk<WT, R, U>(w, xs, v, acc);
        }
        if (v < nvec) {
            u32x4 w[U][R];
#pragma unroll
            for (int j = 0; j < U; ++j) {
                const int vj = min(v + j * 64, nvec - 1);
#pragma unroll
                for (int r = 0; r < R; ++r) w[j][r] = load16<true>(wp[r] + (size_t)vj * 16);
            }
            gemv_chunk<WT, R, U, true>(w, xs, v, acc, nvec);
        }
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = wave_sum(acc[r]);
        epi.store(u, rows, acc, lane);
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = 0.0f;
    }
}

// ---------------------------------------------------------------- attention phase
// Work item = (kv head, workgroup split): 4 waves (a "group"), wave w owns context slice 4s + w, the 4
// slice states merge in this group's LDS region. Every group of a workgroup runs the same number of
// item rounds so the workgroup barriers inside line up.
template <typename KT, int HD, int G>
__device__ __forceinline__ void attn_phase(float* smem, const StepParams& P, int layer) {
    using Geo = AttnGeom<KT, HD>;
    constexpr int EPV = Geo::EPV, LPR = Geo::LPR, RPI = Geo::RPI;
    constexpr int NIT = pattn_nit(G), PPW = NIT * RPI;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int grp = wave >> 2, wig = wave & 3;          // group of 4 waves, wave in group
    const int ngrp = blockDim.x >> 8;
    float* sh = smem + (size_t)grp * kAttnWaves * G * (HD + 2);  // [4][G][HD+2] per group
    const int pos = P.st->pos;
    const int wg_live = pos / (kAttnWaves * PPW) + 1;
    const int n_items = P.hkv * wg_live;
    const int slots = gridDim.x * ngrp;
    const int rounds = (n_items + slots - 1) / slots;
    const long long hs = (long long)P.T * HD;  // head stride of the head-major cache
    const KT* kl = reinterpret_cast<const KT*>(P.kc) + (size_t)layer * P.hkv * hs;
    const KT* vl = reinterpret_cast<const KT*>(P.vc) + (size_t)layer * P.hkv * hs;
    const float scale = 1.0f / sqrtf((float)HD);
    const int sub = lane / LPR, li = lane - (lane / LPR) * LPR;
    for (int rd = 0; rd < rounds; ++rd) {
        const int item = rd * slots + grp * gridDim.x + blockIdx.x;  // spread items over all CUs first
        const bool have = item < n_items;
        const int kvh = have ? item / wg_live : 0;
        const int wgs = have ? item - kvh * wg_live : 0;
        const int t0 = (wgs * kAttnWaves + wig) * PPW;
        const bool live_wave = have && t0 <= pos;
        const int t_end = min(t0 + PPW, pos + 1);
        float m[G], l[G], ov[G][EPV];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            m[g] = -INFINITY;
            l[g] = 0.0f;
#pragma unroll
            for (int e = 0; e < EPV; ++e) ov[g][e] = 0.0f;
        }
        if (live_wave) {
            const KT* kb = kl + (long long)kvh * hs + li * EPV;
            const KT* vb = vl + (long long)kvh * hs + li * EPV;
            u32x4 kr[NIT], vr[NIT];
#pragma unroll
            for (int it = 0; it < NIT; ++it) {
                const int t = min(t0 + it * RPI + sub, t_end - 1);
                kr[it] = load16<false>(kb + (long long)t * HD);
            }
#pragma unroll
            for (int it = 0; it < NIT; ++it) {
                const int t = min(t0 + it * RPI + sub, t_end - 1);
                vr[it] = load16<false>(vb + (long long)t * HD);
            }
            float qv[G][EPV];
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int e = 0; e < EPV; ++e) qv[g][e] = P.q[(size_t)(kvh * G + g) * HD + li * EPV + e];
            float s[NIT][G];
#pragma unroll
            for (int it = 0; it < NIT; ++it) {
                float kf[EPV];
                Vec16<KT>::unpack(kr[it], kf);
                const bool live = (t0 + it * RPI + sub) < t_end;
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    float d = 0.0f;
#pragma unroll
                    for (int e = 0; e < EPV; ++e) d = fmaf(qv[g][e], kf[e], d);
                    d = group_sum<LPR>(d);
                    s[it][g] = live ? d * scale : -INFINITY;
                    m[g] = fmaxf(m[g], s[it][g]);
                }
            }
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int o = LPR; o < 64; o <<= 1) m[g] = fmaxf(m[g], __shfl_xor(m[g], o, kWave));
#pragma unroll
            for (int it = 0; it < NIT; ++it) {
                float vf[EPV];
                Vec16<KT>::unpack(vr[it], vf);
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    const float p = expf(s[it][g] - m[g]);
                    l[g] += p;
#pragma unroll
                    for (int e = 0; e < EPV; ++e) ov[g][e] = fmaf(p, vf[e], ov[g][e]);
                }
            }
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
                float* row = sh + ((size_t)wig * G + g) * (HD + 2);
#pragma unroll
                for (int e = 0; e < EPV; ++e) row[li * EPV + e] = ov[g][e];
                if (li == 0) {
                    row[HD] = m[g];
                    row[HD + 1] = l[g];
                }
            }
        }
        __syncthreads();
        if (have) {
            for (int i = threadIdx.x - grp * 256; i < G * HD; i += 256) {
                const int g = i / HD, d = i - g * HD;
                float M = -INFINITY;
#pragma unroll
                for (int w = 0; w < kAttnWaves; ++w) M = fmaxf(M, sh[((size_t)w * G + g) * (HD + 2) + HD]);
                float o = 0.0f, Ls = 0.0f;
#pragma unroll
                for (int w = 0; w < kAttnWaves; ++w) {
                    const float* row = sh + ((size_t)w * G + g) * (HD + 2);
                    const float c = expf(row[HD] - M);
                    o = fmaf(c, row[d], o);
                    Ls = fmaf(c, row[HD + 1], Ls);
                }
                float* dst = P.part + ((size_t)(kvh * G + g) * P.attn_splits + wgs) * (HD + kPartStride);
                dst[d] = o;
                if (d == 0) {
                    dst[HD] = M;
                    dst[HD + 1] = Ls;
                }
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------- epilogue factories
template <typename KT>
__device__ __forceinline__ EpiQKV<KT> make_qkv(const StepParams& P, int l) {
    KT* kc = reinterpret_cast<KT*>(P.kc) + (size_t)l * P.hkv * P.T * P.hd;
    KT* vc = reinterpret_cast<KT*>(P.vc) + (size_t)l * P.hkv * P.T * P.hd;
    return EpiQKV<KT>{P.q, kc, vc, P.layers[l].qkv_s, &P.st->pos, P.sin_t, P.cos_t, P.hq, P.hkv, P.hd, P.T};
}
__device__ __forceinline__ EpiStore<kPR> make_wo(const StepParams& P, int l) {
    return EpiStore<kPR>{P.partial ? P.xpart : P.x, (!P.partial || P.rank == 0) ? P.x : nullptr, P.layers[l].wo_s,
                         1.0f, P.D};
}
__device__ __forceinline__ EpiSwiGLU make_gu(const StepParams& P, int l) {
    return EpiSwiGLU{P.act, P.layers[l].gu_s, P.Il, P.silu};
}
__device__ __forceinline__ EpiStore<kPR> make_down(const StepParams& P, int l) {
    return EpiStore<kPR>{P.partial ? P.xpart : P.x, (!P.partial || P.rank == 0) ? P.x : nullptr, P.layers[l].down_s,
                         1.0f, P.D};
}
__device__ __forceinline__ EpiLogits<kPR> make_lm(const StepParams& P) {
    return EpiLogits<kPR>{P.logits, P.keys, P.emb_s ? P.emb_s + P.v_lo : nullptr, P.v_n, P.v_lo, 0ull};
}

// Issue the first weight chunk of phase p (GEMV phases only). When nothing is prefetched the registers
// are zeroed so their old contents are dead (keeps them out of the attention phase's register budget).
template <typename WT, typename KT>
__device__ __forceinline__ bool prefetch_phase(const StepParams& P, int p, u32x4 (&pre)[kPF][kPR]) {
    const int l = p / kPhasesPerLayer, k = p - l * kPhasesPerLayer;
    bool ok = false;
    if (l >= P.L) {
        const WT* w = reinterpret_cast<const WT*>(P.emb) + (size_t)P.v_lo * P.D;
        ok = gemv_prefetch<WT>(w, P.D, make_lm(P), pre);
    } else {
        const LayerPtrs& L = P.layers[l];
        switch (k) {
            case kPhQKV: ok = gemv_prefetch<WT>((const WT*)L.qkv, P.D, make_qkv<KT>(P, l), pre); break;
            case kPhWO: ok = gemv_prefetch<WT>((const WT*)L.wo, P.hq * P.hd, make_wo(P, l), pre); break;
            case kPhGU: ok = gemv_prefetch<WT>((const WT*)L.gu, P.D, make_gu(P, l), pre); break;
            case kPhDOWN: ok = gemv_prefetch<WT>((const WT*)L.down, P.Il, make_down(P, l), pre); break;
            default: break;
        }
    }
    if (!ok) {
#pragma unroll
        for (int j = 0; j < kPF; ++j)
#pragma unroll
            for (int r = 0; r < kPR; ++r) pre[j][r] = u32x4{0u, 0u, 0u, 0u};
    }
    return ok;
}

template <typename WT, typename KT, int HD, int G>
__global__ void __launch_bounds__(1024) step_kernel(const StepParams* __restrict__ Pp, int p_begin, int p_end,
                                                   int finalize) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const StepParams& P = *Pp;
    const float* xs = smem + kGemvLdsHead;
    constexpr int PPW_WG = pattn_ppw_wg(HD, (int)sizeof(KT), G);
    const int p_last = P.L * kPhasesPerLayer;  // the LM-head phase
    unsigned epoch = 0;
    u32x4 pre[kPF][kPR];
    bool have_pre = prefetch_phase<WT, KT>(P, p_begin, pre);
    const bool stamp = P.stamps != nullptr && blockIdx.x == 0 && threadIdx.x == 0;
    for (int p = p_begin; p < p_end; ++p) {
        const int l = p / kPhasesPerLayer, k = p - l * kPhasesPerLayer;
        if (stamp) P.stamps[3 * p] = __builtin_amdgcn_s_memrealtime();
        if (p == p_last) {
            stage_norm(smem, P.x, P.norms + (size_t)(2 * P.L) * P.D, P.eps, P.D);
            __syncthreads();
            EpiLogits<kPR> e = make_lm(P);
            gemv_run<WT>(reinterpret_cast<const WT*>(P.emb) + (size_t)P.v_lo * P.D, xs, P.D, e, pre, have_pre);
            e.finish(smem);
        } else if (k == kPhQKV) {
            if (l == 0)
                stage_embed_norm<WT>(smem, P);
            else
                stage_norm(smem, P.x, P.norms + (size_t)(2 * l) * P.D, P.eps, P.D);
            __syncthreads();
            EpiQKV<KT> e = make_qkv<KT>(P, l);
            gemv_run<WT>((const WT*)P.layers[l].qkv, xs, P.D, e, pre, have_pre);
        } else if (k == kPhATTN) {
            attn_phase<KT, HD, G>(smem, P, l);
        } else if (k == kPhWO) {
            stage_combine(smem, P, PPW_WG);
            __syncthreads();
            EpiStore<kPR> e = make_wo(P, l);
            gemv_run<WT>((const WT*)P.layers[l].wo, xs, P.hq * P.hd, e, pre, have_pre);
        } else if (k == kPhGU) {
            stage_norm(smem, P.x, P.norms + (size_t)(2 * l + 1) * P.D, P.eps, P.D);
            __syncthreads();
            EpiSwiGLU e = make_gu(P, l);
            gemv_run<WT>((const WT*)P.layers[l].gu, xs, P.D, e, pre, have_pre);
        } else {
            stage_plain(smem, P.act, P.Il);
            __syncthreads();
            EpiStore<kPR> e = make_down(P, l);
            gemv_run<WT>((const WT*)P.layers[l].down, xs, P.Il, e, pre, have_pre);
        }
        const bool last = p + 1 == p_end;
        if (last && !(finalize && p == p_last)) break;  // the launch boundary orders the rest
        // ---- phase boundary: drain, release, prefetch the next phase's weights, grid barrier
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0 && !(P.debug_flags & 1)) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        have_pre = last ? false : prefetch_phase<WT, KT>(P, p + 1, pre);
        if (stamp) P.stamps[3 * p + 1] = __builtin_amdgcn_s_memrealtime();
        if (threadIdx.x == 0) grid_arrive_wait(P.bar, ++epoch, P.st, P.debug_flags);
        if (stamp) P.stamps[3 * p + 2] = __builtin_amdgcn_s_memrealtime();
        __syncthreads();
    }
    if (finalize && p_end > p_last && blockIdx.x == 0) {  // key reduce + finalize (model.cpp:157-183)
        unsigned long long b = 0;
        for (int i = threadIdx.x; i < (int)gridDim.x; i += blockDim.x) b = P.keys[i] > b ? P.keys[i] : b;
        b = wave_max_u64(b);
        unsigned long long* red = reinterpret_cast<unsigned long long*>(smem);
        __syncthreads();
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = b;
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int w = 0; w < (int)(blockDim.x >> 6); ++w) b = red[w] > b ? red[w] : b;
            P.st->key = b;
            finalize_state(P.st, P.prompt, P.hist, P.T);
        }
    }
}

}  // namespace sli
