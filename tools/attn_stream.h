// attn_stream.h — split-context decode attention with the K/V context streamed through an LDS ring by
// LDS-DMA (global_load_lds_dwordx4), for the engine's decode step (semantics
// mha_kernel.cpp:36-77: s_t = (q·K_t)·scale, softmax over t ≤ pos, o = Σ p_t V_t).
//
// Why: the register-staged kernel (attention.h) holds its in-flight K and V in VGPRs, so a workgroup's
// bytes in flight are bounded by its registers: K first, then V after the scores (two serial round
// trips per workgroup), and at GQA-4 (C4) 128 VGPRs per lane allow only half of the 1024 workgroups to
// be resident — two residency rounds. Here the bytes in flight live in LDS: a workgroup of 4 waves
// owns a contiguous range of one kv head's context and streams it in chunks of 8 KiB of K + 8 KiB of V
// through a ring of D slots, D − 1 chunks in flight while the waves compute on the oldest. Registers
// hold only q, the online-softmax state and one chunk's rows, so the grid is sized for residency
// (1 workgroup per CU with D = 8, 2 with D = 4: one round) and every workgroup keeps ≈ 100 KiB per CU
// in flight for its whole life.
//
// Per chunk and wave: RPW rows (NIT wave-instructions of RPI rows; a row is LPR lanes × 16 B), scores
// by a group sum over the row's lanes, an online-softmax update per lane (m, l, o rescaled by
// e^{m_old − m_new}), then P·V. The row groups of a wave and the 4 waves are merged at the end (the
// same max-rescaled sums as attention.h), and the workgroup's partial (o, m, l) per q head is stored
// plainly for a deferred merge (attention.h defer_merge: the wo GEMV's staging at batch 1,
// attn_merge_kernel when batched).
//
// Pipeline per chunk c (one raw barrier per chunk, never vmcnt(0) inside the loop):
//   s_waitcnt vmcnt(pieces issued after chunk c)   this wave's DMA pieces of chunk c have landed
//   s_barrier                                      every wave's pieces landed; every wave is done with c − 1
//   issue chunk c + D − 1 into slot (c − 1) % D
//   compute chunk c from slot c % D
#pragma once
#include "../simplellminference_amd/csrc/attention.h"

namespace sli {

// W waves per workgroup, each moving P 1-KiB LDS-DMA pieces of K (and P of V) per chunk: a chunk is
// W·P KiB of K rows.
template <typename KT, int HD, int W, int P>
struct AsGeom {
    static constexpr int EPV = Vec16<KT>::N;               // elements per 16-byte lane vector
    static constexpr int LPR = HD / EPV;                   // lanes per cached row
    static constexpr int RPI = 64 / LPR;                   // rows per wave-instruction
    static constexpr int ROWB = HD * (int)sizeof(KT);      // bytes per row
    static constexpr int CHUNK = W * P * 1024;             // K (and V) bytes of one chunk
    static constexpr int C = CHUNK / ROWB;                 // positions per chunk
    static constexpr int RPW = C / W;                      // rows per wave per chunk
    static constexpr int NIT = RPW / RPI;                  // wave-instructions per wave per chunk
    static_assert(NIT >= 1 && RPW % RPI == 0, "chunk geometry");
};

template <int N>
__device__ __forceinline__ void as_wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// this wave's DMA pieces of the oldest outstanding chunk landed, `later` younger chunks may stay in flight
template <int D, int PIECES>
__device__ __forceinline__ void as_wait_chunk(int later) {
    static_assert((D - 2) * PIECES <= 63, "vmcnt range");
    switch (later) {
        case 0: as_wait_vm<0>(); break;
        case 1: as_wait_vm<PIECES>(); break;
        case 2: as_wait_vm<(D >= 4 ? 2 * PIECES : 0)>(); break;
        case 3: as_wait_vm<(D >= 5 ? 3 * PIECES : 0)>(); break;
        case 4: as_wait_vm<(D >= 6 ? 4 * PIECES : 0)>(); break;
        case 5: as_wait_vm<(D >= 7 ? 5 * PIECES : 0)>(); break;
        default: as_wait_vm<(D >= 8 ? 6 * PIECES : 0)>(); break;
    }
}

// grid: n_kv_heads * max_splits workgroups of 64 * W threads; a.ppwg positions per workgroup (a
// multiple of the chunk). Requires a.defer_merge (partials only).
template <typename KT, int HD, int G, int D, int W, int DMA>
__global__ void __launch_bounds__(64 * W) attn_stream_kernel(AttnArgs<KT> a) {
    using Geo = AsGeom<KT, HD, W, DMA>;
    constexpr int EPV = Geo::EPV, LPR = Geo::LPR, RPI = Geo::RPI, ROWB = Geo::ROWB, C = Geo::C;
    constexpr int RPW = Geo::RPW, NIT = Geo::NIT;
    __shared__ __attribute__((aligned(1024))) char ring[D][2][Geo::CHUNK];
    __shared__ __attribute__((aligned(1024))) float qs[(G * HD + 255) / 256 * 256];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (a.stamps && threadIdx.x == 0) a.stamps[blockIdx.x * 4] = __builtin_amdgcn_s_memrealtime();
    const int kvh = blockIdx.x / a.max_splits;
    const int wgs = blockIdx.x - kvh * a.max_splits;
    const int pos = attn_pos(a, kvh);
    const int p0 = wgs * a.ppwg;
    if (p0 > pos) return;  // the whole range is past the live context (uniform)
    const int nch = min(a.ppwg / C, (pos - p0) / C + 1);  // live chunks
    const int ch = a.cache_heads > 0 ? kvh % a.cache_heads : kvh;
    const char* kb = reinterpret_cast<const char*>(a.k + (long long)ch * a.head_stride);
    const char* vb = reinterpret_cast<const char*>(a.v + (long long)ch * a.head_stride);
    const long long rowb = a.pos_stride * (long long)sizeof(KT);

    // chunk c's K and V rows into ring slot c % D; rows past pos are clamped to pos (masked later)
    auto issue = [&](int c) {
        char* sk = ring[c % D][0];
        char* sv = ring[c % D][1];
        const int t0 = p0 + c * C;
#pragma unroll
        for (int j = 0; j < DMA; ++j) {
            const int piece = wave * DMA + j;
            const int byte = piece * 1024 + lane * 16;
            const long long off = (long long)min(t0 + byte / ROWB, pos) * rowb + (byte % ROWB);
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(kb + off),
                                             (__attribute__((address_space(3))) void*)(sk + piece * 1024), 16, 0, 0);
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(vb + off),
                                             (__attribute__((address_space(3))) void*)(sv + piece * 1024), 16, 0, 0);
        }
    };

    // q arrives by LDS-DMA too, ahead of the chunks (wave 0): no global load into a VGPR is outstanding
    // anywhere in the pipeline, so the compiler never inserts a vmcnt(0) of its own for one, and the
    // first chunk's counted wait covers q
    constexpr int QB = G * HD * 4, QP = (QB + 1023) / 1024;
    if (wave == 0) {
        const char* qsrc = reinterpret_cast<const char*>(a.q + (size_t)kvh * G * HD);
#pragma unroll
        for (int j = 0; j < QP; ++j)
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void*)(qsrc + min(j * 1024 + lane * 16, QB - 16)),
                (__attribute__((address_space(3))) void*)(reinterpret_cast<char*>(qs) + j * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int c = 0; c < D - 1; ++c)
        if (c < nch) issue(c);
    const int sub = lane / LPR;
    const int li = lane - sub * LPR;
    float qv[G][EPV];

    float m[G], l[G], ov[G][EPV];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        m[g] = -INFINITY;
        l[g] = 0.0f;
#pragma unroll
        for (int e = 0; e < EPV; ++e) ov[g][e] = 0.0f;
    }
    for (int c = 0; c < nch; ++c) {
        as_wait_chunk<D, 2 * DMA>(min(D - 2, nch - 1 - c));
        __builtin_amdgcn_s_barrier();
        if (c == 0) {
            if (a.stamps && threadIdx.x == 0) a.stamps[blockIdx.x * 4 + 1] = __builtin_amdgcn_s_memrealtime();
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int e = 0; e < EPV; ++e) qv[g][e] = qs[g * HD + li * EPV + e];
        }
        if (c + D - 1 < nch) issue(c + D - 1);
        const char* sk = ring[c % D][0];
        const char* sv = ring[c % D][1];
        const int tc = p0 + c * C + wave * RPW + sub;  // this lane's row of instruction 0
        float s[NIT][G];
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
            const int row = wave * RPW + it * RPI + sub;
            const u32x4 kr = *reinterpret_cast<const u32x4*>(sk + row * ROWB + li * 16);
            float kf[EPV];
            Vec16<KT>::unpack(kr, kf);
            const bool live = tc + it * RPI <= pos;
#pragma unroll
            for (int g = 0; g < G; ++g) {
                float d = 0.0f;
#pragma unroll
                for (int e = 0; e < EPV; ++e) d = fmaf(qv[g][e], kf[e], d);
                d = group_sum<LPR>(d);
                s[it][g] = live ? d * a.scale : -INFINITY;  // mha_kernel.cpp:51-60 (sum * scale)
            }
        }
        float p[NIT][G];
#pragma unroll
        for (int g = 0; g < G; ++g) {  // online softmax: this lane's row group over its rows so far
            float mn = m[g];
#pragma unroll
            for (int it = 0; it < NIT; ++it) mn = fmaxf(mn, s[it][g]);
            const float corr = m[g] == -INFINITY ? 0.0f : expf(m[g] - mn);
            l[g] *= corr;
#pragma unroll
            for (int e = 0; e < EPV; ++e) ov[g][e] *= corr;
            m[g] = mn;
#pragma unroll
            for (int it = 0; it < NIT; ++it) {
                p[it][g] = s[it][g] == -INFINITY ? 0.0f : expf(s[it][g] - mn);
                l[g] += p[it][g];
            }
        }
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
            const int row = wave * RPW + it * RPI + sub;
            const u32x4 vr = *reinterpret_cast<const u32x4*>(sv + row * ROWB + li * 16);
            float vf[EPV];
            Vec16<KT>::unpack(vr, vf);
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int e = 0; e < EPV; ++e) ov[g][e] = fmaf(p[it][g], vf[e], ov[g][e]);
        }
    }
    // the wave's row groups: max-rescaled sums across the lanes LPR, 2·LPR, … apart
#pragma unroll
    for (int o = LPR; o < 64; o <<= 1) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const float mo = __shfl_xor(m[g], o, kWave);
            const float lo = __shfl_xor(l[g], o, kWave);
            const float M = fmaxf(m[g], mo);
            const float c1 = m[g] == -INFINITY ? 0.0f : expf(m[g] - M);
            const float c2 = mo == -INFINITY ? 0.0f : expf(mo - M);
            l[g] = l[g] * c1 + lo * c2;
#pragma unroll
            for (int e = 0; e < EPV; ++e) {
                const float oo = __shfl_xor(ov[g][e], o, kWave);
                ov[g][e] = ov[g][e] * c1 + oo * c2;
            }
            m[g] = M;
        }
    }
    if (a.stamps && threadIdx.x == 0) a.stamps[blockIdx.x * 4 + 2] = __builtin_amdgcn_s_memrealtime();
    // the waves' states go through the ring's first slot once every wave is done with the last chunk
    static_assert(sizeof(float) * W * G * (HD + 2) <= sizeof(ring), "merge scratch");
    auto sh = reinterpret_cast<float(*)[G][HD + 2]>(&ring[0][0][0]);
    __syncthreads();
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
    for (int i = threadIdx.x; i < G * HD; i += 64 * W) {  // the workgroup's partial per q head
        const int g = i / HD, d = i - g * HD;
        float M = -INFINITY;
#pragma unroll
        for (int w = 0; w < W; ++w) M = fmaxf(M, sh[w][g][HD]);
        float o = 0.0f, L = 0.0f;
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const float mw = sh[w][g][HD];
            const float cw = mw == -INFINITY ? 0.0f : expf(mw - M);  // a wave past the context: nothing
            o = fmaf(cw, sh[w][g][d], o);
            L = fmaf(cw, sh[w][g][HD + 1], L);
        }
        float* dst = a.part + ((size_t)(kvh * G + g) * a.max_splits + wgs) * (HD + kAttnPartPad);
        dst[d] = o;
        if (d == 0) {
            dst[HD] = M;
            dst[HD + 1] = L;
        }
    }
    if (a.stamps && threadIdx.x == 0) a.stamps[blockIdx.x * 4 + 3] = __builtin_amdgcn_s_memrealtime();
}

}  // namespace sli
